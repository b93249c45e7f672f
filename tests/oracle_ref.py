"""ctypes wrapper of oracle/build/libmcmc_oracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; never by
the product. Builds the oracle with make if it is missing and the sources are present.
"""
from __future__ import annotations

import ctypes
import subprocess
from ctypes import POINTER, byref, c_double, c_float, c_int, c_int32, c_uint32, c_uint64, c_void_p
from dataclasses import dataclass
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "build" / "libmcmc_oracle.so"


class OracleParams(ctypes.Structure):
    _fields_ = [("nCol", c_uint32), ("epsilon", c_float), ("lambda_", c_float), ("ratioFreezed", c_float),
                ("numColorRatio", c_float), ("maxRip", c_uint32), ("tabooIteration", c_uint32),
                ("tailcut", c_int32), ("tailcutRepair", c_int32)]


class OracleResult(ctypes.Structure):
    _fields_ = [("iter", c_uint32), ("maxIterReached", c_int32), ("finalViol", c_uint64), ("trajLen", c_uint64),
                ("glibcDraws", c_uint64), ("initDraws", c_uint64), ("loopSeconds", c_double),
                ("sweepsRun", c_uint32), ("tailcutPasses", c_uint32)]


class OracleGpuResult(ctypes.Structure):
    _fields_ = [("rip", c_uint32), ("maxIterReached", c_int32), ("sweeps", c_uint32), ("tailcutPasses", c_uint32),
                ("conflictCounter", c_uint64), ("finalConflicts", c_uint64), ("trajLen", c_uint64)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            subprocess.run(["make", "-C", str(ORACLE_DIR), "-j4"], check=True, capture_output=True)
        L = ctypes.CDLL(str(ORACLE_LIB))
        L.oracle_rand.restype = c_int32
        L.oracle_srand.argtypes = [c_uint32]
        L.oracle_rand_skip.argtypes = [c_uint64]
        L.oracle_set_glibc_window.argtypes = [c_void_p]
        L.oracle_minstd_seq.argtypes = [c_uint32, c_uint64, c_void_p]
        L.oracle_canonical_seq.argtypes = [c_uint32, c_uint64, c_uint64, c_void_p]
        L.oracle_uniform_int_seq.argtypes = [c_uint32, c_uint32, c_uint64, c_void_p]
        L.oracle_uniform_int_seq.restype = c_uint64
        L.oracle_setup_rnd2.argtypes = [c_uint32, c_float, POINTER(POINTER(c_uint64)), POINTER(POINTER(c_uint32)),
                                        POINTER(c_uint64)]
        L.oracle_max_deg.argtypes = [c_uint32, c_void_p]
        L.oracle_er_fast.argtypes = [c_uint32, ctypes.c_double, c_uint64, POINTER(POINTER(c_uint64)),
                                     POINTER(POINTER(c_uint32)), POINTER(c_uint64)]
        L.oracle_max_deg.restype = c_uint32
        L.oracle_er_rows.argtypes = [c_uint32, ctypes.c_double, c_uint64, c_void_p, c_uint32, c_int,
                                     POINTER(POINTER(c_uint64)), POINTER(POINTER(c_uint32))]
        L.oracle_canonical_at.argtypes = [c_uint32, c_void_p, c_uint64, c_void_p]
        L.oracle_canonical_from.argtypes = [c_uint32, c_uint64, c_uint64, c_void_p]
        L.oracle_vertex_update.argtypes = [c_uint32, c_float, c_uint32, c_void_p, c_uint64, c_float,
                                           POINTER(c_uint32), POINTER(c_int)]
        L.oracle_free.argtypes = [c_void_p]
        L.oracle_mcmc_run.argtypes = [c_uint32, c_void_p, c_void_p, POINTER(OracleParams), c_uint32, c_void_p,
                                      c_void_p, c_void_p, c_uint64, c_uint32, c_int, POINTER(OracleResult)]
        L.oracle_xorwow_init.argtypes = [c_uint64, c_uint64, c_int, c_void_p]
        L.oracle_xorwow_next.argtypes = [c_void_p, c_uint32, c_void_p]
        L.oracle_gpurand_init.argtypes = [c_uint32, c_uint32, c_void_p]
        L.oracle_mcmc_gpu_run.argtypes = [c_uint32, c_void_p, c_void_p, POINTER(OracleParams), c_void_p, c_void_p,
                                          c_void_p, c_uint64, c_uint32, c_void_p, POINTER(OracleGpuResult)]
        _lib = L
    return _lib


def _p(a: np.ndarray) -> c_void_p:
    return a.ctypes.data_as(c_void_p)


def srand(seed: int) -> None:
    lib().oracle_srand(seed & 0xFFFFFFFF)


def rand(count: int) -> list[int]:
    return [lib().oracle_rand() for _ in range(count)]


def set_glibc_window(window: np.ndarray) -> None:
    w = np.ascontiguousarray(window, dtype=np.uint32)
    lib().oracle_set_glibc_window(_p(w))


def setup_rnd2(n: int, prob: float) -> tuple[np.ndarray, np.ndarray]:
    """Graph(n, prob, seed) -> setupRnd2 from the current glibc stream position."""
    off = POINTER(c_uint64)()
    idx = POINTER(c_uint32)()
    m = c_uint64()
    rc = lib().oracle_setup_rnd2(n, c_float(prob), byref(off), byref(idx), byref(m))
    assert rc == 0
    a = np.ctypeslib.as_array(off, (n + 1,)).copy()
    b = np.ctypeslib.as_array(idx, (max(m.value, 1),))[: m.value].copy()
    lib().oracle_free(ctypes.cast(off, c_void_p))
    lib().oracle_free(ctypes.cast(idx, c_void_p))
    return a, b


def er_fast(n: int, prob: float, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """The build's counter-based G(n, p) (csrc/er_gen.h), restated on the CPU; rows ascending."""
    off = POINTER(c_uint64)()
    idx = POINTER(c_uint32)()
    m = c_uint64()
    rc = lib().oracle_er_fast(n, prob, seed, byref(off), byref(idx), byref(m))
    assert rc == 0
    a = np.ctypeslib.as_array(off, (n + 1,)).copy()
    b = np.ctypeslib.as_array(idx, (max(m.value, 1),))[: m.value].copy()
    lib().oracle_free(ctypes.cast(off, c_void_p))
    lib().oracle_free(ctypes.cast(idx, c_void_p))
    return a, b


def er_rows(n: int, prob: float, seed: int, rows, nthreads: int = 0) -> list[np.ndarray]:
    """Neighbour lists (ascending) of the given rows of er_fast(n, prob, seed), found without
    enumerating the graph (streams into the rows' column blocks only)."""
    import os

    r = np.ascontiguousarray(rows, dtype=np.uint32)
    off = POINTER(c_uint64)()
    idx = POINTER(c_uint32)()
    th = nthreads or int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    rc = lib().oracle_er_rows(n, prob, seed, _p(r), len(r), th, byref(off), byref(idx))
    assert rc == 0
    o = np.ctypeslib.as_array(off, (len(r) + 1,)).copy()
    m = int(o[-1])
    b = np.ctypeslib.as_array(idx, (max(m, 1),))[:m].copy()
    lib().oracle_free(ctypes.cast(off, c_void_p))
    lib().oracle_free(ctypes.cast(idx, c_void_p))
    return [b[o[i]:o[i + 1]] for i in range(len(r))]


def canonical_at(seed: int, positions) -> np.ndarray:
    """u of engine draws `positions` (1-based) of default_random_engine(seed)."""
    pos = np.ascontiguousarray(positions, dtype=np.uint64)
    out = np.zeros(len(pos), dtype=np.float32)
    lib().oracle_canonical_at(seed & 0xFFFFFFFF, _p(pos), len(pos), _p(out))
    return out


def canonical_from(seed: int, start: int, count: int) -> np.ndarray:
    """u of engine draws start, start + 1, ..., start + count - 1 (1-based) of default_random_engine(seed)."""
    out = np.zeros(count, dtype=np.float32)
    lib().oracle_canonical_from(seed & 0xFFFFFFFF, start, count, _p(out))
    return out


def vertex_update(nCol: int, eps: float, cv: int, nbr_colors: np.ndarray, u: float):
    """(new colour or None on a CDF overflow, viol) of one vertex (coloringMCMC_CPU.cpp:183-204)."""
    nc = np.ascontiguousarray(nbr_colors, dtype=np.uint32)
    col, viol = c_uint32(), c_int()
    ov = lib().oracle_vertex_update(nCol, eps, cv, _p(nc) if len(nc) else None, len(nc), u, byref(col), byref(viol))
    return (None if ov else col.value), bool(viol.value)


def max_deg(row_off: np.ndarray) -> int:
    return int(np.max(np.diff(row_off.astype(np.int64)))) if len(row_off) > 1 else 0


@dataclass
class OracleRun:
    colors: np.ndarray
    init: np.ndarray
    traj: np.ndarray
    res: OracleResult


def mcmc_run(row_off: np.ndarray, col_idx: np.ndarray, nCol: int, seed: int, *, epsilon: float = 1e-8,
             maxRip: int = 250, tabooIteration: int = 0, tailcut: bool = False, tailcutRepair: bool = False,
             sweep_limit: int = 0, nthreads: int = 1) -> OracleRun:
    """ColoringMCMC_CPU(g, params, seed).run() from the current glibc stream position."""
    row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
    col_idx = np.ascontiguousarray(col_idx, dtype=np.uint32)
    n = len(row_off) - 1
    prm = OracleParams(nCol, epsilon, 1.0, 0.01, 1.0, maxRip, tabooIteration, int(tailcut), int(tailcutRepair))
    colors = np.zeros(n, dtype=np.uint32)
    init = np.zeros(n, dtype=np.uint32)
    traj = np.zeros(maxRip + 2, dtype=np.uint64)
    res = OracleResult()
    rc = lib().oracle_mcmc_run(n, _p(row_off), _p(col_idx) if len(col_idx) else None, byref(prm), seed & 0xFFFFFFFF,
                               _p(init), _p(colors), _p(traj), len(traj), sweep_limit, nthreads, byref(res))
    assert rc == 0
    return OracleRun(colors, init, traj[: res.trajLen].copy(), res)


# ---- reference-GPU-semantics mode (oracle/mcmc_gpu_ref.cpp) ----------------------------------
def xorwow_init(seed: int, subsequence: int, flavor: int = 0) -> np.ndarray:
    out = np.zeros(6, dtype=np.uint32)
    lib().oracle_xorwow_init(seed, subsequence, flavor, _p(out))
    return out


def xorwow_next(state: np.ndarray, count: int) -> np.ndarray:
    """Advances `state` (6 words, in place) and returns `count` outputs."""
    out = np.zeros(count, dtype=np.uint32)
    lib().oracle_xorwow_next(_p(state), count, _p(out))
    return out


def gpurand_init(n: int, seed: int) -> np.ndarray:
    """GPURand(n, seed) -> [n][6] states."""
    st = np.zeros((n, 6), dtype=np.uint32)
    lib().oracle_gpurand_init(n, seed & 0xFFFFFFFF, _p(st))
    return st


@dataclass
class OracleGpuRun:
    colors: np.ndarray
    traj: np.ndarray
    tail_traj: np.ndarray
    res: OracleGpuResult


def mcmc_gpu_run(row_off: np.ndarray, col_idx: np.ndarray, nCol: int, states: np.ndarray, *,
                 epsilon: float = 1e-8, maxRip: int = 250, tabooIteration: int = 0, tailcut: bool = False,
                 tail_max_passes: int = 1000) -> OracleGpuRun:
    """ColoringMCMC (GPU, default build) run() from per-vertex XORWOW `states` ([n][6], advanced in place)."""
    row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
    col_idx = np.ascontiguousarray(col_idx, dtype=np.uint32)
    n = len(row_off) - 1
    assert states.shape == (n, 6) and states.dtype == np.uint32 and states.flags.c_contiguous
    prm = OracleParams(nCol, epsilon, 1.0, 0.01, 1.0, maxRip, tabooIteration, int(tailcut), 0)
    colors = np.zeros(n, dtype=np.uint32)
    traj = np.zeros(maxRip + 2, dtype=np.uint64)
    tail = np.zeros(max(tail_max_passes, 1), dtype=np.uint64)
    res = OracleGpuResult()
    rc = lib().oracle_mcmc_gpu_run(n, _p(row_off), _p(col_idx) if len(col_idx) else None, byref(prm), _p(states),
                                   _p(colors), _p(traj), len(traj), tail_max_passes, _p(tail), byref(res))
    assert rc == 0
    return OracleGpuRun(colors, traj[: res.trajLen].copy(), tail[: res.tailcutPasses].copy(), res)
