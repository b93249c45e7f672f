"""ctypes binding of libmcmc_hip.so (include/mcmc_hip.h).

The product path has no fallback: if the HIP library is missing or fails to load, importing
the colorer raises. Build it with ``python -m mcmc_colorer_amd.build`` (or ``__graft_entry__.build``).
"""
from __future__ import annotations

import ctypes
import os
import sys
from ctypes import POINTER, byref, c_char_p, c_double, c_float, c_int, c_int32, c_uint32, c_uint64, c_void_p
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("MCMC_HIP_LIB", Path(__file__).resolve().parent / "libmcmc_hip.so"))

# Every symbol declared in include/mcmc_hip.h, with (restype, argtypes).
_u32p = POINTER(c_uint32)
_u64p = POINTER(c_uint64)
SIGNATURES: dict[str, tuple] = {
    "mcmc_last_error": (c_char_p, []),
    "mcmc_version": (c_int, []),
    "mcmc_glibc_window": (c_int, [c_uint32, c_uint64, _u32p]),
    "mcmc_glibc_draw": (c_int, [_u32p, c_uint32, _u32p]),
    "mcmc_graph_upload": (c_int, [_u64p, _u32p, c_uint32, c_uint64, c_int, POINTER(c_void_p)]),
    "mcmc_graph_simulate": (c_int, [c_uint32, c_float, _u32p, c_int, POINTER(c_void_p)]),
    "mcmc_graph_er_fast": (c_int, [c_uint32, c_double, c_uint64, c_int, POINTER(c_void_p)]),
    "mcmc_graph_er_fast_part": (c_int, [c_uint32, c_double, c_uint64, c_uint32, c_uint32, c_int, POINTER(c_void_p)]),
    "mcmc_graph_er_fast_rows": (c_int, [c_uint32, c_double, c_uint64, c_uint32, c_uint32, c_int, POINTER(c_void_p)]),
    "mcmc_graph_rmat": (c_int, [c_uint32, c_uint32, c_double, c_double, c_double, c_uint64, c_int, POINTER(c_void_p)]),
    "mcmc_graph_info": (c_int, [c_void_p, _u32p, _u64p, _u32p, _u32p]),
    "mcmc_color_bytes": (c_uint32, [c_uint32]),
    "mcmc_greedyff_run": (c_int, [c_void_p, _u32p, _u32p, _u32p]),
    "mcmc_luby_run": (c_int, [c_void_p, c_void_p, _u32p, _u32p, _u32p]),
    "mcmc_vff_run": (c_int, [c_void_p, _u32p, _u32p, _u32p, POINTER(c_int)]),
    "mcmc_graph_device_ptrs": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_void_p)]),
    "mcmc_graph_download": (c_int, [c_void_p, _u64p, _u32p]),
    "mcmc_graph_materialize_csr": (c_int, [c_void_p]),
    "mcmc_graph_rows": (c_int, [c_void_p, _u32p, c_uint32, _u64p, _u32p, c_uint64, _u64p]),
    "mcmc_graph_destroy": (None, [c_void_p]),
    "mcmc_create": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, POINTER(c_void_p)]),
    "mcmc_set_glibc_window": (c_int, [c_void_p, _u32p]),
    "mcmc_get_glibc_window": (c_int, [c_void_p, _u32p]),
    "mcmc_init_coloring": (c_int, [c_void_p, _u32p]),
    "mcmc_run": (c_int, [c_void_p, c_uint32, c_void_p]),
    "mcmc_get_coloring": (c_int, [c_void_p, _u32p]),
    "mcmc_count_violations": (c_int, [c_void_p, _u64p, c_void_p]),
    "mcmc_set_tailcut_repair": (c_int, [c_void_p, c_uint32]),
    "mcmc_get_trajectory": (c_int, [c_void_p, _u64p, c_uint64, _u64p]),
    "mcmc_bench_sweeps": (c_int, [c_void_p, c_uint32, POINTER(c_double), POINTER(c_double)]),
    "mcmc_bench_prepare": (c_int, [c_void_p, c_uint32]),
    "mcmc_set_bench_mode": (c_int, [c_void_p, c_int]),
    "mcmc_set_scan_stats": (c_int, [c_void_p, c_int]),
    "mcmc_get_scan_stats": (c_int, [c_void_p, _u64p, _u64p]),
    "mcmc_get_scan_stats_ex": (c_int, [c_void_p, _u64p, _u64p, _u64p]),
    "mcmc_get_scan_stats_v2": (c_int, [c_void_p, _u64p]),
    "mcmc_get_wide_inc_stats": (c_int, [c_void_p, _u64p]),
    "mcmc_get_wide_solo_stats": (c_int, [c_void_p, _u64p]),
    "mcmc_get_dense_stats": (c_int, [c_void_p, _u64p]),
    "mcmc_get_dense_stats_v2": (c_int, [c_void_p, _u64p]),
    "mcmc_get_dense_counts": (c_int, [c_void_p, c_uint32, c_uint32, _u32p, _u32p]),
    "mcmc_get_info": (c_int, [c_void_p, c_void_p]),
    "mcmc_cdf_walk": (c_uint32, [_u32p, c_uint32, c_uint32, c_float, c_float, c_float]),
    "mcmc_refstruct_bench": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32, POINTER(c_double), _u64p]),
    "mcmc_destroy": (None, [c_void_p]),
    "mcmc_part_plan_rows": (c_int, [c_uint32, c_uint32, _u32p]),
    "mcmc_part_plan": (c_int, [c_void_p, c_uint32, c_int, _u32p]),
    "mcmc_part_plan_csr": (c_int, [_u64p, c_uint32, c_uint32, _u32p]),
    "mcmc_part_attach": (c_int, [c_void_p, c_uint32, c_uint32, _u32p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
                                 c_void_p]),
    "mcmc_part_sweep_async": (c_int, [c_void_p]),
    "mcmc_part_commit_async": (c_int, [c_void_p]),
    "mcmc_part_state": (c_int, [c_void_p, POINTER(c_int32), _u32p, _u32p]),
    "mcmc_part_spill_counts": (c_int, [c_void_p, _u32p]),
    "mcmc_part_spill_local": (c_int, [c_void_p, c_void_p, _u32p]),
    "mcmc_part_spill_commit_async": (c_int, [c_void_p, c_void_p, c_uint32]),
    "mcmc_part_attach_delta": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mcmc_part_delta_ok": (c_int, [c_void_p]),
    "mcmc_part_sweep_mode_async": (c_int, [c_void_p, c_int]),
    "mcmc_part_commit_mode_async": (c_int, [c_void_p, c_int, c_void_p, c_uint32]),
    "mcmc_part_sync_remote_async": (c_int, [c_void_p]),
    "mcmc_part_exchange_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                         POINTER(c_uint64)]),
    "mcmc_comm_unique_id": (c_int, [c_void_p]),
    "mcmc_comm_init_rank": (c_int, [c_void_p, c_uint32, c_uint32, c_int, POINTER(c_void_p)]),
    "mcmc_comm_init_all": (c_int, [POINTER(c_int), c_uint32, POINTER(c_void_p)]),
    "mcmc_comm_destroy": (None, [c_void_p]),
    "mcmc_part_create": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, _u32p, c_void_p, POINTER(c_void_p)]),
    "mcmc_part_run": (c_int, [POINTER(c_void_p), c_uint32, c_uint32, c_void_p]),
    "mcmc_part_bench_rank": (c_int, [c_void_p, c_uint32, c_void_p]),
    "mcmc_xorwow_state": (c_int, [c_uint64, c_uint64, c_int, _u32p]),
    "mcmc_gpurand_create": (c_int, [c_uint32, c_uint32, c_int, POINTER(c_void_p)]),
    "mcmc_gpurand_states": (c_int, [c_void_p, _u32p]),
    "mcmc_gpurand_destroy": (None, [c_void_p]),
    "mcmc_ref_create": (c_int, [c_void_p, c_void_p, c_void_p, POINTER(c_void_p)]),
    "mcmc_ref_run": (c_int, [c_void_p, c_uint32, c_void_p]),
    "mcmc_ref_init": (c_int, [c_void_p]),
    "mcmc_get_tail_trajectory": (c_int, [c_void_p, _u64p, c_uint64, _u64p]),
    "mcmc_device_mem_info": (c_int, [c_int, _u64p, _u64p]),
    "mcmc_hip_versions": (c_int, [POINTER(c_int), POINTER(c_int)]),
}


class MCMCParams(ctypes.Structure):
    """mcmc_params == ColoringMCMCParams (graph_coloring/coloring.h:65-74) + seed."""

    _fields_ = [
        ("nCol", c_uint32),
        ("epsilon", c_float),
        ("lambda_", c_float),
        ("ratioFreezed", c_float),
        ("numColorRatio", c_float),
        ("maxRip", c_uint32),
        ("tabooIteration", c_uint32),
        ("tailcut", c_int32),
        ("seed", c_uint32),
    ]


class MCMCRunStats(ctypes.Structure):
    _fields_ = [
        ("iter", c_uint32),
        ("maxIterReached", c_int32),
        ("finalViol", c_uint64),
        ("trajLen", c_uint64),
        ("glibcDraws", c_uint64),
        ("initDraws", c_uint64),
        ("loopMs", c_double),
        ("sweepsRun", c_uint32),
        ("tailcutPasses", c_uint32),
    ]


class MCMCCtxInfo(ctypes.Structure):
    _fields_ = [
        ("variant", c_int32),
        ("resident", c_int32),
        ("block_log2", c_uint32),
        ("nblocks", c_uint32),
        ("grp_rows", c_uint32),
        ("ngroups", c_uint32),
        ("sub_log2", c_uint32),
        ("grid", c_uint32),
        ("block", c_uint32),
        ("reserved", c_uint32),
        ("lds_bytes", c_uint64),
        ("layout_bytes", c_uint64),
        ("sweep_bytes", c_uint64),
        ("ref_bytes", c_uint64),
    ]

    VARIANTS = {0: "lds", 1: "blocked", 2: "global", 3: "tiled", 4: "wide", 5: "ref-wide", 6: "wide-tiled"}

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}
        d["variant"] = self.VARIANTS.get(self.variant, str(self.variant))
        d["resident"] = bool(self.resident)
        return d


class MCMCError(RuntimeError):
    pass


_lib = None


def _hip_runtimes() -> set:
    """Paths of the HIP runtimes (libamdhip64) mapped into this process."""
    try:
        with open("/proc/self/maps") as f:
            return {ln.split()[-1] for ln in f if "libamdhip64" in ln and ln.split()[-1].startswith("/")}
    except OSError:
        return set()


def _process_hip_runtime():
    """The HIP runtime this process has or will have: one already mapped (torch imported first), else
    the one torch bundles when torch is installed (it carries its own libamdhip64.so with the soname
    libamdhip64.so.7 and its own HSA runtime), else None (the library's /opt/rocm runtime)."""
    mapped = _hip_runtimes()
    if mapped:
        return sorted(mapped)[0]
    import importlib.util

    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is not None and spec.origin:
        cand = Path(spec.origin).parent / "lib" / "libamdhip64.so"
        if cand.exists():
            return str(cand)
    return None


def lib() -> ctypes.CDLL:
    """Loads libmcmc_hip.so once. Raises (never falls back) when it is missing.

    One HIP runtime per process: the library needs libamdhip64.so.7 and librccl.so.1, which torch's
    bundled ROCm also provides under those sonames. Loaded first, the library would bring /opt/rocm's
    runtime and a later `import torch` its own -- two HSA runtimes, and one of them finds no GPU. So
    the runtime the process uses (torch's when torch is installed) and its RCCL are loaded before
    the library, which then binds to them by soname; torch, imported later, finds them mapped.

    They are loaded RTLD_LOCAL: binding by soname does not need the global scope. r05 loaded them
    RTLD_GLOBAL, and a process that loaded the library before torch aborted at exit with "double
    free or corruption" -- a stack scan of the abort (scripts/rt_exit_probe.py, gpurun_out/r06c)
    put it in librocm_smi64's destructor of a static std::map, the RCCL dependency that the global
    preload exposed to every later load; with RTLD_LOCAL every import order exits cleanly
    (gpurun_out/r06d, tests/test_runtime.py). Two runtimes mapped anyway is an error. The runtime's
    version is not queried here (hipRuntimeGetVersion initialises the runtime); mcmc_hip_versions
    reports it beside the version the library was built for (tests/test_runtime.py: same major)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise MCMCError(f"{LIB_PATH} not found: build it with `python -m mcmc_colorer_amd.build`")
        rt = _process_hip_runtime()
        if rt is not None and os.environ.get("MCMC_OWN_HIP_RUNTIME") != "1":
            ctypes.CDLL(rt, mode=ctypes.RTLD_LOCAL)
            rccl = Path(rt).parent / "librccl.so"   # (soname librccl.so.1: the library's RCCL too)
            if rccl.exists():
                ctypes.CDLL(str(rccl), mode=ctypes.RTLD_LOCAL)
        L = ctypes.CDLL(str(LIB_PATH))
        both = _hip_runtimes()
        if len(both) > 1:
            raise MCMCError(f"two HIP runtimes in one process ({', '.join(sorted(both))}): load "
                            f"libmcmc_hip.so after the runtime the process uses (import torch first)")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().mcmc_last_error()
        raise MCMCError(f"libmcmc_hip error {rc}: {msg.decode() if msg else ''}")


def u32ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(_u32p)


def u64ptr(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(_u64p)


__all__ = ["lib", "check", "MCMCParams", "MCMCRunStats", "MCMCError", "SIGNATURES", "u32ptr", "u64ptr", "byref"]
