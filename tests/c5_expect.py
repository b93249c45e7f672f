"""Expected colourings of the configs[4] stand-in (R-MAT scale 22, nCol = maxDeg, the wide sweep) for
EVERY vertex, computed on the host from the downloaded CSR.

A vertex that does not violate takes fill_p's case (iii) (coloringMCMC_CPU.cpp:471-479: own colour
1-(nCol-1)eps, others eps), so its update depends only on C_t[v] and u_v: the fp32 CDF before the own
colour is the eps prefix E[k] (k-fold sequential fp32 sum), at the own colour fl(E[cv] + hi), which
is >= 0.5, where adding eps (< half an ulp) leaves the sum unchanged -- so the walk gives the first
k < cv with E[k+1] > u, else cv when fl(E[cv] + hi) > u, else a CDF overflow. Vectorised over all
non-violators and pinned against the oracle's one-vertex update (oracle_vertex_update) in pin(). A
violator's update (cases (i)/(ii)) is the oracle's one-vertex update on its row's neighbour colours.
Overflow events take glibc rand() in ascending vertex order (:517-520).
"""
import numpy as np

import oracle_ref as O


def _tables(nCol: int, eps: float):
    e = np.float32(eps)
    E = np.zeros(nCol + 1, dtype=np.float32)
    E[1:] = np.cumsum(np.full(nCol, e, dtype=np.float32), dtype=np.float32)   # sequential fp32 sums
    hi = np.float32(1.0) - np.float32(nCol - 1) * e
    return E, hi


def walk_free(cv: np.ndarray, u: np.ndarray, nCol: int, eps: float) -> np.ndarray:
    """Case (iii) walk for non-violators: new colour, or nCol on a CDF overflow."""
    E, hi = _tables(nCol, eps)
    assert np.float32(E[nCol - 1] + hi) >= 0.5
    k = np.searchsorted(E[1:], u, side="right").astype(np.int64)   # first k with E[k+1] > u
    own = (E[cv] + hi).astype(np.float32)
    return np.where(k < cv, k, np.where(own > u, cv, nCol)).astype(np.uint32)


def pin(nCol: int, eps: float, k: int = 3000, seed: int = 7) -> None:
    rng = np.random.default_rng(seed)
    cv = rng.integers(0, nCol, k).astype(np.uint32)
    u = rng.random(k).astype(np.float32)
    E, _ = _tables(nCol, eps)
    u[: k // 4] = (E[cv[: k // 4]] * rng.random(k // 4)).astype(np.float32)   # below the own colour
    u[-8:] = np.float32(1 - 2**-24)
    w = walk_free(cv, u, nCol, eps)
    empty = np.zeros(0, dtype=np.uint32)
    for i in range(k):
        c, viol = O.vertex_update(nCol, eps, int(cv[i]), empty, float(u[i]))
        assert not viol
        assert (nCol if c is None else c) == int(w[i]), (i, int(cv[i]), float(u[i]))


def violators(off: np.ndarray, idx: np.ndarray, C: np.ndarray) -> np.ndarray:
    """violation_count's flags (coloringMCMC_CPU.cpp:329-351): own colour among the neighbours'."""
    n = len(off) - 1
    deg = np.diff(off.astype(np.int64))
    row = np.repeat(np.arange(n, dtype=np.int32), deg)
    eq = C[idx] == C[row]
    return np.bincount(row[eq], minlength=n) > 0


def expected(off, idx, nCol: int, sweeps: int, eps: float = 1e-8, seed: int = 1):
    """The reference loop for at most `sweeps` sweeps (run(), coloringMCMC_CPU.cpp:136: it stops once
    Cviol_t == 0): C_0 .. C_last, the trajectory (Cviol of every colouring swept, plus the final 0 when
    it converged), the overflow events per sweep, the engine start K0."""
    n = len(off) - 1
    c0 = np.zeros(n, dtype=np.uint32)
    k0 = int(O.lib().oracle_uniform_int_seq(seed, nCol, n, O._p(c0)))
    C, traj, events = [c0], [], []
    O.srand(1)
    vid = np.arange(n, dtype=np.uint64)
    for t in range(sweeps):
        cur = C[-1]
        u = O.canonical_at(seed, np.uint64(k0) + np.uint64(t) * np.uint64(n) + vid + np.uint64(1))
        vl = violators(off, idx, cur)
        traj.append(int(vl.sum()))
        if traj[-1] == 0:   # while (Cviol > z), z = 0: converged, no further sweep
            break
        nxt = walk_free(cur, u, nCol, eps)
        for v in np.nonzero(vl)[0].tolist():
            c, viol = O.vertex_update(nCol, eps, int(cur[v]), cur[idx[off[v]:off[v + 1]]], float(u[v]))
            assert viol
            nxt[v] = nCol if c is None else c
        ov = np.nonzero(nxt == nCol)[0]
        if len(ov):
            d = np.array(O.rand(len(ov)), dtype=np.uint64)
            nxt[ov] = (d % np.uint64(nCol - 1)).astype(np.uint32)
        events.append(len(ov))
        C.append(nxt)
    else:
        traj.append(int(violators(off, idx, C[-1]).sum()))   # the count that ends the capped loop
    return C, traj, events, k0
