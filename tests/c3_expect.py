"""Expected colourings of the C3 graph (configs[2]/[3]) for every vertex, without the graph.

At C3 (mean degree 1e4, 32 colours) every row's neighbourhood holds all 32 colours (a row misses a
colour with probability ~32 (31/32)^9600 ~ 1e-131), so count_free_colors gives Zvcomp = 0 and every
vertex is a violator: fill_p takes case (i) (coloringMCMC_CPU.cpp:402-412: own colour 1-(nCol-1)eps,
others eps) and the update depends only on C_t[v] and u_v. This module restates that case in
vectorised float32 (the CDF walk of extract_new_color, :493-528, strict >, no FMA) for all n
vertices, CDF overflows taking the glibc rand() stream in ascending vertex order (:517-520). The walk
is pinned against the oracle's one-vertex update (oracle_vertex_update) on sampled (C_t[v], u_v) in
pin_walk(). A row that was not full would make the device differ from this expectation (case (ii)):
the comparison cannot pass silently on a wrong assumption.
"""
import numpy as np

import oracle_ref as O

N, P, SEED, NCOL = 10_000_000, 0.001, 1, 32


def walk(cv: np.ndarray, u: np.ndarray, nCol: int, eps: float) -> np.ndarray:
    """Case (i) CDF walk for every vertex: new colour, or nCol where the walk overflows."""
    e = np.float32(eps)
    hi = np.float32(1.0) - np.float32(nCol - 1) * e
    cdf = np.zeros(len(cv), dtype=np.float32)
    out = np.full(len(cv), nCol, dtype=np.uint32)
    for c in range(nCol):
        cdf = cdf + np.where(cv == c, hi, e).astype(np.float32)
        hit = (out == nCol) & (cdf > u)
        out[hit] = c
    return out


def pin_walk(nCol: int, eps: float, k: int = 4000, seed: int = 5) -> None:
    """walk() == the oracle's one-vertex update with every colour among the neighbours."""
    rng = np.random.default_rng(seed)
    cv = rng.integers(0, nCol, k).astype(np.uint32)
    u = rng.random(k).astype(np.float32)
    u[:8] = np.float32(1 - 2**-24)   # the largest canonical value: overflow-prone
    w = walk(cv, u, nCol, eps)
    nbr = np.arange(nCol, dtype=np.uint32)
    for i in range(k):
        c, viol = O.vertex_update(nCol, eps, int(cv[i]), nbr, float(u[i]))
        assert viol
        assert (nCol if c is None else c) == int(w[i]), (i, int(cv[i]), float(u[i]))


def expected(sweeps: int, eps: float, nCol: int = NCOL, n: int = N, seed: int = SEED):
    """C_0 .. C_sweeps of the reference loop on a C3-like all-full graph, glibc unseeded (srand(1)):
    colourings, engine start K0, overflow events per sweep."""
    c0 = np.zeros(n, dtype=np.uint32)
    k0 = int(O.lib().oracle_uniform_int_seq(seed, nCol, n, O._p(c0)))
    C = [c0]
    events = []
    O.srand(1)
    vid = np.arange(n, dtype=np.uint64)
    for t in range(sweeps):
        u = O.canonical_at(seed, np.uint64(k0) + np.uint64(t) * np.uint64(n) + vid + np.uint64(1))
        nxt = walk(C[-1], u, nCol, eps)
        ov = np.nonzero(nxt == nCol)[0]
        if len(ov):
            d = np.array(O.rand(len(ov)), dtype=np.uint64)
            nxt[ov] = (d % np.uint64(nCol - 1)).astype(np.uint32)
        events.append(len(ov))
        C.append(nxt)
    return C, k0, events


M31 = np.uint64(2147483647)
A_MINSTD = 16807


def _mulmod(x: np.ndarray, y) -> np.ndarray:
    """x * y mod (2^31 - 1) for uint64 arrays of values < 2^31 (the product fits 62 bits)."""
    p = x * np.uint64(y) if np.isscalar(y) else x * y
    r = (p & M31) + (p >> np.uint64(31))
    r = (r & M31) + (r >> np.uint64(31))
    return np.where(r >= M31, r - M31, r)


def minstd_powers(n: int) -> np.ndarray:
    """16807^j mod (2^31 - 1) for j = 1..n (uint64), blockwise (4096 sequential, then one
    vectorised multiplication per block)."""
    B = 4096
    head = np.empty(B, dtype=np.uint64)
    x = 1
    for j in range(B):
        x = x * A_MINSTD % 2147483647
        head[j] = x
    out = np.empty(((n + B - 1) // B) * B, dtype=np.uint64)
    step = pow(A_MINSTD, B, 2147483647)
    s = 1
    for b in range(len(out) // B):
        out[b * B:(b + 1) * B] = _mulmod(head, s)
        s = s * step % 2147483647
    return out[:n]


def canonical(x: np.ndarray) -> np.ndarray:
    """generate_canonical<float,24> of minstd states: float(x - 1) / 2^31, clamped below 1."""
    u = (x - np.uint64(1)).astype(np.float32) * np.float32(2.0 ** -31)
    return np.where(u >= np.float32(1.0), np.float32(np.nextafter(np.float32(1), np.float32(0))), u).astype(np.float32)


def expected_final(sweeps: int, eps: float, nCol: int = NCOL, n: int = N, seed: int = SEED,
                   check_every: int = 50):
    """C_sweeps of the reference loop on an all-full graph, streamed (no colouring kept but the
    last), and the glibc draws it took (overflow events). Per sweep the draws u_v (engine position
    K0 + t n + v + 1) come from minstd powers; a vertex whose u lies in [E[nCol-1], S[0]) keeps
    its colour whatever the colour (the CDF before its colour, a sum of eps, is at most E[nCol-1]
    <= u, and its own step reaches S[cv] >= S[0] > u; E, S the literal fp32 partial sums); every
    other vertex takes the literal walk(). The draws of a sweep are the oracle's sequential minstd
    (canonical_from); every check_every sweeps 2000 sampled ones are checked against its per-position
    skip-ahead (canonical_at). Returns (C_sweeps, k0, events per sweep)."""
    c0 = np.zeros(n, dtype=np.uint32)
    k0 = int(O.lib().oracle_uniform_int_seq(seed, nCol, n, O._p(c0)))
    e = np.float32(eps)
    hi = np.float32(1.0) - np.float32(nCol - 1) * e
    E = [np.float32(0.0)]
    for _ in range(nCol - 1):
        E.append(np.float32(E[-1] + e))
    e_max, s_min = E[-1], np.float32(E[0] + hi)
    rng = np.random.default_rng(7)
    C = c0
    events = []
    O.srand(1)
    for t in range(sweeps):
        u = O.canonical_from(seed, k0 + t * n + 1, n)   # the sweep's bulk draw, in vertex order (:139)
        if t % check_every == 0:
            vs = rng.integers(0, n, 2000).astype(np.uint64)
            ref = O.canonical_at(seed, np.uint64(k0) + np.uint64(t) * np.uint64(n) + vs + np.uint64(1))
            assert np.array_equal(u[vs.astype(np.int64)], ref), f"draws of sweep {t}"
        idx = np.nonzero((u < e_max) | (u >= s_min))[0]
        nxt = C.copy()
        if len(idx):
            w = walk(C[idx], u[idx], nCol, eps)
            ov = idx[w == nCol]
            nxt[idx] = w
            if len(ov):
                d = np.array(O.rand(len(ov)), dtype=np.uint64)
                nxt[ov] = (d % np.uint64(nCol - 1)).astype(np.uint32)
            events.append(len(ov))
        else:
            events.append(0)
        C = nxt
    return C, k0, events
