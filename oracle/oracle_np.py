"""oracle/oracle_np.py -- TEST INFRASTRUCTURE ONLY.

An independent float32 restatement of the reference's ``--mcmccpu`` path, written without
libstdc++ or glibc: its own minstd_rand0, generate_canonical<float,24>, uniform_int_distribution
and glibc TYPE_3 rand(). It exists to cross-check ``oracle/mcmc_cpu_ref.cpp`` (which calls the
real libraries, exactly like the reference) on small graphs, so that the C++ oracle is pinned by
two restatements that share no code. Pure-Python loops: keep n small (<= a few hundred).

Reference lines restated (paths relative to /root/reference/src):
  graph/graphCPU.cpp:291-404            setupRnd2 (Erdos-Renyi via glibc rand())
  graph_coloring/coloringMCMC_CPU.cpp   ctor :53-61, run :115-270, violation_count :329-351,
                                        count_free_colors :362-383, fill_p :393-481,
                                        extract_new_color :493-528
  graph_coloring/coloringGreedyFF.cu    run :50-84 and its kernels (greedy_ff)
  graph_coloring/coloringLubyFast.cu    run_fast / fast_colorer_k and the Luby kernels (luby,
  graph_coloring/coloringLuby.cu        with xorwow_step / curand_uniform for GPURand's states)
  graph_coloring/coloringVFF.cu         run, run_balancing and its kernels (vff)
Also the build's own generators (er_fast: csrc/er_gen.h; rmat: the C5 stand-in), which have no
reference counterpart. The colorer restatements are vectorised numpy (n up to a few thousand).
"""
from __future__ import annotations

import numpy as np

M31 = 2147483647
A_MINSTD = 16807
F32 = np.float32


class Minstd:
    """std::minstd_rand0 (C++ [rand.predef]): x <- 16807 x mod (2^31 - 1)."""

    def __init__(self, seed: int):
        s = seed % M31
        self.x = 1 if s == 0 else s

    def __call__(self) -> int:
        self.x = (self.x * A_MINSTD) % M31
        return self.x


def canonical(x: int) -> np.float32:
    """generate_canonical<float,24> over minstd: float(x-1) / 2^31, clamped below 1."""
    r = F32(x - 1) / F32(2147483648.0)
    if r >= F32(1.0):
        r = np.nextafter(F32(1.0), F32(0.0))
    return F32(r)


def uniform_int(gen: Minstd, ncol: int) -> tuple[int, int]:
    """uniform_int_distribution<uint32_t>(0, ncol-1), libstdc++ 'fallback (2 divisions)' path.
    Returns (value, engine draws consumed)."""
    urngrange = 2147483645
    scaling = urngrange // ncol
    past = ncol * scaling
    draws = 0
    while True:
        r = gen() - 1
        draws += 1
        if r < past:
            return r // scaling, draws


class GlibcRand:
    """glibc random_r.c TYPE_3 (degree 31, separation 3): r[i] = r[i-3] + r[i-31] mod 2^32,
    output r >> 1, first 310 outputs discarded; srand(0) behaves as srand(1)."""

    def __init__(self, seed: int = 1):
        seed = seed & 0xFFFFFFFF
        if seed == 0:
            seed = 1
        r = [0] * 34
        r[0] = seed
        for i in range(1, 31):
            # Schrage's method on a signed 32-bit word with C (truncating) division, as glibc does
            w = r[i - 1] if r[i - 1] < 2**31 else r[i - 1] - 2**32
            hi = abs(w) // 127773 * (1 if w >= 0 else -1)
            lo = w - hi * 127773
            word = 16807 * lo - 2836 * hi
            if word < 0:
                word += 2147483647
            r[i] = word & 0xFFFFFFFF
        for i in range(31, 34):
            r[i] = r[i - 31]
        self.win = r[3:34]  # the last 31 values r[3..33]
        for _ in range(310):
            self._step()

    def _step(self) -> int:
        v = (self.win[-31] + self.win[-3]) & 0xFFFFFFFF
        self.win.append(v)
        del self.win[0]
        return v

    def __call__(self) -> int:
        return self._step() >> 1


def setup_rnd2(n: int, prob: float, rng: GlibcRand):
    """Graph::setupRnd2 -> CSR (row_off uint64[n+1], col_idx uint32[m]), neighbours ascending."""
    p = float(np.float32(prob))
    adj = [[] for _ in range(n)]
    for j in range(n):
        for i in range(j, n):
            bit = (rng() / 2147483647.0) < p
            if bit and i != j:
                adj[j].append(i)
                adj[i].append(j)
    for lst in adj:
        lst.sort()
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(a) for a in adj])
    idx = np.array([w for a in adj for w in a], dtype=np.uint32)
    return off, idx


def mcmc_run(off, idx, ncol: int, seed: int, glibc: GlibcRand, max_rip: int = 250,
             taboo_iter: int = 0, z: int = 0, eps: np.float32 = F32(1e-8)):
    """ColoringMCMC_CPU ctor + run(); returns (colors, trajectory, iter, max_iter_reached, init)."""
    n = len(off) - 1
    gen = Minstd(seed)
    C = np.array([uniform_int(gen, ncol)[0] for _ in range(n)], dtype=np.int64)
    init = C.copy()
    taboo = np.zeros(n, dtype=np.int64)
    hi = F32(F32(1.0) - F32(ncol - 1) * eps)
    nbrs = [idx[off[v]:off[v + 1]].astype(np.int64) for v in range(n)]

    def viol_vec(col):
        return np.array([bool(np.any(col[nb] == col[v])) for v, nb in enumerate(nbrs)])

    traj = []
    it = 0
    max_reached = False
    cviol = int(viol_vec(C).sum())
    while cviol > z:
        u = [canonical(gen()) for _ in range(n)]
        viols = viol_vec(C)
        cviol = int(viols.sum())
        traj.append(cviol)
        Cs = C.copy()
        for v in range(n):
            occ = np.zeros(ncol, dtype=bool)
            occ[C[nbrs[v]]] = True
            zvcomp = ncol - int(occ.sum())
            zv = ncol - zvcomp
            if viols[v] and zvcomp > 0:
                pf = F32(F32(F32(1.0) - F32(eps * F32(zv))) / F32(zvcomp))
                p = [eps if occ[c] else pf for c in range(ncol)]
            else:
                p = [hi if c == C[v] else eps for c in range(ncol)]
            if taboo[v] > 0:
                taboo[v] -= 1
                Cs[v] = C[v]
                continue
            cdf = F32(0.0)
            new = ncol
            for c in range(ncol):
                cdf = F32(cdf + p[c])
                if cdf > u[v]:
                    new = c
                    break
            if new >= ncol:
                new = glibc() % (ncol - 1)
            Cs[v] = new
            taboo[v] = (1 if new == C[v] else 0) * taboo_iter
        cstar_viol = int(viol_vec(Cs).sum())
        C = Cs
        cviol = cstar_viol
        it += 1
        if it > max_rip:
            max_reached = True
            break
    traj.append(cviol)
    return C.astype(np.uint32), traj, it, max_reached, init.astype(np.uint32)


# ---- the build's counter-based G(n, p) (mcmc_colorer_amd/csrc/er_gen.h), vectorised over streams --
# TEST INFRASTRUCTURE: an independent restatement used to pin oracle_er_fast (C) on small graphs.
_ER_T = 65536
_ER_TAG = 0x45524721
_M32 = np.uint64(0xFFFFFFFF)


def _philox4x32_10(c0, c1, c2, c3, k0, k1):
    c = [np.asarray(x, dtype=np.uint64) & _M32 for x in (c0, c1, c2, c3)]
    k = [np.uint64(k0), np.uint64(k1)]
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k[0]) & _M32, p1 & _M32,
             ((p0 >> np.uint64(32)) ^ c[3] ^ k[1]) & _M32, p0 & _M32]
        k = [(k[0] + np.uint64(0x9E3779B9)) & _M32, (k[1] + np.uint64(0xBB67AE85)) & _M32]
    return c


def _series_log(u):
    bits = np.asarray(u, dtype=np.float64).view(np.uint64)
    e = ((bits >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64) - 1023
    m = ((bits & np.uint64(0x000FFFFFFFFFFFFF)) | np.uint64(0x3FF0000000000000)).view(np.float64)
    big = m > 1.4142135623730951
    m = np.where(big, m * 0.5, m)
    e = e + big
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    poly = np.full_like(s, 1.0 / 25.0)
    for k in range(11, -1, -1):
        poly = poly * s2 + 1.0 / float(2 * k + 1)
    ef = e.astype(np.float64)
    return (ef * 6.93147180369123816490e-01 + 2.0 * s * poly) + ef * 1.90821492927058770002e-10


def er_fast(n: int, prob: float, seed: int):
    """Edges (i < j) of the counter-based G(n, p), as an (E, 2) int64 array, streams walked in lock-step."""
    import math

    p = float(np.float32(prob))
    if p <= 0.0 or n < 2:
        return np.zeros((0, 2), dtype=np.int64)
    ii, yy = [], []
    nb = (n + _ER_T - 1) // _ER_T
    for Y in range(nb):
        rows = np.arange(0, min(n, (Y + 1) * _ER_T), dtype=np.int64)
        ii.append(rows)
        yy.append(np.full(len(rows), Y, dtype=np.int64))
    i = np.concatenate(ii)
    Y = np.concatenate(yy)
    end = np.minimum(n, (Y + 1) * _ER_T)
    j = np.maximum(Y * _ER_T, i + 1)
    keep = j < end
    i, Y, end, j = i[keep], Y[keep], end[keep], j[keep]
    if p >= 1.0:
        out = [np.stack([np.repeat(i, end - j), np.concatenate([np.arange(a, b) for a, b in zip(j, end)])], 1)]
        return np.concatenate(out) if len(i) else np.zeros((0, 2), dtype=np.int64)
    inv = 1.0 / math.log1p(-p)
    j = j - 1
    k = 0
    out = []
    active = np.ones(len(i), dtype=bool)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    while active.any():
        idx = np.nonzero(active)[0]
        r = _philox4x32_10(np.full(len(idx), k, dtype=np.uint64), i[idx].astype(np.uint64),
                           Y[idx].astype(np.uint64), np.full(len(idx), _ER_TAG, dtype=np.uint64), k0, k1)
        alive = np.ones(len(idx), dtype=bool)
        for q in range(4):
            x = r[q].astype(np.float64)
            t = _series_log((x + 1.0) * 2.3283064365386963e-10) * inv
            skip = np.where(t < 2147483647.0, 1 + np.floor(np.minimum(t, 2147483647.0)).astype(np.int64), 0x7FFFFFFF)
            jj = j[idx] + np.where(alive, skip, 0)
            j[idx] = jj
            hit = alive & (jj < end[idx])
            out.append(np.stack([i[idx][hit], jj[hit]], 1))
            alive &= hit
        active[idx[~alive]] = False
        k += 1
    return np.concatenate(out) if out else np.zeros((0, 2), dtype=np.int64)


# ---- R-MAT stand-in for configs[4] (mcmc_colorer_amd/csrc/er_gen.h rmat_edge), vectorised ----------
# TEST INFRASTRUCTURE: an independent restatement pinning mcmc_graph_rmat on small graphs.
_RMAT_TAG = 0x524D4154


def _rmat_threshold(x: float) -> int:
    import math

    return int(min(4294967295.0, math.floor(max(0.0, x) * 4294967296.0)))


def _rmat_scramble(x, scale: int, k0: int):
    M = np.uint64((1 << scale) - 1)
    h = np.uint64((scale + 1) // 2)
    x = np.asarray(x, dtype=np.uint64)
    x = (x * np.uint64(0x9E3779B1)) & _M32 & M
    x = x ^ (x >> h)
    x = (x * np.uint64(0x85EBCA6B)) & _M32 & M
    x = x ^ (x >> h)
    return (x ^ np.uint64((k0 * 0xC2B2AE35) & 0xFFFFFFFF)) & M


def rmat(scale: int, edge_factor: int, a: float, b: float, c: float, seed: int):
    """CSR (row_off uint64, col_idx uint32) of mcmc_graph_rmat(scale, edge_factor, a, b, c, seed)."""
    n = 1 << scale
    E = edge_factor * n
    tA, tAB, tABC = _rmat_threshold(a), _rmat_threshold(a + b), _rmat_threshold(a + b + c)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    e = np.arange(E, dtype=np.uint64)
    i = np.zeros(E, dtype=np.uint64)
    j = np.zeros(E, dtype=np.uint64)
    for l0 in range(0, scale, 4):
        r = _philox4x32_10(e & _M32, e >> np.uint64(32), np.full(E, l0 >> 2, dtype=np.uint64),
                           np.full(E, _RMAT_TAG, dtype=np.uint64), k0, k1)
        for q in range(4):
            if l0 + q >= scale:
                break
            x = r[q]
            ib = (x >= np.uint64(tAB)).astype(np.uint64)
            jb = (((x >= np.uint64(tA)) & (x < np.uint64(tAB))) | (x >= np.uint64(tABC))).astype(np.uint64)
            i = (i << np.uint64(1)) | ib
            j = (j << np.uint64(1)) | jb
    i = _rmat_scramble(i, scale, k0)
    j = _rmat_scramble(j, scale, k0)
    keep = i != j
    i, j = i[keep], j[keep]
    keys = np.unique(np.concatenate([(i << np.uint64(32)) | j, (j << np.uint64(32)) | i]))
    rows = (keys >> np.uint64(32)).astype(np.int64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.add.at(off, rows + 1, 1)
    return np.cumsum(off).astype(np.uint64), (keys & _M32).astype(np.uint32)


def greedy_ff(off, idx):
    """ColoringGreedyFF::run (graph_coloring/coloringGreedyFF.cu:50-84; kernels tentative_coloring
    :88-129, conflict_detection :134-163, update_coloring_GPU :166-174, check_uncolored_nodes :179-190),
    restated with numpy, one Jacobi round per loop iteration. Returns (colours, 1-based; rounds).

    Semantics kept from the reference:
      * every round, each uncoloured node marks the colours of its neighbours (the colouring at the
        round's start, 0 included) in its row of forbiddenColors by writing its own id; the rows are
        never cleared, so marks from earlier rounds stay (a sticky forbidden set), and it takes the
        first colour i >= 1 (i < maxDeg + 1) not marked;
      * node 0 always takes colour 1 (:99-101; its all-zero row reads as fully marked);
      * a coloured node with a same-coloured neighbour of smaller id is uncoloured (:154-160);
      * the loop ends when no node is uncoloured.
    The reference reads the rows of cudaMalloc'ed (uninitialised) memory; zero-initialised rows are
    assumed, which is what a fresh allocation returns in practice. Colours stop at maxDeg (i <
    maxDeg + 1, :17), so a node whose forbidden set fills up (K2: node 1 needs colour 2) never gets
    one and the reference never returns; this restatement (and the HIP colorer) raise instead,
    after 4 maxColors + 64 rounds."""
    off = np.asarray(off, dtype=np.int64)
    idx = np.asarray(idx, dtype=np.int64)
    n = len(off) - 1
    if n == 0:
        return np.zeros(0, dtype=np.uint32), 0
    deg = np.diff(off)
    max_colors = int(deg.max()) + 1
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    col = np.zeros(n, dtype=np.int64)
    temp = np.zeros(n, dtype=np.int64)
    forb = np.zeros((n, max_colors), dtype=bool)
    rounds = 0
    while True:
        rounds += 1
        unc = col == 0
        temp[0] = 1
        m = unc[rows]
        forb[rows[m], col[idx[m]]] = True
        free = ~forb[:, 1:]
        has = free.any(axis=1)
        first = np.argmax(free, axis=1) + 1 if max_colors > 1 else np.ones(n, dtype=np.int64)
        upd = unc & has
        upd[0] = False
        temp[upd] = first[upd]
        col = temp.copy()
        bad = (col[rows] != 0) & (col[rows] == col[idx]) & (rows > idx)
        temp[rows[bad]] = 0
        col = temp.copy()
        if not (col == 0).any():
            return col.astype(np.uint32), rounds
        if rounds > 4 * max_colors + 64:   # a full forbidden set: the reference loops forever here
            raise RuntimeError("greedy first fit: no progress (a node's forbidden set is full)")


def xorwow_step(states):
    """One curand() call on every state at once (xorwow: cuRAND's device header, restated in
    mcmc_colorer_amd/csrc/xorwow.h and pinned by tests/test_xorwow.py). states: [n][6] uint32
    {v0..v4, d}, advanced in place; returns the outputs."""
    s = states
    t = s[:, 0] ^ (s[:, 0] >> np.uint32(2))
    s[:, 0:4] = s[:, 1:5].copy()
    s[:, 4] = (s[:, 4] ^ (s[:, 4] << np.uint32(4))) ^ (t ^ (t << np.uint32(1)))
    s[:, 5] = s[:, 5] + np.uint32(362437)
    return s[:, 4] + s[:, 5]


def curand_uniform(x):
    """curand_uniform: x 2^-32 + 2^-33 in fp32, the product exact, one rounding of the sum."""
    return x.astype(F32) * F32(2.0 ** -32) + F32(2.0 ** -33)


def luby(off, idx, states, max_stale: int = 100000):
    """ColoringLuby::run_fast (graph_coloring/coloringLubyFast.cu:21-110: fast_colorer_k's loops;
    kernels prune_eligible_clear_is :112-118, set_initial_distr_k coloringLuby.cu:232-243,
    check_conflicts_fast_k :121-148, update_eligible_fast_k :150-168, check_finished_k
    coloringLuby.cu:316-324, add_color_and_check_uncolored_k :328-341), restated with numpy.
    states: [n][6] uint32 per-node XORWOW states (GPURand), advanced in place -- every node draws
    once per inner round. Returns (colours 1..k, k, inner rounds).

    The conflict step reads the round's selection snapshot (the reference clears flags in place,
    so its result depends on thread timing; this is its schedule with every read before every
    write): a selected node survives iff no selected neighbour has degree >= its own. A candidate
    that can never survive (a self loop) makes the reference spin; this raises after max_stale
    rounds without a survivor."""
    off = np.asarray(off, dtype=np.int64)
    idx = np.asarray(idx, dtype=np.int64)
    n = len(off) - 1
    deg = np.diff(off)
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    coloring = np.zeros(n, dtype=np.uint32)
    k = rounds = 0
    if n == 0:
        return coloring, 0, 0
    while True:
        cand = coloring == 0
        is_ = np.zeros(n, dtype=bool)
        stale = 0
        while True:
            rounds += 1
            u = curand_uniform(xorwow_step(states))
            sel = (u < F32(0.5)) & cand
            clash = sel[rows] & sel[idx] & (deg[rows] <= deg[idx])
            keep = sel.copy()
            keep[rows[clash]] = False
            is_ |= keep
            cand &= ~keep
            cand[idx[keep[rows]]] = False
            if not cand.any():
                break
            stale = 0 if keep.any() else stale + 1
            if stale > max_stale:
                raise RuntimeError("Luby: no progress")
        k += 1
        coloring[is_] = k
        if not (coloring == 0).any():
            return coloring, k, rounds


def vff(off, idx, max_iter: int = 100000):
    """ColoringVFF::run (graph_coloring/coloringVFF.cu: run :50-56, run_coloring :58-99 -- the
    GreedyFF rounds, restated by greedy_ff above -- run_balancing :101-228, kernels
    detect_unbalanced_nodes :300-311, is_unbalanced :314-323, tentative_rebalancing :326-365,
    update_bins :368-383, solve_conflicts :386-409, ensure_not_looping :412-434), restated with
    numpy. Returns (colours, numColors, balancing iterations, valid).

    Kept from the reference: numColors = distinct greedy colours, gamma = n // numColors; a node is
    unbalanced when its colour's bin holds more than gamma nodes; each iteration an unbalanced node
    forbids its own and its neighbours' colours (of the iteration's input colouring) and moves to
    the first colour 1..numColors not forbidden whose bin (sizes of the previous iteration) holds
    MORE than gamma nodes -- the reference's test, kept as written; node 0's forbidden row is
    flagged with 0, the memset value, so it never moves; then bins are recounted, and an unbalanced
    node stops being unbalanced unless a neighbour of smaller id has its new colour (its colour is
    not reverted). The loop stops when no node is unbalanced or when the unbalanced set has been
    the same for nine snapshots, the ten-row history starting all-false (ensure_not_looping): then
    the result is the greedy colouring and valid is False -- also when one iteration balances
    everything, since the history is then all-false. Deviations: greedy colours that are not
    1..numColors make the reference read past its bins and forbidden rows; this raises instead, as
    it does after max_iter iterations (a cycle longer than the history never ends there)."""
    off = np.asarray(off, dtype=np.int64)
    idx = np.asarray(idx, dtype=np.int64)
    n = len(off) - 1
    gff, _ = greedy_ff(off, idx)
    if n == 0:
        return gff, 0, 0, True
    gff = gff.astype(np.int64)
    ncol = len(np.unique(gff))
    if gff.max() != ncol or gff.min() < 1:
        raise RuntimeError("VFF: greedy colours are not 1..numColors")
    deg = np.diff(off)
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    gamma = n // ncol
    bins = np.bincount(gff, minlength=ncol + 1)
    bins[0] = 0
    unb = gamma < bins[gff]
    coloring = gff.copy()
    hist = [np.zeros(n, dtype=bool) for _ in range(8)]   # the 8 previous snapshots, oldest first
    it = 0
    valid = True
    while unb.any() and valid:
        it += 1
        if it > max_iter:
            raise RuntimeError("VFF: no progress")
        temp = coloring.copy()
        over = gamma < bins                                  # bins[0] = 0: colour 0 never qualifies
        movers = np.nonzero(unb)[0]
        movers = movers[movers != 0]
        if len(movers):
            forb = np.zeros((n, ncol + 1), dtype=bool)
            forb[movers, coloring[movers]] = True
            m = unb[rows] & (rows != 0)
            forb[rows[m], coloring[idx[m]]] = True
            ok = ~forb[movers] & over[None, :]
            ok[:, 0] = False
            has = ok.any(axis=1)
            temp[movers[has]] = np.argmax(ok[has], axis=1)
        bins = np.bincount(temp, minlength=ncol + 1)
        bins[0] = 0
        clash = unb[rows] & (temp[rows] == temp[idx]) & (rows > idx)
        stay = np.zeros(n, dtype=bool)
        stay[rows[clash]] = True
        unb = unb & stay
        coloring = temp
        if all(np.array_equal(unb, h) for h in hist):
            valid = False
        hist = hist[1:] + [unb.copy()]
    out = coloring if valid else gff
    return out.astype(np.uint32), ncol, it, valid
