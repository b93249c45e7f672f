"""The wide sweep (nCol > 256: uint16 colour replicas, csrc/sweep_wide.h).

The reference's default colour count is maxDeg (main.cu:53,162), so power-law and dense graphs run
with hundreds to thousands of colours. The wide sweep keeps the --mcmccpu semantics
(coloringMCMC_CPU.cpp:115-270) bit-exactly; its CDF walk jumps over runs of equal probabilities
(csrc/cdf_walk.h), which the CPU tests pin against a plain float32 step-by-step walk, and the GPU
tests pin against the oracle (final colouring, trajectory, iter, glibc draws).
"""
import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O
from mcmc_colorer_amd import _lib


def naive_walk(mask_bits, ncol, eps, p, u):
    """extract_new_color (:505-520) literally: cdf += p[c] in float32, stop on cdf > u."""
    eps, p, u = np.float32(eps), np.float32(p), np.float32(u)
    cdf = np.float32(0.0)
    for c in range(ncol):
        cdf = np.float32(cdf + (eps if mask_bits[c] else p))
        if cdf > u:
            return c
    return ncol


def lib_walk(mask_bits, ncol, cv, eps, p, u):
    L = _lib.lib()
    if mask_bits is None:
        return L.mcmc_cdf_walk(None, ncol, cv, eps, p, u)
    words = np.zeros((ncol + 31) // 32, dtype=np.uint32)
    for c in np.nonzero(mask_bits)[0]:
        words[c >> 5] |= np.uint32(1 << (int(c) & 31))
    return L.mcmc_cdf_walk(_lib.u32ptr(words), ncol, cv, eps, p, u)


def canon(x):
    """generate_canonical<float,24> of a minstd draw."""
    u = np.float32(np.float32(x - 1) / np.float32(2147483648.0))
    return u if u < 1 else np.float32(np.nextafter(np.float32(1), np.float32(0)))


@pytest.mark.parametrize("case", range(6))
def test_cdf_walk_matches_stepwise_float32(case):
    rng = np.random.default_rng(100 + case)
    eps = [1e-8, 1e-8, 1e-3, 3e-5, 2.0 ** -30 * 77, 1e-8][case]
    mism = []
    for it in range(40):
        ncol = int(rng.integers(2, 1500 if case < 5 else 4000))
        dens = rng.random() ** 3
        bits = rng.random(ncol) < dens
        pop = int(bits.sum())
        if it % 4 == 0:
            u = np.float32(1.0) - np.float32(int(rng.integers(0, 4096))) * np.float32(2.0 ** -24)
        elif it % 4 == 1:
            u = np.float32(int(rng.integers(0, 100000)) * 1e-12)
        else:
            u = canon(int(rng.integers(1, 2**31 - 1)))
        u = np.float32(min(u, np.float32(np.nextafter(np.float32(1), np.float32(0)))))
        if 0 < pop < ncol:
            pf = np.float32((np.float32(1.0) - np.float32(eps) * np.float32(pop)) / np.float32(ncol - pop))
            a, b = lib_walk(bits, ncol, 0, eps, pf, u), naive_walk(bits, ncol, eps, pf, u)
            if a != b:
                mism.append(("mask", ncol, pop, float(u), a, b))
        cv = int(rng.integers(0, ncol))
        hi = np.float32(np.float32(1.0) - np.float32(ncol - 1) * np.float32(eps))
        own = np.zeros(ncol, dtype=bool)
        own[:] = True
        own[cv] = False   # naive_walk: eps where the bit is set, p (= hi) where clear
        a, b = lib_walk(None, ncol, cv, eps, hi, u), naive_walk(own, ncol, eps, hi, u)
        if a != b:
            mism.append(("own", ncol, cv, float(u), a, b))
    assert not mism, mism[:5]


@pytest.mark.parametrize("case", range(4))
def test_cdf_walk_prefix_wave_large_ncol(case):
    """walk_mask_pre (the wide walk's 64-lane binade search, host build) at nCol up to 65535 and
    hub-like occupancies; the hook also checks it against the per-word serial walk (0xFFFFFFFF on
    disagreement), and both against the literal float32 walk."""
    rng = np.random.default_rng(700 + case)
    eps = [1e-8, 1e-8, 2e-6, 1e-4][case]
    mism = []
    for it in range(12):
        ncol = int(rng.integers(3000, 65536))
        dens = [0.02, 0.5, 0.97, rng.random()][it % 4]
        bits = rng.random(ncol) < dens
        if it % 3 == 0:   # long runs of occupied / free colours
            bits[: ncol // 3] = True
            bits[ncol // 3: ncol // 2] = False
        pop = int(bits.sum())
        if not 0 < pop < ncol:
            continue
        u = [canon(int(rng.integers(1, 2**31 - 1))), np.float32(1.0) - np.float32(2.0 ** -24),
             np.float32(int(rng.integers(0, 1000)) * 1e-9)][it % 3]
        pf = np.float32((np.float32(1.0) - np.float32(eps) * np.float32(pop)) / np.float32(ncol - pop))
        a, b = lib_walk(bits, ncol, 0, eps, pf, u), naive_walk(bits, ncol, eps, pf, u)
        if a != b:
            mism.append((ncol, pop, float(u), a, b))
    assert not mism, mism[:5]


def test_cdf_walk_tie_binades_long_runs():
    """A violator with few free colours (long runs of occupied ones): where an addend's increment
    ties (x / ulp a half-integer) the walk steps runs with cdf_run instead of colour by colour; every
    case against the literal float32 walk, pf with odd and even mantissas, u up to just below 1."""
    rng = np.random.default_rng(4242)
    mism, odd = [], 0
    for it in range(24):
        ncol = int(rng.integers(2000, 30000))
        gap = int(rng.integers(50, 900))
        bits = np.ones(ncol, dtype=bool)
        bits[rng.integers(0, gap)::gap] = False
        pop = int(bits.sum())
        eps = [1e-8, 3e-7, 2.0 ** -30 * 3][it % 3]
        pf = np.float32((np.float32(1.0) - np.float32(eps) * np.float32(pop)) / np.float32(ncol - pop))
        odd += int(np.frombuffer(pf.tobytes(), dtype=np.uint32)[0] & 1)
        for u in (np.float32(1.0) - np.float32(2.0 ** -24), canon(int(rng.integers(1, 2**31 - 1))),
                  np.float32(pf * np.float32(rng.integers(1, 6)))):
            a, b = lib_walk(bits, ncol, 0, eps, pf, u), naive_walk(bits, ncol, eps, pf, u)
            if a != b:
                mism.append((ncol, gap, eps, float(pf), float(u), a, b))
    assert odd > 0
    assert not mism, mism[:5]


def _tie_binades(pf):
    """Binades E (biased exponents above pf's, up to 1.0's) where adding pf ties (x / ulp = d + 1/2)."""
    b = int(np.frombuffer(np.float32(pf).tobytes(), dtype=np.uint32)[0])
    ex, mx = b >> 23, (b & 0x7FFFFF) | 0x800000
    return [E for E in range(ex + 1, 127) if E - ex <= 25 and (mx & ((1 << (E - ex)) - 1)) == 1 << (E - ex - 1)]


def test_cdf_walk_tie_binades_mixed_masks():
    """A violator's mask with short runs (random occupancy 5-60 %) whose pf ties in a wide binade:
    walk_mask_pre's word-function path (each word a function of the mantissa's parity, composed 64
    words at a time) against the literal float32 walk, u inside, below and above the tie binade."""
    rng = np.random.default_rng(9090)
    mism, cases = [], 0
    for it in range(4000):
        if cases >= 40:
            break
        ncol = int(rng.integers(1500, 20000))
        dens = float(rng.uniform(0.05, 0.6))
        bits = rng.random(ncol) < dens
        pop = int(bits.sum())
        eps = [1e-8, 3e-7, 2.0 ** -30 * 3][it % 3]
        pf = np.float32((np.float32(1.0) - np.float32(eps) * np.float32(pop)) / np.float32(ncol - pop))
        ties = [E for E in _tie_binades(pf) if E >= 120]
        if not ties:
            continue
        cases += 1
        E = ties[-1]
        lo = np.float32(2.0 ** (E - 127))
        for u in (np.float32(lo * np.float32(1.5)), np.float32(lo * np.float32(1.999)), np.float32(lo * np.float32(0.75)),
                  np.float32(1.0) - np.float32(2.0 ** -24), canon(int(rng.integers(1, 2**31 - 1)))):
            u = np.float32(min(u, np.float32(np.nextafter(np.float32(1), np.float32(0)))))
            a, b = lib_walk(bits, ncol, 0, eps, pf, u), naive_walk(bits, ncol, eps, pf, u)
            if a != b:
                mism.append((ncol, pop, eps, float(pf), float(u), a, b))
    assert cases >= 20
    assert not mism, mism[:5]


def test_cdf_walk_tie_binade_large_free_increment():
    """eps ties in the binade of 2 eps (odd mantissa) while pf / eps is 32-512: there a free colour
    moves the mantissa integer by up to 2^31 units, so a 32-colour word's increment does not fit 32
    bits. Masks enter that binade through occupied colours and then mix free ones; every
    case against the literal float32 walk."""
    rng = np.random.default_rng(5151)
    mism, cases = [], 0
    for it in range(300):
        eps = np.float32(rng.uniform(2e-6, 5e-5))
        b = int(np.frombuffer(eps.tobytes(), dtype=np.uint32)[0]) | 1   # odd mantissa: ties at 2 eps
        eps = np.frombuffer(np.uint32(b).tobytes(), dtype=np.float32)[0]
        ratio = float(rng.uniform(32, 512))
        nfree = max(2, int(1.0 / (float(eps) * ratio)))
        ncol = nfree + int(rng.integers(nfree // 4 + 1, 2 * nfree + 2))
        bits = np.ones(ncol, dtype=bool)
        free = rng.choice(np.arange(2, ncol), size=nfree, replace=False)
        bits[free] = False
        bits[:2] = True                                   # cdf = 2 eps: the tie binade
        bits[2:2 + int(rng.integers(2, 30))] = False      # then a run of free colours in that word
        pop = int(bits.sum())
        pf = np.float32((np.float32(1.0) - eps * np.float32(pop)) / np.float32(ncol - pop))
        if not (32 <= pf / eps <= 512):
            continue
        cases += 1
        for u in (canon(int(rng.integers(1, 2**31 - 1))), np.float32(pf * np.float32(rng.uniform(1, 20))),
                  np.float32(1.0) - np.float32(2.0 ** -24), np.float32(eps * np.float32(rng.uniform(2, 40)))):
            u = np.float32(min(u, np.float32(np.nextafter(np.float32(1), np.float32(0)))))
            a, b2 = lib_walk(bits, ncol, 0, eps, pf, u), naive_walk(bits, ncol, eps, pf, u)
            if a != b2:
                mism.append((ncol, pop, float(eps), float(pf), float(u), a, b2))
    assert cases >= 50
    assert not mism, mism[:5]


# ---------------------------------------------------------------------------------------------
# GPU parity


@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def run_both(M, off, idx, ncol, seed=1, variant="wide", **kw):
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, epsilon=kw.get("epsilon", 1e-8), maxRip=kw.get("maxRip", 250),
                                  tabooIteration=kw.get("tabooIteration", 0), tailcut=kw.get("tailcut", False))
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, seed, M.GlibcRand(1)), params)
    st = col.run(0)
    O.srand(1)   # both glibc streams at srand(1), no draws
    r = O.mcmc_run(off, idx, ncol, seed, **kw)
    assert col.info()["variant"] == variant
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws, st.initDraws) == (
        r.res.iter, bool(r.res.maxIterReached), r.res.finalViol, r.res.glibcDraws, r.res.initDraws)
    return st, r


@pytest.mark.gpu
def test_wide_default_ncol_maxdeg_dense():
    """nCol = maxDeg > 256 by default (main.cu:162) on an exact --simulate graph."""
    import mcmc_colorer_amd.colorer as M

    O.srand(1)
    off, idx = O.setup_rnd2(1200, 0.3)
    ncol = O.max_deg(off)
    assert ncol > 256
    run_both(M, off, idx, ncol)


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,seed", [(4000, 0.1, 7), (9000, 0.04, 3)])
def test_wide_generated_graph_default_ncol(n, p, seed):
    """The reference's default nCol = maxDeg (main.cu:162) on a graph of the build's generator
    (--simulate at C3/C4 scale, no CSR until the wide sweep asks for one): mcmc_create builds the
    CSR from the tiled layout (mcmc_graph_materialize_csr) and runs the wide sweep; colouring,
    trajectory and loop state equal the oracle's run on the oracle's restatement of the same graph."""
    import mcmc_colorer_amd.colorer as M

    off, idx = O.er_fast(n, p, seed)
    ncol = O.max_deg(off)
    assert ncol > 256
    g = M.Graph.er_fast(n, p, seed)
    assert g.maxDeg == ncol and g.nEdges == len(idx)
    params = M.ColoringMCMCParams(nCol=M.default_ncol(g, M.ColoringMCMCParams(nCol=0)), maxRip=40)
    assert params.nCol == ncol
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), params)
    st = col.run(0)
    assert col.info()["variant"] == "wide"
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=40)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    col.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ncol,eps,taboo,tailcut", [(300, 1e-8, 0, False), (1000, 1e-8, 2, False),
                                                     (700, 1e-3, 0, False), (4000, 1e-8, 0, True),
                                                     (65535, 1e-8, 0, False)])
def test_wide_sparse(M, ncol, eps, taboo, tailcut):
    O.srand(1)
    off, idx = O.setup_rnd2(3000, 0.01)
    run_both(M, off, idx, ncol, epsilon=eps, tabooIteration=taboo, tailcut=tailcut)


@pytest.mark.gpu
@pytest.mark.parametrize("ncol,eps,taboo", [(16, 1e-8, 0), (16, 1e-3, 0), (7, 1e-8, 3), (256, 1e-2, 0)])
def test_wide_forced_small_ncol(M, monkeypatch, ncol, eps, taboo):
    """MCMC_GATHER=wide on nCol <= 256: every vertex violates (C2-like), events, taboo."""
    monkeypatch.setenv("MCMC_GATHER", "wide")
    O.srand(1)
    off, idx = O.setup_rnd2(2000, 0.05)
    run_both(M, off, idx, ncol, epsilon=eps, tabooIteration=taboo, maxRip=60)


# The wide sweep over the tiled layout (variant 6, csrc/wide_tiled.h): what a generated graph too
# large for a CSR beside its layout runs at nCol > 256 (C3 at nCol = maxDeg, tests/test_c3_full.py).
# MCMC_GATHER=wide-tiled forces it on CSR graphs (the layout is built from the CSR) and on small nCol.


@pytest.mark.gpu
@pytest.mark.parametrize("ncol,eps,taboo,tailcut", [(300, 1e-8, 0, False), (1000, 1e-8, 2, False),
                                                     (700, 1e-3, 0, False), (4000, 1e-8, 0, True),
                                                     (65535, 1e-8, 0, False)])
def test_wide_tiled_sparse(M, monkeypatch, ncol, eps, taboo, tailcut):
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    O.srand(1)
    off, idx = O.setup_rnd2(3000, 0.01)
    run_both(M, off, idx, ncol, variant="wide-tiled", epsilon=eps, tabooIteration=taboo, tailcut=tailcut)


@pytest.mark.gpu
@pytest.mark.parametrize("ncol,eps,taboo", [(16, 1e-8, 0), (16, 1e-3, 0), (7, 1e-8, 3), (256, 1e-2, 0)])
def test_wide_tiled_forced_small_ncol(M, monkeypatch, ncol, eps, taboo):
    """Every vertex violates (C2-like): the mask walk on every row, CDF overflow events, taboo."""
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    O.srand(1)
    off, idx = O.setup_rnd2(2000, 0.05)
    run_both(M, off, idx, ncol, variant="wide-tiled", epsilon=eps, tabooIteration=taboo, maxRip=60)


@pytest.mark.gpu
def test_wide_tiled_dense_default_ncol(M, monkeypatch):
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    O.srand(1)
    off, idx = O.setup_rnd2(1200, 0.3)
    run_both(M, off, idx, O.max_deg(off), variant="wide-tiled")


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ["1", "7", "1024"])
def test_wide_tiled_skewed_degrees(M, monkeypatch, rows):
    """A hub row of ~4 000 arcs beside empty ones, several group sizes of the layout."""
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    monkeypatch.setenv("MCMC_GROUP_ROWS", rows)
    off, idx = _hub_graph()
    run_both(M, off, idx, O.max_deg(off), variant="wide-tiled")
    run_both(M, off, idx, 300, variant="wide-tiled", maxRip=30)


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,seed", [(4000, 0.1, 7), (70000, 0.01, 3)])
def test_wide_tiled_generated_graph(M, monkeypatch, n, p, seed):
    """The build's generated G(n, p) at nCol = maxDeg over its own layout (no CSR at all; the second
    graph spans two 64 Ki column blocks), against the oracle's run on its restatement of the graph."""
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    off, idx = O.er_fast(n, p, seed)
    ncol = O.max_deg(off)
    g = M.Graph.er_fast(n, p, seed)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=12))
    st = col.run(0)
    assert col.info()["variant"] == "wide-tiled"
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=12)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    col.close()


@pytest.mark.gpu
@pytest.mark.parametrize("inc", ["0", "1", "2", "1/div2", "1/scan", "2/scan"])
@pytest.mark.parametrize("case", ["sparse", "taboo", "eps1e3", "hub", "every_vertex", "tailcut", "generated"])
def test_wide_tiled_incremental(M, monkeypatch, inc, case):
    """The wide tiled sweep's incremental violation counts (csrc/wide_tiled.h wt_*): MCMC_WT_INC=0
    scans every sweep, 1 (default) chooses per sweep (incremental while the changed rows' arcs are at
    most 1 / MCMC_WT_ARCS_DIV of the layout's, default 32 with the recount, 2 with the mask scan;
    "1/div2": 2), 2 runs every sweep after the first from the counts (lane-per-row evaluation,
    violators walked from a list, the counts moved by the changed rows). A full sweep is the
    block-major recount + those kernels (default) or the mask scan ("/scan": MCMC_WT_RC=0). Each run
    equals the oracle's; the statistics show which sweeps were incremental."""
    monkeypatch.setenv("MCMC_GATHER", "wide-tiled")
    if inc == "1/div2":
        inc = "1"
        monkeypatch.setenv("MCMC_WT_ARCS_DIV", "2")
    elif inc.endswith("/scan"):
        inc = inc[0]
        monkeypatch.setenv("MCMC_WT_RC", "0")
    monkeypatch.setenv("MCMC_WT_INC", inc)
    kw = {}
    if case == "generated":
        off, idx = O.er_fast(70000, 0.01, 3)
        ncol, kw = O.max_deg(off), {"maxRip": 12}
        g = M.Graph.er_fast(70000, 0.01, 3)
        col = M.ColoringMCMC(g, M.GPURand(70000, 3, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=12))
        st = col.run(0)
        O.srand(1)
        r = O.mcmc_run(off, idx, ncol, 3, maxRip=12)
        assert col.coloring().tolist() == r.colors.tolist()
        assert col.trajectory().tolist() == r.traj.tolist()
        assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
        ws = col.wide_inc_stats()
    else:
        if case == "hub":
            off, idx = _hub_graph()
            ncol = 300
            kw = {"maxRip": 30}
        elif case == "every_vertex":   # nCol 16: every vertex violates every sweep
            O.srand(1)
            off, idx = O.setup_rnd2(2000, 0.05)
            ncol, kw = 16, {"maxRip": 40}
        else:
            O.srand(1)
            off, idx = O.setup_rnd2(3000, 0.01)
            ncol = {"sparse": 300, "taboo": 1000, "eps1e3": 700, "tailcut": 4000}[case]
            kw = {"taboo": {"tabooIteration": 2}, "eps1e3": {"epsilon": 1e-3},
                  "tailcut": {"tailcut": True}}.get(case, {})
        g = M.Graph.from_csr(off, idx)
        params = M.ColoringMCMCParams(nCol=ncol, epsilon=kw.get("epsilon", 1e-8), maxRip=kw.get("maxRip", 250),
                                      tabooIteration=kw.get("tabooIteration", 0), tailcut=kw.get("tailcut", False))
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
        st = col.run(0)
        O.srand(1)
        r = O.mcmc_run(off, idx, ncol, 1, **kw)
        assert col.info()["variant"] == "wide-tiled"
        assert col.coloring().tolist() == r.colors.tolist()
        assert col.trajectory().tolist() == r.traj.tolist()
        assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws) == (
            r.res.iter, bool(r.res.maxIterReached), r.res.finalViol, r.res.glibcDraws)
        ws = col.wide_inc_stats()
    sweeps = int(st.sweepsRun)
    if inc == "0":
        assert not ws["enabled"]
    else:
        assert ws["enabled"] and ws["full_sweeps"] >= 1
        if inc == "2" and sweeps > 1:
            assert ws["incremental_sweeps"] >= 1 and ws["full_sweeps"] == 1, ws
    col.close()


def _hub_graph(n=5000):
    """A hub joined to n - 1000 vertices plus a sparse remainder: one long row, many empty/short ones."""
    rng = np.random.default_rng(5)
    E = set()
    for v in range(1, n):
        E.add((0, v))
    for _ in range(8000):
        a, b = rng.integers(1, n, 2)
        if a != b:
            E.add((min(a, b), max(a, b)))
    for v in range(n - 1000, n):   # isolated tail: drop the hub arcs too
        E.discard((0, v))
    arcs = sorted([(a, b) for a, b in E] + [(b, a) for a, b in E])
    src = np.array([a for a, _ in arcs], dtype=np.int64)
    idx = np.array([b for _, b in arcs], dtype=np.uint32)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.add.at(off, src + 1, 1)
    off = np.cumsum(off).astype(np.uint64)
    return off, idx


@pytest.mark.gpu
def test_wide_skewed_degrees(M):
    """A hub joined to every vertex plus a sparse remainder: one long row, many empty/short ones."""
    off, idx = _hub_graph()
    ncol = O.max_deg(off)
    run_both(M, off, idx, ncol)
    run_both(M, off, idx, 300, maxRip=30)


INC_CASES = {
    # name: (graph, nCol, run kwargs, env)
    "rmat-maxdeg": ("rmat", None, {}, {}),
    "rmat-300": ("rmat", 300, {"maxRip": 25}, {}),
    "hub": ("hub", 300, {"maxRip": 30}, {}),
    "big-hub": ("bighub", 300, {"maxRip": 30}, {}),   # a 10 999-arc hub: three delta tasks (kIncHubTask)
    "sparse-taboo": ("sparse", 1000, {"tabooIteration": 2, "maxRip": 40}, {}),
    "sparse-eps": ("sparse", 700, {"epsilon": 1e-3, "maxRip": 40}, {}),
    "dense-all-change": ("dense", 16, {"maxRip": 30}, {"MCMC_GATHER": "wide"}),
}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["0", "1", "2"])
@pytest.mark.parametrize("case", list(INC_CASES))
def test_wide_incremental_counts(M, monkeypatch, mode, case):
    """The wide sweep's incremental violation counts (sweep_wide.h wide_inc_*): each sweep moves
    every row's same-colour count by the rows that changed colour instead of rescanning every edge
    (violation_count, coloringMCMC_CPU.cpp:329-351, is count > 0). Off (0), the default choice per
    sweep (1) and forced after the first full sweep (2) -- including sweeps where EVERY vertex
    changes (nCol 16: both ends of most arcs changed), hubs past kIncHub arcs (their own
    kernel), taboo, eps 1e-3 (own-colour moves) -- give the oracle's colouring and trajectory."""
    graph, ncol, kw, env = INC_CASES[case]
    monkeypatch.setenv("MCMC_WIDE_INC", mode)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if graph == "rmat":
        off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    elif graph == "hub":
        off, idx = _hub_graph()
    elif graph == "bighub":
        off, idx = _hub_graph(12000)
    elif graph == "sparse":
        O.srand(1)
        off, idx = O.setup_rnd2(3000, 0.01)
    else:
        O.srand(1)
        off, idx = O.setup_rnd2(2000, 0.05)
    ncol = ncol or O.max_deg(off)
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, epsilon=kw.get("epsilon", 1e-8), maxRip=kw.get("maxRip", 250),
                                  tabooIteration=kw.get("tabooIteration", 0))
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    st = col.run(0)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, 1, **kw)
    assert col.info()["variant"] == "wide"
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    s = col.wide_inc_stats()
    assert s["enabled"] == (mode != "0")
    if mode == "2" and st.iter > 1:
        assert s["full_sweeps"] == 1 and s["incremental_sweeps"] >= 1, s
    col.close()


WS_CASES = {
    # name: (graph, nCol, run kwargs, env, what the stats must show)
    "rmat-300": ("rmat", 300, {"maxRip": 25}, {}, "walk_phases"),
    "rmat-phases": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_LEAD_ARCS": "0", "MCMC_WS_LIGHT": "8"}, "delta_phases"),
    "rmat-maxdeg": ("rmat", None, {}, {}, "sweeps"),
    "hub-300": ("hub", 300, {"maxRip": 30}, {}, "sweeps"),
    "hub-heavy": ("hub", 300, {"maxRip": 30}, {"MCMC_WS_LIGHT": "1", "MCMC_WS_LEAD_ARCS": "0"}, "delta_phases"),
    "dense-maxdeg": ("dense", None, {}, {}, "sweeps"),
    "sparse-eps": ("sparse", 1000, {"epsilon": 2e-6, "maxRip": 40}, {}, "candidates"),
    "sparse-65535": ("sparse", 65535, {"maxRip": 40}, {}, "sweeps"),
    "all-change-16": ("dense16", 16, {"maxRip": 30}, {"MCMC_GATHER": "wide"}, "walk_phases"),
    "rmat-poll-debug": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_POLL": "8", "MCMC_WS_DEBUG": "1"}, "walk_phases"),
    "rmat-poll-spin": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_POLL": "0", "MCMC_WS_POLL_IDLE": "0"}, "walk_phases"),
    "rmat-poll-idle": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_POLL_IDLE": "256"}, "walk_phases"),
    "rmat-light-4096": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_LIGHT": "4096"}, "walk_phases"),
    "hub-lead-heavy": ("hub", 300, {"maxRip": 30}, {"MCMC_WS_LEAD_HEAVY": "65536"}, "sweeps"),
    "rmat-lead-heavy": ("rmat", 300, {"maxRip": 25}, {"MCMC_WS_LEAD_HEAVY": "65536"}, "sweeps"),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(WS_CASES))
def test_wide_persistent(M, monkeypatch, case):
    """The persistent wide sweep (csrc/wide_solo.h): candidate rows from the discrete-log window,
    violators walked by the leader or by walk phases (a wave each, heavy rows a workgroup), counts
    moved by the leader or by delta phases, the violator list kept or recollected. Every case equals
    the oracle's run (colouring, trajectory, iter, glibc draws); the statistics show the path ran."""
    graph, ncol, kw, env, key = WS_CASES[case]
    monkeypatch.setenv("MCMC_WS_ENTER", "-1")   # every batch (default: only once Cviol <= 512)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if graph == "rmat":
        off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    elif graph == "hub":
        off, idx = _hub_graph()
    elif graph == "sparse":
        O.srand(1)
        off, idx = O.setup_rnd2(3000, 0.01)
    elif graph == "dense16":
        O.srand(1)
        off, idx = O.setup_rnd2(2000, 0.05)
    else:
        O.srand(1)
        off, idx = O.setup_rnd2(1200, 0.3)
    ncol = ncol or O.max_deg(off)
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, epsilon=kw.get("epsilon", 1e-8), maxRip=kw.get("maxRip", 250))
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    st = col.run(0)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, 1, **kw)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws) == (
        r.res.iter, bool(r.res.maxIterReached), r.res.finalViol, r.res.glibcDraws)
    ws = col.wide_solo_stats()
    assert ws["enabled"] == 1 and ws["sweeps"] >= 1 and ws[key] > 0, ws
    col.close()
    # MCMC_WS_MAX below the window: no persistent sweep, the same run
    monkeypatch.setenv("MCMC_WS_MAX", "1")
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    col.run(0)
    assert col.wide_solo_stats()["enabled"] == 0 and col.coloring().tolist() == r.colors.tolist()
    monkeypatch.delenv("MCMC_WS_MAX")
    # the same run from the same colouring with the per-sweep path only
    monkeypatch.setenv("MCMC_WIDE_SOLO", "0")
    col2 = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    st2 = col2.run(0)
    assert col2.wide_solo_stats()["enabled"] == 0
    assert col2.coloring().tolist() == r.colors.tolist() and st2.iter == st.iter
    col.close()
    col2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("enter", ["-1", "1000000000"])
def test_wide_persistent_steps_alternate(M, monkeypatch, enter):
    """step() batches of 1, 3, 16 and 2 sweeps through the persistent launch (each entry finds the
    violator list the last launch left): the trajectory and colouring equal one uninterrupted
    oracle run of 22 sweeps. enter = 1e9: the first batch of a fresh colouring (Cviol unknown) takes
    the per-sweep path, the later ones the persistent sweep."""
    monkeypatch.setenv("MCMC_GATHER", "wide")   # nCol 16 on a dense graph: violators every sweep
    monkeypatch.setenv("MCMC_WS_ENTER", enter)
    O.srand(1)
    off, idx = O.setup_rnd2(2000, 0.05)
    ncol = 16
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, maxRip=40)
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    col.init(0)
    for k in (1, 3, 16, 2):
        col.step(k)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, 1, maxRip=40, sweep_limit=22)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist()[:22] == r.traj.tolist()[:22]
    assert col.wide_solo_stats()["sweeps"] >= (20 if enter == "-1" else 19)
    col.close()


@pytest.mark.gpu
@pytest.mark.parametrize("enter", [None, "1000000000"])
def test_wide_persistent_hybrid(M, monkeypatch, enter):
    """The default path choice: a run's first batch (16 sweeps) takes the per-sweep path, later
    batches the persistent sweep once Cviol <= MCMC_WS_ENTER (default 512); one run switching paths
    equals the oracle's run."""
    if enter is not None:
        monkeypatch.setenv("MCMC_WS_ENTER", enter)
    off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    g = M.Graph.from_csr(off, idx)
    kw = {"maxRip": 40}
    params = M.ColoringMCMCParams(nCol=300, maxRip=40)
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), params)
    st = col.run(0)
    O.srand(1)
    r = O.mcmc_run(off, idx, 300, 1, **kw)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    ws = col.wide_solo_stats()
    traj = r.traj.tolist()
    if enter is not None and len(traj) > 17:
        assert 1 <= ws["sweeps"] <= len(traj) - 16, (ws, len(traj))
    elif len(traj) <= 16 or min(traj[15:]) > 512:
        assert ws["sweeps"] == 0, ws
    col.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scan", ["lds", "l2", "csr"])
def test_wide_rmat_both_scans(M, monkeypatch, scan):
    """Power-law graph (R-MAT): the slab edge layouts (one entry per edge, both ends flagged; LDS
    colour tiles or 8 XCD slabs through L2) and the CSR arc scan give the oracle's run, at nCol = maxDeg and at a smaller nCol whose
    sweeps keep hundreds of violators (the workgroup-per-violator walk)."""
    monkeypatch.setenv("MCMC_WIDE_SCAN", scan)
    off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    ncol = O.max_deg(off)
    assert ncol > 256
    run_both(M, off, idx, ncol)
    run_both(M, off, idx, 300, maxRip=25)


@pytest.mark.gpu
@pytest.mark.parametrize("split_arcs", [7, 64, 1 << 20])
def test_wide_split_walks(M, monkeypatch, split_arcs):
    """The walk kernel's tasks: a violator above split_arcs arcs has its gathers dealt out over the
    grid and merged in a global mask that the last task walks (while kSplitMax masks last; then one
    workgroup each). Hubs cut into many tasks, more split violators than masks, no split at all."""
    monkeypatch.setenv("MCMC_SPLIT_ARCS", str(split_arcs))
    off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    run_both(M, off, idx, O.max_deg(off))
    run_both(M, off, idx, 300, maxRip=25)


@pytest.mark.gpu
def test_wide_asymmetric_csr(M):
    """Directed arcs without their reverse (mcmc_graph_upload accepts any CSR): the slab layout
    must keep every arc and flag only its row (violation_count reads N(v) only, :329-351)."""
    rng = np.random.default_rng(9)
    n = 3000
    E = set()
    for _ in range(30000):
        a, b = rng.integers(0, n, 2)
        if a != b:
            E.add((int(a), int(b)))
    arcs = sorted(E)
    src = np.array([a for a, _ in arcs], dtype=np.int64)
    idx = np.array([b for _, b in arcs], dtype=np.uint32)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.add.at(off, src + 1, 1)
    off = np.cumsum(off).astype(np.uint64)
    run_both(M, off, idx, 300, maxRip=30)
    run_both(M, off, idx, 20000, maxRip=10)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("scan", ["lds", "csr"])
def test_wide_partitioned_lockstep(M, monkeypatch, world, scan):
    """configs[4]'s multi-GPU shape: the wide sweep vertex-partitioned (2-byte colour regions +
    footers, one all-gather per sweep, rank-ordered glibc replay), ranks in lock-step on one GPU,
    equal to the unpartitioned oracle run -- at nCol = maxDeg and with persistent violators."""
    from test_gpu_parity import _lockstep

    monkeypatch.setenv("MCMC_WIDE_SCAN", scan)
    off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
    for ncol, maxrip in ((O.max_deg(off), 250), (300, 20)):
        ranks = _lockstep(M, off, idx, ncol, 1, world, maxRip=maxrip, draws=0)
        O.srand(1)
        r = O.mcmc_run(off, idx, ncol, 1, maxRip=maxrip)
        for b in ranks:
            assert b.info()["variant"] == "wide"
            assert b.state()[0]
            assert b.coloring().tolist() == r.colors.tolist()
            assert b.trajectory().tolist() == r.traj.tolist()
        for b in ranks:
            b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("graph,ncol,forced", [("simulate", 260, False), ("simulate", 300, False),
                                               ("rmat", 60, True), ("rmat", 100, True), ("simulate", 40, True)])
def test_wide_tailcut_repair(M, monkeypatch, graph, ncol, forced):
    """The corrected tail cut (coloringMCMC_CPU.cpp:272-311, k++) on the wide sweep's uint16
    replicas (--tailcut --tailcutRepair with nCol > 256, configs[4]'s shape on R-MAT graphs):
    colouring, repaired Cviol, passes and trajectory equal the oracle's."""
    if forced:
        monkeypatch.setenv("MCMC_GATHER", "wide")
    if graph == "rmat":
        off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 3)
        draws = 0
    else:
        O.srand(1)
        off, idx = O.setup_rnd2(1500, 0.2)
        draws = 1500 * 1501 // 2
    n = len(off) - 1
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, maxRip=60, tailcut=True, tailcutRepair=1000)
    col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1, draws)), params)
    st = col.run(0)
    O.srand(1)
    if draws:
        O.setup_rnd2(1500, 0.2)
    r = O.mcmc_run(off, idx, ncol, 1, maxRip=60, tailcut=True, tailcutRepair=True)
    assert col.info()["variant"] == "wide"
    assert r.res.tailcutPasses >= 1 or ncol == 40
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.tailcutPasses, st.glibcDraws) == (
        r.res.iter, r.res.finalViol, r.res.tailcutPasses, r.res.glibcDraws)
