"""Pins the oracle (oracle/mcmc_cpu_ref.cpp) before anything is checked against it.

1. Known-answer tests for the third-party arithmetic the reference calls:
   C++ [rand.predef] minstd_rand0, glibc rand(), generate_canonical<float,24>, uniform_int.
2. An independent numpy restatement (oracle/oracle_np.py, no libstdc++/glibc) must agree with
   the C++ oracle bit-for-bit on small graphs, including taboo, tail-cut threshold and
   CDF-overflow (glibc replay) cases.
3. The OpenMP variant (CPU baseline on many cores) equals the faithful single-thread run.
"""
import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O


def test_minstd_kat():
    out = np.zeros(10000, dtype=np.uint32)
    O.lib().oracle_minstd_seq(1, 10000, out.ctypes.data)
    assert out[:3].tolist() == [16807, 282475249, 1622650073]
    assert int(out[9999]) == 1043618065          # C++ [rand.predef]: 10000th output


def test_glibc_kat():
    O.srand(1)
    assert O.rand(5) == [1804289383, 846930886, 1681692777, 1714636915, 1957747793]
    g = NP.GlibcRand(1)
    assert [g() for _ in range(5)] == [1804289383, 846930886, 1681692777, 1714636915, 1957747793]


@pytest.mark.parametrize("seed", [0, 2, 12345, 2**31 + 5, 2**32 - 1])
def test_glibc_seeds_match_numpy(seed):
    O.srand(seed)
    g = NP.GlibcRand(seed)
    assert O.rand(400) == [g() for _ in range(400)]


def test_canonical_clamp_and_values():
    # generate_canonical<float,24>: x - 1 >= 2147483584 rounds to 2^31 and clamps to 1 - 2^-24.
    for x in (1, 2, 1000, 2147483520, 2147483521, 2147483584, 2147483585, 2147483646):
        u = NP.canonical(x)
        assert np.float32(u) < np.float32(1.0)
    assert NP.canonical(2147483646) == np.nextafter(np.float32(1), np.float32(0))
    assert NP.canonical(1) == np.float32(0.0)
    out = np.zeros(2000, dtype=np.float32)
    O.lib().oracle_canonical_seq(7, 0, 2000, out.ctypes.data)
    m = NP.Minstd(7)
    assert np.array_equal(out, np.array([NP.canonical(m()) for _ in range(2000)], dtype=np.float32))


@pytest.mark.parametrize("ncol", [1, 2, 3, 16, 32, 137, 1000])
def test_uniform_int_matches_numpy(ncol):
    out = np.zeros(3000, dtype=np.uint32)
    draws = O.lib().oracle_uniform_int_seq(3, ncol, 3000, out.ctypes.data)
    m = NP.Minstd(3)
    ref, d = [], 0
    for _ in range(3000):
        v, k = NP.uniform_int(m, ncol)
        ref.append(v)
        d += k
    assert out.tolist() == ref and draws == d


CASES = [
    # n, p, nCol, seed, eps, taboo, maxRip
    (40, 0.3, 6, 1, 1e-8, 0, 250),
    (60, 0.2, 5, 7, 1e-8, 0, 20),
    (50, 0.5, 8, 3, 1e-8, 2, 30),
    (30, 0.9, 4, 11, 3.3e6, 1, 15),
    (80, 0.3, 7, 5, 3.3e6, 0, 12),
    (70, 0.1, 2, 9, 1e-8, 0, 10),
    (45, 0.4, 40, 2, 1e-8, 0, 30),
]


@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip", CASES)
def test_cpp_oracle_equals_numpy_restatement(n, p, ncol, seed, eps, taboo, maxrip):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    r = O.mcmc_run(off, idx, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    g = NP.GlibcRand(1)
    off2, idx2 = NP.setup_rnd2(n, p, g)
    assert np.array_equal(off, off2) and np.array_equal(idx, idx2)
    C, traj, it, maxr, init = NP.mcmc_run(off2, idx2, ncol, seed, g, max_rip=maxrip, taboo_iter=taboo,
                                         eps=np.float32(eps))
    assert np.array_equal(r.init, init)
    assert np.array_equal(r.colors, C)
    assert r.traj.tolist() == traj
    assert r.res.iter == it and bool(r.res.maxIterReached) == maxr
    # the glibc streams must have advanced identically (events drew the same number of rand())
    assert O.rand(3) == [g() for _ in range(3)]


def test_events_case_really_draws_glibc():
    O.srand(1)
    off, idx = O.setup_rnd2(80, 0.3)
    r = O.mcmc_run(off, idx, 7, 5, epsilon=3.3e6, maxRip=12)
    assert r.res.glibcDraws > 0


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_openmp_variant_bit_identical(threads):
    O.srand(1)
    off, idx = O.setup_rnd2(600, 0.05)
    for eps, taboo in ((1e-8, 0), (3.3e6, 2)):
        O.srand(77)
        a = O.mcmc_run(off, idx, 9, 4, epsilon=eps, tabooIteration=taboo, maxRip=40)
        O.srand(77)
        b = O.mcmc_run(off, idx, 9, 4, epsilon=eps, tabooIteration=taboo, maxRip=40, nthreads=threads)
        assert np.array_equal(a.colors, b.colors)
        assert a.traj.tolist() == b.traj.tolist()
        assert a.res.glibcDraws == b.res.glibcDraws


def _viol_flags(off, idx, C):
    return np.array([bool(np.any(C[idx[off[i]:off[i + 1]]] == C[i])) for i in range(len(off) - 1)])


def _py_tail_cut(off, idx, C, flags, ncol, z, cap=1000):
    """coloringMCMC_CPU.cpp:272-311 with k++ (the reference increments i and never returns),
    restated in Python: colorIdx by ascending histogram when z > 0 (a stable sort equals libstdc++'s
    std::sort for nCol <= 16, a plain insertion sort), then Gauss-Seidel passes over the flagged
    vertices, first free colour in colorIdx order, recount."""
    C = C.copy()
    order = list(range(ncol))
    if z > 0:
        hist = np.bincount(C, minlength=ncol)
        order = sorted(order, key=lambda c: hist[c])
    cviol, passes = int(_viol_flags(off, idx, C).sum()), 0
    while cviol > 0 and passes < cap:
        for i in np.flatnonzero(flags):
            used = set(C[idx[off[i]:off[i + 1]]].tolist())
            for c in order:
                if c not in used:
                    C[i] = c
                    break
        flags = _viol_flags(off, idx, C)
        cviol, passes = int(flags.sum()), passes + 1
    return C, cviol, passes


@pytest.mark.parametrize("n,p,ncol,seed,maxrip,tailcut", [
    (400, 0.05, 12, 2, 250, True),   # loop stops at Cviol <= 50, one pass repairs the rest
    (500, 0.02, 7, 1, 250, True),    # stops within z, the repair oscillates: runs to the pass bound
    (250, 0.2, 5, 3, 30, False),     # too few colours: cap reached, passes hit the bound
    (200, 0.01, 16, 4, 250, True),   # initial colouring already within z: no accepted sweep
    (300, 0.1, 40, 5, 3, False),     # nCol > 16, identity colorIdx
])
def test_oracle_tail_cut_equals_python_restatement(n, p, ncol, seed, maxrip, tailcut):
    """Pins the oracle's corrected tail cut, including the reference's quirk that the first pass
    visits the vertices flagged in the colouring BEFORE the last accepted sweep (run() swaps C and
    Cstar but not Cviols, coloringMCMC_CPU.cpp:259-260). The reference itself never returns from
    its tail cut (:289 increments i), so this restatement is the pin (parity unpinned against the
    reference's own output: there is none)."""
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    O.srand(1)
    O.setup_rnd2(n, p)
    base = O.mcmc_run(off, idx, ncol, seed, maxRip=maxrip, tailcut=tailcut)
    O.srand(1)
    O.setup_rnd2(n, p)
    rep = O.mcmc_run(off, idx, ncol, seed, maxRip=maxrip, tailcut=tailcut, tailcutRepair=True)
    K = base.res.iter
    if K >= 1:
        O.srand(1)
        O.setup_rnd2(n, p)
        prev = O.mcmc_run(off, idx, ncol, seed, maxRip=maxrip, tailcut=tailcut, sweep_limit=K - 1).colors
    else:
        prev = base.colors
    z = max(50, n // 2000) if tailcut else 0
    C, cviol, passes = _py_tail_cut(off, idx, base.colors, _viol_flags(off, idx, prev), ncol, z)
    assert rep.traj.tolist() == base.traj.tolist()
    assert rep.colors.tolist() == C.tolist()
    assert (rep.res.finalViol, rep.res.tailcutPasses) == (cviol, passes)
    assert passes > 0 or base.res.finalViol == 0


# ---- per-row / per-vertex pieces used by the full-size C3 check (tests/test_c3_full.py) ----------
def test_er_rows_equal_full_generator_rows():
    """oracle_er_rows (streams into the sampled rows' blocks only) == the rows of oracle_er_fast."""
    n, p, seed = 140000, 0.0002, 7   # 3 column blocks
    off, idx = O.er_fast(n, p, seed)
    rng = np.random.default_rng(3)
    rows = np.concatenate([[0, 1, 65535, 65536, 131071, 131072, n - 1], rng.integers(0, n, 60)]).astype(np.uint32)
    got = O.er_rows(n, p, seed, rows, nthreads=4)
    for v, g in zip(rows, got):
        assert g.tolist() == idx[off[v]:off[v + 1]].tolist(), v


def test_canonical_at_equals_sequential_draws():
    seq = np.zeros(3000, dtype=np.float32)
    O.lib().oracle_canonical_seq(5, 0, 3000, O._p(seq))
    pos = np.array([1, 2, 3, 999, 2000, 3000], dtype=np.uint64)
    assert O.canonical_at(5, pos).tolist() == seq[(pos - 1).astype(np.int64)].tolist()


@pytest.mark.parametrize("ncol,eps", [(16, 1e-8), (7, 1e-8), (12, 3e7)])
def test_vertex_update_equals_one_oracle_sweep(ncol, eps):
    """Every vertex of one full oracle sweep, recomputed from C_0, its neighbours and u_v = draw
    K0 + v + 1; CDF-overflow vertices (colour from rand()) are the only ones left out."""
    O.srand(1)
    off, idx = O.setup_rnd2(600, 0.05)
    n = len(off) - 1
    r1 = O.mcmc_run(off, idx, ncol, 3, epsilon=eps, sweep_limit=1)
    u = O.canonical_at(3, r1.res.initDraws + np.arange(n, dtype=np.uint64) + 1)
    events = 0
    for v in range(n):
        c, viol = O.vertex_update(ncol, eps, int(r1.init[v]), r1.init[idx[off[v]:off[v + 1]]], float(u[v]))
        if c is None:
            events += 1
        else:
            assert c == r1.colors[v], v
    assert events == r1.res.glibcDraws


def test_c3_expect_walk_pinned():
    """tests/c3_expect.py's vectorised all-full CDF walk (the full-size C3/C4 checks' expectation)
    equals the oracle's one-vertex update, at the default eps and at 1e-3."""
    import c3_expect as X

    X.pin_walk(32, 1e-8)
    X.pin_walk(32, 1e-3)
    X.pin_walk(16, 3.3e6, k=500)
