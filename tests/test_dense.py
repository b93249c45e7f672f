"""The dense-count sweep (mcmc_colorer_amd/csrc/dense_counts.h) against the oracle.

Each tiled context keeps, per row, the counts of the colours of its neighbours in a dense column
range S of its own rows, moved every sweep by the vertices of S that changed colour (or rebuilt);
a row whose dense mask is full is evaluated without scanning, the others scan their remaining
column blocks first. Bar: bit-exact -- colouring, per-sweep Cviol trajectory, iteration count and
glibc draws equal the oracle's restatement of ColoringMCMC_CPU::run (coloringMCMC_CPU.cpp:115-270).
MCMC_DENSE_ROWS shrinks S so that most rows scan past it and the update lists overflow (the
rebuild path); MCMC_DENSE=0 is the tiled scan sweep.
"""
import ctypes

import numpy as np
import pytest

import oracle_ref as O
from test_gpu_parity import assert_same, circulant, gpu_run, oracle_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def dense_stats(col):
    from mcmc_colorer_amd._lib import check, lib, u64ptr

    out = np.zeros(10, dtype=np.uint64)
    check(lib().mcmc_get_dense_stats(col._ctx, u64ptr(out)))
    return {"on": int(out[0]), "s0": int(out[1]), "s1": int(out[2]), "incremental": int(out[3]),
            "rebuilds": int(out[4]), "listed": int(out[5]), "open": int(out[6]), "max": int(out[7]),
            "changed": int(out[8]), "copies": int(out[9])}


CASES = [
    # n, p, nCol, seed, eps, taboo, maxRip, |S| (None: the library's choice)
    (3000, 0.02, 16, 31, 1e-8, 0, 60, None),
    (3000, 0.02, 16, 31, 1e-8, 0, 60, 40),
    (2000, 0.05, 100, 32, 1e-8, 2, 20, 300),
    (1500, 0.3, 5, 33, 3.3e6, 1, 15, 200),
    (2500, 0.1, 200, 34, 1e-8, 0, 10, 1000),
    (4000, 0.05, 32, 35, 1e-3, 0, 30, 2000),
    (4000, 0.05, 32, 36, 1e-3, 3, 30, None),
    (900, 0.08, 33, 3, 1e-8, 4, 40, 100),
    (1200, 0.05, 64, 4, 1e-8, 1, 40, 64),
    (3000, 0.01, 9, 10, 1e-8, 0, 250, 500),
    (64, 0.5, 2, 11, 1e-8, 0, 50, None),
    (1, 0.5, 1, 12, 1e-8, 0, 5, None),
]


@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip,srows", CASES)
def test_dense_matches_oracle(M, monkeypatch, n, p, ncol, seed, eps, taboo, maxrip, srows):
    if srows is not None:
        monkeypatch.setenv("MCMC_DENSE_ROWS", str(srows))
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=maxrip, taboo=taboo)
    assert_same(col, st, r)
    ds = dense_stats(col)
    assert ds["on"] == 1 and ds["s0"] == 0 and ds["s1"] == (min(srows, n) if srows else ds["s1"])
    if st.iter >= 1:
        assert ds["rebuilds"] >= 1   # the first accepted sweep built the counts
    if st.sweepsRun > 3 and eps <= 1e-8:
        assert ds["incremental"] >= 1
    if srows is not None and srows < n // 4 and n > 1000:
        assert ds["open"] > 0    # rows whose neighbours in S miss a colour scanned the other blocks


def test_dense_list_overflow_rebuilds(M, monkeypatch):
    """eps = 3.3e6 changes most colours every sweep: with |S| = 600 (rebuild threshold 75 listed
    vertices) the update lists outgrow the threshold and the counts are rebuilt, still exact."""
    monkeypatch.setenv("MCMC_DENSE_ROWS", "600")
    off, idx, nc, r = oracle_case(1500, 0.3, 7, 9, epsilon=3.3e6, tabooIteration=0, maxRip=25)
    col, st, _ = gpu_run(M, off, idx, nc, 9, 1500 * 1501 // 2, eps=3.3e6, maxRip=25)
    assert_same(col, st, r)
    ds = dense_stats(col)
    assert ds["max"] == 75 and ds["rebuilds"] > 1


@pytest.mark.parametrize("eps,cap", [(1e-3, 64), (1e-3, 8), (3.3e6, 64), (1e-8, 2)])
def test_dense_restore_lists(M, monkeypatch, eps, cap):
    """The evaluation writes only rows that change colour; the next sweep's buffer gets them back
    from the restore list -- applied by the commit (lists up to cap / 2), by the next launch's
    update tasks (longer ones), or by a full copy once the list overflows (MCMC_DENSE_CHG_CAP)."""
    monkeypatch.setenv("MCMC_DENSE_CHG_CAP", str(cap))
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 37, epsilon=eps, tabooIteration=1, maxRip=40)
    col, st, _ = gpu_run(M, off, idx, nc, 37, 3000 * 3001 // 2, eps=eps, maxRip=40, taboo=1)
    assert_same(col, st, r)
    ds = dense_stats(col)
    assert ds["on"] == 1 and ds["changed"] > 0
    if eps > 1.0:
        assert ds["copies"] > 0   # most colours change every sweep: the lists overflow


def test_dense_off_is_the_scan_sweep(M, monkeypatch):
    monkeypatch.setenv("MCMC_DENSE", "0")
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 31, epsilon=1e-8, maxRip=60)
    col, st, _ = gpu_run(M, off, idx, nc, 31, 3000 * 3001 // 2, maxRip=60)
    assert_same(col, st, r)
    assert dense_stats(col)["on"] == 0


def test_dense_needs_simple_symmetric_graph(M):
    """A directed ring (v -> v+1..v+4 only) and a CSR with a repeated arc: the counts could not be
    moved through the changed vertices' own rows, so the context keeps the scan sweep (exact)."""
    n, K = 3000, 4
    idx = ((np.arange(n)[:, None] + np.arange(1, K + 1)[None, :]) % n).astype(np.uint32)
    idx.sort(axis=1)
    off = np.arange(0, n * K + 1, K, dtype=np.uint64)
    O.srand(1)
    r = O.mcmc_run(off, idx.ravel(), 3, 5, maxRip=20)
    col, st, _ = gpu_run(M, off, idx.ravel(), 3, 5, 0, maxRip=20)
    assert_same(col, st, r)
    assert dense_stats(col)["on"] == 0
    off2, idx2 = circulant(2000, 3)
    rows = np.split(idx2, off2[1:-1].astype(np.int64))
    rows[5] = np.sort(np.append(rows[5], rows[5][0]))
    idx3 = np.concatenate(rows).astype(np.uint32)
    off3 = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.uint64)
    O.srand(1)
    r = O.mcmc_run(off3, idx3, 4, 6, maxRip=20)
    col, st, _ = gpu_run(M, off3, idx3, 4, 6, 0, maxRip=20)
    assert_same(col, st, r)
    assert dense_stats(col)["on"] == 0


@pytest.mark.parametrize("eps,srows", [(1e-8, None), (1e-3, None), (1e-8, 3000)])
def test_dense_generated_graph_matches_oracle(M, monkeypatch, eps, srows):
    """The counter-based G(n, p) (no CSR: rows come from the tiled layout), n = 150000, mean degree
    450, 32 colours: 8 sweeps equal to the oracle on the same graph."""
    if srows:
        monkeypatch.setenv("MCMC_DENSE_ROWS", str(srows))
    n, p, seed = 150000, 0.003, 8
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, 32, seed, epsilon=eps, maxRip=7, nthreads=8)
    g = M.Graph.er_fast(n, p, seed)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32, epsilon=eps, maxRip=7))
    st = col.run(0)
    assert_same(col, st, r)
    ds = dense_stats(col)
    assert ds["on"] == 1 and ds["incremental"] >= 6
    if srows:
        assert ds["open"] > 0


@pytest.mark.parametrize("world", [2, 3])
def test_dense_partitioned_loopback(M, monkeypatch, world):
    """Every rank keeps the counts of its own rows over a range of its own rows (|S| = 150 each:
    most rows scan past it); the native loopback driver's run equals the oracle's."""
    from mcmc_colorer_amd.distributed import LoopbackPartition, plan_rows

    monkeypatch.setenv("MCMC_DENSE_ROWS", "150")
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 41, epsilon=1e-3, maxRip=30)
    g = M.Graph.from_csr(off, idx)
    lp = LoopbackPartition(g, M.ColoringMCMCParams(nCol=nc, epsilon=1e-3, maxRip=30), 41, plan_rows(3000, world))
    st = lp.run(M.GlibcRand(1, 3000 * 3001 // 2))
    for k in range(world):
        assert lp.coloring(k).tolist() == r.colors.tolist(), k
        assert lp.trajectory(k).tolist() == r.traj.tolist(), k
        assert (st[k].iter, st[k].finalViol, st[k].glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    from mcmc_colorer_amd._lib import check, lib, u64ptr

    out = np.zeros(10, dtype=np.uint64)
    check(lib().mcmc_get_dense_stats(lp._ctx[world - 1], u64ptr(out)))
    b = plan_rows(3000, world)
    assert out[0] == 1 and out[1] == b[world - 1] and out[2] == b[world - 1] + 150 and out[3] > 0
    lp.close()


def dense_stats_v2(col):
    return col.dense_stats()


@pytest.mark.parametrize("n,p,ncol,seed,eps,maxrip,srows,solo_min", [
    (3000, 0.3, 16, 31, 1e-8, 60, None, 58),    # C2-like (every row full): every sweep but the rebuild solo
    (1500, 0.6, 48, 55, 1e-8, 40, None, 1),     # NW = 2
    (2000, 0.5, 100, 52, 1e-8, 30, None, 1),    # NW = 4, a few open rows (evaluated by the leader)
    (2500, 0.8, 200, 53, 1e-8, 20, None, 1),    # NW = 8
    (3000, 0.3, 16, 54, 1e-8, 30, 40, 0),       # |S| = 40: most rows open, full sweeps inside the launch
])
@pytest.mark.parametrize("bs", ["", "1024"])
def test_dense_persistent_matches_oracle(M, monkeypatch, n, p, ncol, seed, eps, maxrip, srows, solo_min, bs):
    """The persistent dense sweep (csrc/dense_sparse.h): the leader's solo sweeps evaluate only the
    candidate rows of the discrete-log window and the open rows; full sweeps (the count rebuild, open
    rows past the solo limit) run on the whole grid inside the same launch. Bit-exact vs the oracle,
    at the default 512-thread workgroups and at MCMC_DCM_BS=1024."""
    if bs:
        monkeypatch.setenv("MCMC_DCM_BS", bs)
    if srows is not None:
        monkeypatch.setenv("MCMC_DENSE_ROWS", str(srows))
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, maxRip=maxrip)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=maxrip)
    assert_same(col, st, r)
    ds = dense_stats_v2(col)
    assert ds["enabled"] and ds["persistent"] and ds["window_states"] > 0
    assert ds["solo_sweeps"] >= solo_min, ds


def test_dense_persistent_off_matches(M, monkeypatch):
    """MCMC_DENSE_MULTI=0: one dc_eval_kernel per sweep, the same results."""
    monkeypatch.setenv("MCMC_DENSE_MULTI", "0")
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 31, epsilon=1e-8, maxRip=60)
    col, st, _ = gpu_run(M, off, idx, nc, 31, 3000 * 3001 // 2, maxRip=60)
    assert_same(col, st, r)
    ds = dense_stats_v2(col)
    assert ds["enabled"] and not ds["persistent"] and ds["solo_sweeps"] == 0


@pytest.mark.parametrize("eps", [1e-8, 1e-3])
def test_dense_persistent_generated_graph(M, eps):
    """The generated G(n, p) (n = 150000, mean degree 450, 32 colours): 40 sweeps of the persistent
    launch (eps 1e-8: solo sweeps; 1e-3: the window is too large, the per-sweep kernel) equal the oracle."""
    n, p, seed = 150000, 0.003, 8
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, 32, seed, epsilon=eps, maxRip=39, nthreads=8)
    g = M.Graph.er_fast(n, p, seed)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32, epsilon=eps, maxRip=39))
    st = col.run(0)
    assert_same(col, st, r)
    ds = dense_stats_v2(col)
    assert (ds["window_states"] > 0) == (eps < 1e-6)   # eps 1e-3: no closed-form walk, no window
    if eps < 1e-6:
        assert ds["solo_sweeps"] >= 30, ds


@pytest.mark.parametrize("rb", ["0", "1"])
@pytest.mark.parametrize("n,p,ncol,seed,eps,srows", [(3000, 0.02, 16, 61, 1e-3, 1000), (2500, 0.1, 200, 62, 1e-3, 700),
                                                     (2000, 0.05, 33, 63, 3.3e6, None)])
def test_dense_rebuild_forms(M, monkeypatch, rb, n, p, ncol, seed, eps, srows):
    """The count rebuild two ways -- a wave per row (MCMC_DENSE_RB=0) and the streaming chunks of a
    row group (dense_counts.h dc_rebuild_chunk, the default) -- over list overflows (eps 3.3e6:
    every sweep rebuilds) and partial column blocks of S: the same colourings as the oracle."""
    monkeypatch.setenv("MCMC_DENSE_RB", rb)
    if srows:
        monkeypatch.setenv("MCMC_DENSE_ROWS", str(srows))
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, maxRip=20)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=20)
    assert_same(col, st, r)
    assert dense_stats_v2(col)["rebuilds"] >= 1


def _random_csr(n, deg, seed):
    """A simple symmetric random graph (sorted rows) built on the host."""
    rng = np.random.default_rng(seed)
    m = n * deg // 2
    u = rng.integers(0, n, m, dtype=np.int64)
    v = rng.integers(0, n, m, dtype=np.int64)
    keep = u != v
    a = np.minimum(u, v)[keep]
    b = np.maximum(u, v)[keep]
    key = np.unique(a * n + b)
    a, b = key // n, key % n
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    off = np.zeros(n + 1, dtype=np.uint64)
    np.add.at(off, src + 1, 1)
    return np.cumsum(off).astype(np.uint64), dst.astype(np.uint32)


def _expected_counts(off, idx, colors, ncol, s0, s1):
    n = len(off) - 1
    rows = np.repeat(np.arange(n), np.diff(off).astype(np.int64))
    ins = (idx >= s0) & (idx < s1)
    cnt = np.zeros((n, ncol), dtype=np.uint32)
    np.add.at(cnt, (rows[ins], colors[idx[ins]].astype(np.int64)), 1)
    return cnt


@pytest.mark.parametrize("rb", ["", "tid0", "1"])
@pytest.mark.parametrize("n,deg,ncol,bl,srows", [
    (5000, 200, 32, 9, None),     # S = every row: 9 whole 512-vertex blocks + a partial one
    (5000, 200, 32, 8, 2900),     # S ends inside block 11
    (6000, 120, 16, 6, 1000),     # 64-vertex blocks: 15 whole blocks, one partial
    (4000, 300, 5, 7, None),
    (3000, 90, 1, 8, None),       # one colour
    (3000, 60, 31, 4, 777),       # 16-vertex blocks (one 16-byte piece per slice)
    (7000, 40, 32, 16, None),     # the default 65536-vertex block: S inside block 0 (partial)
])
def test_dense_rebuild_counts_exact(M, monkeypatch, rb, n, deg, ncol, bl, srows):
    """The count rebuild's per-row counts and masks equal a host recount from the CSR and C_0 -- the
    lane rebuild (dense_counts.h dc_rebuild_lanes: bit-plane counts in registers, padding counted
    and subtracted inside S, every id tested in a partial block) by default, reading the
    tile-transposed copy of S's ids; with MCMC_DC_TID=0 ("tid0") reading the layout lane by lane; the
    chunk rebuild with MCMC_DENSE_RB=1 -- over whole and partial column blocks of S (MCMC_BLOCK_LOG2
    shrinks blocks)."""
    from mcmc_colorer_amd._lib import check, lib, u32ptr

    if rb == "tid0":
        monkeypatch.setenv("MCMC_DC_TID", "0")
    elif rb:
        monkeypatch.setenv("MCMC_DENSE_RB", rb)
    monkeypatch.setenv("MCMC_GATHER", "tiled")
    monkeypatch.setenv("MCMC_BLOCK_LOG2", str(bl))
    if srows:
        monkeypatch.setenv("MCMC_DENSE_ROWS", str(srows))
    off, idx = _random_csr(n, deg, n + deg)
    g = M.Graph.from_csr(off, idx)
    col = M.ColoringMCMC(g, M.GPURand(n, 7, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=3))
    col.init(0)
    c0 = col.coloring()
    col.step(1)   # the first sweep's update rebuilds the counts from C_0
    ds = dense_stats_v2(col)
    assert ds["enabled"] and ds["rebuilds"] >= 1
    assert ds["transposed_ids"] == (rb == "" and ncol <= 32), ds
    s0, s1 = ds["s0"], ds["s1"]
    cnt = np.zeros((n, ncol), dtype=np.uint32)
    nw = (ncol + 31) // 32
    msk = np.zeros((n, nw), dtype=np.uint32)
    check(lib().mcmc_get_dense_counts(col._ctx, 0, n, u32ptr(cnt), u32ptr(msk)))
    exp = _expected_counts(off, idx, c0, ncol, s0, s1)
    bad = np.nonzero((cnt != exp).any(axis=1))[0]
    assert len(bad) == 0, (len(bad), bad[:5], cnt[bad[:2]], exp[bad[:2]])
    expm = np.zeros((n, nw), dtype=np.uint32)
    for c in range(ncol):
        expm[:, c // 32] |= ((exp[:, c] != 0).astype(np.uint32) << np.uint32(c % 32))
    assert np.array_equal(msk, expm)


@pytest.mark.parametrize("poll", ["8", "64"])
def test_dense_poll_interval(M, monkeypatch, poll):
    """MCMC_DC_POLL: the persistent dense sweep's helpers sleep that many s_sleep(4) rounds between
    polls of the leader's flag (default 1). A scheduling knob only: the same results as the oracle."""
    monkeypatch.setenv("MCMC_DC_POLL", poll)
    off, idx, nc, r = oracle_case(3000, 0.3, 16, 31, epsilon=1e-8, maxRip=60)
    col, st, _ = gpu_run(M, off, idx, nc, 31, 3000 * 3001 // 2, maxRip=60)
    assert_same(col, st, r)
    ds = dense_stats_v2(col)
    assert ds["persistent"] and ds["solo_sweeps"] >= 50, ds
