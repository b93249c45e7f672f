"""GPU parity: the HIP sweep (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact -- final colouring, per-sweep conflict trajectory (the reference's
"C violations" log, coloringMCMC_CPU.cpp:152), iteration count, max-iteration flag and the
number of glibc rand() draws taken by CDF-overflow events must all be identical.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def gpu_run(M, off, idx, ncol, seed, draws_before, *, eps=1e-8, maxRip=250, taboo=0, tailcut=False,
            iteration=0, glibc=None):
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, epsilon=eps, maxRip=maxRip, tabooIteration=taboo, tailcut=tailcut)
    rs = M.GPURand(g.nNodes, seed, glibc if glibc is not None else M.GlibcRand(1, draws_before))
    col = M.ColoringMCMC(g, rs, params)
    st = col.run(iteration)
    return col, st, rs


def set_gather(monkeypatch, spec):
    """MCMC_GATHER[:MCMC_BLOCK_LOG2[:MCMC_SUB_LOG2[:MCMC_GROUP_ROWS[:MCMC_TILE_STREAM]]]] test knobs
    (an empty field keeps the library's choice)."""
    parts = spec.split(":")
    monkeypatch.setenv("MCMC_GATHER", parts[0])
    for key, v in zip(("MCMC_BLOCK_LOG2", "MCMC_SUB_LOG2", "MCMC_GROUP_ROWS", "MCMC_TILE_STREAM"), parts[1:]):
        if v:
            monkeypatch.setenv(key, v)


def oracle_case(n, p, ncol, seed, **kw):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    nc = ncol or O.max_deg(off)
    r = O.mcmc_run(off, idx, nc, seed, **kw)
    return off, idx, nc, r


def _first_diff(got, want):
    """A short message for two unequal sequences (pytest's list diff takes minutes on 1e3+ entries)."""
    got, want = np.asarray(got), np.asarray(want)
    if got.shape != want.shape:
        return f"lengths {got.shape} vs {want.shape}"
    bad = np.flatnonzero(got != want)
    return f"{bad.size} of {got.size} differ, first at {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


def assert_same(col, st, r):
    got = col.coloring()
    assert np.array_equal(got, r.colors), "colours: " + _first_diff(got, r.colors)
    traj = col.trajectory()
    assert np.array_equal(traj, r.traj), "trajectory: " + _first_diff(traj, r.traj)
    assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws, st.initDraws) == (
        r.res.iter, bool(r.res.maxIterReached), r.res.finalViol, r.res.glibcDraws, r.res.initDraws)


def test_c1_graph_generated_on_gpu_is_exact(M):
    """configs[0]: --simulate 0.1 -n 1000 -- the GPU setupRnd2 replay equals the reference's CSR."""
    O.srand(1)
    off, idx = O.setup_rnd2(1000, 0.1)
    rng = M.GlibcRand(1)
    g = M.Graph.simulate(1000, 0.1, rng)
    s = g.getStruct()
    assert np.array_equal(s.cumulDegs, off) and np.array_equal(s.neighs, idx)
    assert g.getMaxNodeDeg() == O.max_deg(off)
    # the stream advanced by n(n+1)/2 draws
    assert np.array_equal(rng.window, M.GlibcRand(1, 1000 * 1001 // 2).window)


@pytest.mark.parametrize("n,p", [(1, 0.5), (2, 1.0), (37, 0.5), (400, 0.03), (2500, 0.01), (3000, 0.9)])
def test_gpu_generator_exact(M, n, p):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    g = M.Graph.simulate(n, p, M.GlibcRand(1))
    s = g.getStruct()
    assert np.array_equal(s.cumulDegs, off) and np.array_equal(s.neighs, idx)


SMALL = json.loads((GOLDEN / "small.json").read_text())


@pytest.mark.parametrize("name", sorted(SMALL))
def test_gpu_matches_golden(M, name):
    d = SMALL[name]
    rng = M.GlibcRand(1)
    g = M.Graph.simulate(d["n"], d["prob"], rng)
    s = g.getStruct()
    assert sha(s.cumulDegs.astype(np.uint64)) == d["row_off_sha256"]
    assert sha(s.neighs.astype(np.uint32)) == d["col_idx_sha256"]
    params = M.ColoringMCMCParams(nCol=d["nCol"], epsilon=d["epsilon"], maxRip=d["maxRip"],
                                  tabooIteration=d["tabooIteration"], tailcut=d["tailcut"])
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, d["seed"], rng), params)
    st = col.run(0)
    assert col.coloring().tolist() == d["colors"]
    assert col.trajectory().tolist() == d["traj"]
    assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws) == (
        d["iter"], d["maxIterReached"], d["finalViol"], d["glibcDraws"])


GRID = [
    # n, p, nCol, seed, eps, taboo, maxRip, tailcut
    (500, 0.05, 0, 1, 1e-8, 0, 250, False),
    (700, 0.1, 16, 2, 1e-8, 0, 30, False),
    (900, 0.08, 31, 3, 1e-8, 0, 40, False),
    (900, 0.08, 32, 3, 1e-8, 4, 40, False),
    (900, 0.08, 33, 3, 1e-8, 0, 40, False),
    (1200, 0.05, 64, 4, 1e-8, 1, 40, False),
    (1200, 0.05, 65, 4, 1e-8, 0, 40, False),
    (1500, 0.1, 128, 5, 1e-8, 0, 20, False),
    (1500, 0.15, 129, 6, 1e-8, 2, 20, False),
    (2000, 0.12, 256, 7, 1e-8, 0, 10, False),
    (800, 0.3, 3, 8, 3.3e6, 0, 25, False),
    (800, 0.3, 7, 9, 3.3e6, 3, 25, False),
    (3000, 0.01, 9, 10, 1e-8, 0, 250, True),
    (64, 0.5, 2, 11, 1e-8, 0, 50, False),
    (1, 0.5, 1, 12, 1e-8, 0, 5, False),
    (100, 0.0, 4, 13, 1e-8, 0, 5, False),
]


@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip,tailcut", GRID)
def test_gpu_matches_oracle_grid(M, n, p, ncol, seed, eps, taboo, maxrip, tailcut):
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip,
                                  tailcut=tailcut)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=maxrip, taboo=taboo,
                         tailcut=tailcut)
    assert_same(col, st, r)


def circulant(n, K):
    """Ring lattice: v ~ v +- 1..K (sorted rows), a CSR the tests can build without setupRnd2."""
    nb = sorted([d for k in range(1, K + 1) for d in (k, -k)])
    idx = ((np.arange(n)[:, None] + np.array(nb)[None, :]) % n).astype(np.uint32)
    idx.sort(axis=1)
    off = np.arange(0, n * len(nb) + 1, len(nb), dtype=np.uint64)
    return off, idx.ravel()


@pytest.mark.parametrize("gather", ["lds", "global", "blocked:17", "blocked:8", "blocked:6", "tiled",
                                    "tiled:8", "tiled:6:0:7", "tiled:7:3:1", "tiled:4:6:33", "tiled:9:2:100",
                                    "tiled::::0", "tiled:8:1:50:0", "tiled:6:2:7:0", "tiled:10:5:1:0"])
@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip", [(3000, 0.02, 16, 31, 1e-8, 0, 60),
                                                            (2000, 0.05, 100, 32, 1e-8, 2, 20),
                                                            (1500, 0.3, 5, 33, 3.3e6, 1, 15),
                                                            (2500, 0.1, 200, 34, 1e-8, 0, 10)])
def test_all_gather_variants(M, monkeypatch, gather, n, p, ncol, seed, eps, taboo, maxrip):
    """LDS-staged, L2-gather, column-blocked (down to 64-vertex blocks, i.e. dozens of column
    blocks and many chunks) and tiled sweeps (spec tiled:block_log2:lanes_log2:group_rows:stream --
    16-vertex blocks, 1..64 lanes per row segment, odd group sizes; streamed slices by default,
    stream=0 the LDS-resident replica) give the same bit-exact results."""
    set_gather(monkeypatch, gather)
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=maxrip, taboo=taboo)
    assert_same(col, st, r)


def test_many_events_global_sort_path(M):
    """~20000 CDF-overflow events in ONE sweep (epsilon = 3e7 makes the fp32 CDF of a vertex whose
    colour is 0 cancel to 0): exercises the commit's in-global-memory sort and a long ordered
    glibc replay."""
    off, idx = circulant(60000, 4)
    O.srand(1)
    r = O.mcmc_run(off, idx, 3, 21, epsilon=3e7, maxRip=0, nthreads=8)
    assert r.res.glibcDraws > 16384          # all in the single sweep
    col, st, _ = gpu_run(M, off, idx, 3, 21, 0, eps=3e7, maxRip=0)
    assert_same(col, st, r)
    O.srand(1)
    r = O.mcmc_run(off, idx, 3, 22, epsilon=3e7, maxRip=4, nthreads=8)
    col, st, _ = gpu_run(M, off, idx, 3, 22, 0, eps=3e7, maxRip=4)
    assert_same(col, st, r)


def test_repetitions_share_glibc_stream(M):
    """--repet: seed + i per repetition (main.cu:171), one glibc stream across them."""
    n, p, ncol = 600, 0.3, 7
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    refs = [O.mcmc_run(off, idx, ncol, 100 + i, epsilon=3.3e6, maxRip=8) for i in range(3)]
    assert sum(r.res.glibcDraws for r in refs) > 0
    g = M.Graph.from_csr(off, idx)
    rs = M.GPURand(n, 100, M.GlibcRand(1, n * (n + 1) // 2))
    col = M.ColoringMCMC(g, rs, M.ColoringMCMCParams(nCol=ncol, epsilon=3.3e6, maxRip=8))
    for i, r in enumerate(refs):
        st = col.run(i)
        assert_same(col, st, r)


def test_early_stop_max_sweeps(M):
    off, idx, nc, r = oracle_case(2000, 0.05, 12, 3, maxRip=250, sweep_limit=5)
    g = M.Graph.from_csr(off, idx)
    c2 = M.ColoringMCMC(g, M.GPURand(2000, 3, M.GlibcRand(1, 2000 * 2001 // 2)), M.ColoringMCMCParams(nCol=nc))
    st2 = c2.run(0, max_sweeps=5)
    assert st2.iter == 5 and c2.coloring().tolist() == r.colors.tolist()
    assert c2.trajectory().tolist() == r.traj.tolist()[:5]


def test_c2_full_run_matches_golden(M):
    """configs[1]: --mcmcgpu --simulate 0.01 -n 100000, 16 colours: exact graph (5e9 glibc draws on
    the GPU), 251 sweeps, trajectory and final colouring identical to the oracle's."""
    d = json.loads((GOLDEN / "c2.json").read_text())
    rng = M.GlibcRand(1)
    g = M.Graph.simulate(d["n"], d["prob"], rng)
    s = g.getStruct()
    assert g.nEdges == d["m"] and g.getMaxNodeDeg() == d["maxDeg"]
    assert sha(s.cumulDegs.astype(np.uint64)) == d["row_off_sha256"]
    assert sha(s.neighs.astype(np.uint32)) == d["col_idx_sha256"]
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, d["seed"], rng), M.ColoringMCMCParams(nCol=d["nCol"]))
    st = col.run(0)
    assert col.trajectory().tolist() == d["traj"]
    assert sha(col.coloring()) == d["colors_sha256"]
    assert (st.iter, bool(st.maxIterReached), st.finalViol, st.glibcDraws) == (
        d["iter"], d["maxIterReached"], d["finalViol"], d["glibcDraws"])


def _lockstep_exchange(ranks, t):
    """The exchange of sweep t between HipRank backends on one GPU: every rank's row range and
    footer slot copied into every other rank's buffers."""
    from mcmc_colorer_amd.distributed import FOOTER_WORDS

    bufs = [b.exchange_buffers(t) for b in ranks]
    for q, (Cq, _, Fq, _) in enumerate(bufs):
        for r, (Cr, rngs, Fr, _) in enumerate(bufs):
            if r != q:
                lo, hi = rngs[r]
                Cq[lo:hi].copy_(Cr[lo:hi])
                Fq[r * FOOTER_WORDS:(r + 1) * FOOTER_WORDS].copy_(Fr[r * FOOTER_WORDS:(r + 1) * FOOTER_WORDS])


def _lockstep_drive(ranks, limit):
    """Sweep / exchange / commit in lock-step until done, with the spill exchange (the full sorted
    lists, all-gathered with a common stride) when a sweep pauses."""
    import torch

    t, spills = 0, 0
    while t < limit:
        for b in ranks:
            b.sweep()
        _lockstep_exchange(ranks, t)
        for b in ranks:
            b.commit()
        t += 1
        done, tdev, err = ranks[0].state()
        assert not (err & 1)
        if err & 2:
            stride = int(max(1, ranks[0].spill_counts().max()))
            gathered = torch.cat([b.spill_local(stride) for b in ranks])
            for b in ranks:
                b.spill_commit(gathered, stride)
            spills += 1
            done, t, err = ranks[0].state()
        if done:
            break
    return spills


def _lockstep(M, off, idx, ncol, seed, world, eps=1e-8, taboo=0, maxRip=250, draws=None, bounds=None):
    """`world` HipRank backends on one GPU, exchanged by tensor copies in lock-step: the device
    side of the partitioned protocol (replicas in vertex order, per-rank row ranges and footer
    slots exchanged, rank-ordered replay, spill exchange)."""
    import torch

    from mcmc_colorer_amd.distributed import HipRank

    n = len(off) - 1
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, epsilon=eps, maxRip=maxRip, tabooIteration=taboo)
    ranks = [HipRank(g, params, seed, world, r, torch.device("cuda", 0), bounds=bounds) for r in range(world)]
    for b in ranks:
        b.init(seed, M.GlibcRand(1, n * (n + 1) // 2 if draws is None else draws))
    ranks_spills = _lockstep_drive(ranks, maxRip + 2)
    for b in ranks:
        b.spills = ranks_spills
    return ranks


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip", [(3000, 0.02, 16, 41, 1e-8, 0, 40),
                                                            (1500, 0.3, 5, 42, 3.3e6, 2, 12)])
def test_partitioned_lockstep(M, world, n, p, ncol, seed, eps, taboo, maxrip):
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    ranks = _lockstep(M, off, idx, nc, seed, world, eps=eps, taboo=taboo, maxRip=maxrip)
    for b in ranks:
        assert b.state()[0]
        assert b.coloring().tolist() == r.colors.tolist()
        assert b.trajectory().tolist() == r.traj.tolist()


def test_partitioned_driver_nccl_world1(M):
    """The real driver over torch.distributed 'nccl' (RCCL), world_size 1."""
    import os

    import torch
    import torch.distributed as dist

    from mcmc_colorer_amd.distributed import PartitionedColoringMCMC

    n, p, ncol, seed = 2000, 0.05, 12, 43
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=250)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        g = M.Graph.from_csr(off, idx)
        drv = PartitionedColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1, n * (n + 1) // 2)),
                                      M.ColoringMCMCParams(nCol=nc))
        drv.run(0)
        assert drv.coloring().tolist() == r.colors.tolist()
        assert drv.trajectory().tolist() == r.traj.tolist()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("gather", ["blocked:7", "tiled:7", "tiled:7:::0"])
def test_blocked_unsorted_upload(M, monkeypatch, gather):
    """Uploaded rows in arbitrary order (as --graph produces) are sorted once for the blocked and
    tiled variants; the result is unchanged (the sweep is order-independent)."""
    set_gather(monkeypatch, gather)
    n, p, ncol, seed = 2000, 0.05, 9, 51
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=40)
    rnd = np.random.default_rng(0)
    shuf = idx.copy()
    for v in range(n):
        seg = shuf[off[v]:off[v + 1]]
        rnd.shuffle(seg)
    col, st, _ = gpu_run(M, off, shuf, nc, seed, n * (n + 1) // 2, maxRip=40)
    assert_same(col, st, r)


@pytest.mark.parametrize("gather", ["blocked:15", "blocked:12", "tiled", "tiled:12", "tiled::::0", "tiled:14:2::0"])
def test_c2_blocked_matches_golden(M, monkeypatch, gather):
    """configs[1] full run through the column-blocked kernel (4 and 25 column blocks) and the tiled
    kernel (streamed slices with 2 and 25 column blocks; LDS-resident replica with 2 and 7)."""
    set_gather(monkeypatch, gather)
    d = json.loads((GOLDEN / "c2.json").read_text())
    rng = M.GlibcRand(1)
    g = M.Graph.simulate(d["n"], d["prob"], rng)
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, d["seed"], rng), M.ColoringMCMCParams(nCol=d["nCol"]))
    st = col.run(0)
    assert col.trajectory().tolist() == d["traj"]
    assert sha(col.coloring()) == d["colors_sha256"]


@pytest.mark.parametrize("world", [2, 5])
@pytest.mark.parametrize("gather", ["tiled:9", "tiled:9:::0", "tiled:6:1:5:0"])
def test_partitioned_lockstep_tiled(M, monkeypatch, world, gather):
    set_gather(monkeypatch, gather)
    off, idx, nc, r = oracle_case(3000, 0.03, 20, 61, maxRip=30)
    ranks = _lockstep(M, off, idx, nc, 61, world, maxRip=30)
    for b in ranks:
        assert b.coloring().tolist() == r.colors.tolist()
        assert b.trajectory().tolist() == r.traj.tolist()


def test_refstruct_baseline_runs(M):
    """The refstruct timing baseline (reference per-sweep structure) runs and counts conflicts."""
    import ctypes

    from mcmc_colorer_amd._lib import check, lib

    O.srand(1)
    off, idx = O.setup_rnd2(2000, 0.05)
    g = M.Graph.from_csr(off, idx)
    ms, conf = ctypes.c_double(), ctypes.c_uint64()
    check(lib().mcmc_refstruct_bench(g.handle, 8, 3, 1, ctypes.byref(ms), ctypes.byref(conf)))
    assert ms.value > 0
    # monochromatic edges of a colouring with 8 colours on ~50 000 edges: some, not all
    assert 0 < conf.value < len(idx) // 2


# ---- the build's counter-based G(n, p) (C3/C4 generator), generated into the tiled layout --------
@pytest.mark.parametrize("n,p,seed", [(1000, 0.05, 7), (70000, 0.0005, 3), (131073, 0.0002, 11), (300, 1.0, 1),
                                      (500, 0.0, 1), (2, 0.5, 9), (200000, 0.001, 5)])
def test_er_fast_generator_matches_restatement(M, n, p, seed):
    """GPU generator (straight into the tiled layout, CSR rebuilt by download) == oracle_er_fast."""
    off, idx = O.er_fast(n, p, seed)
    g = M.Graph.er_fast(n, p, seed)
    assert g.nEdges == len(idx) and g.maxDeg == O.max_deg(off)
    s = g.getStruct()
    assert np.array_equal(s.cumulDegs, off) and np.array_equal(s.neighs, idx)


@pytest.mark.parametrize("n,p,ncol,seed,stream", [(130000, 0.004, 16, 5, "0"), (200000, 0.003, 32, 6, "1"),
                                                  (130000, 0.004, 16, 7, "1")])
def test_er_fast_sweep_matches_oracle(M, monkeypatch, n, p, ncol, seed, stream):
    """MCMC on a generated graph (resident replica; streamed slices) == the oracle on the restated CSR."""
    monkeypatch.setenv("MCMC_TILE_STREAM", stream)
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=12, nthreads=8)
    g = M.Graph.er_fast(n, p, seed)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=12))
    st = col.run(0)
    assert_same(col, st, r)


@pytest.mark.parametrize("world", [2, 3])
def test_er_fast_part_lockstep(M, world):
    """Each rank generates only its rows (mcmc_graph_er_fast_part); the partitioned protocol over
    those per-rank graphs == the oracle on the whole restated graph."""
    import torch

    from mcmc_colorer_amd.distributed import HipRank

    n, p, ncol, seed, maxrip = 150000, 0.003, 16, 8, 10
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=maxrip, nthreads=8)
    params = M.ColoringMCMCParams(nCol=ncol, maxRip=maxrip)
    graphs = [M.Graph.er_fast(n, p, seed, world=world, rank=k) for k in range(world)]
    assert sum(gr.nEdges for gr in graphs) == len(idx)
    ranks = [HipRank(graphs[k], params, seed, world, k, torch.device("cuda", 0)) for k in range(world)]
    for b in ranks:
        b.init(seed, M.GlibcRand(1))
    _lockstep_drive(ranks, maxrip + 2)
    for b in ranks:
        assert b.coloring().tolist() == r.colors.tolist()
        assert b.trajectory().tolist() == r.traj.tolist()


def test_gpu_generator_exact_at_1e6(M):
    """the reference's exact setupRnd2 graph at n = 1e6 (5e11 glibc draws,
    far beyond a CPU replay). Size-independent checks: the stream advances n(n+1)/2 draws; the CSR
    is symmetric, loop-free and sorted; and sampled rows' upper neighbours equal the REAL glibc
    rand() draws (the oracle's libc, positioned at row v's first draw v*n - v(v-1)/2 by the
    jump-ahead that test_capi pins against glibc), thresholded as graphCPU.cpp:308 does."""
    n, p = 1_000_000, 1e-4
    rng = M.GlibcRand(1)
    g = M.Graph.simulate(n, p, rng)
    assert np.array_equal(rng.window, M.GlibcRand(1, n * (n + 1) // 2).window)
    s = g.getStruct()
    off, idx = s.cumulDegs.astype(np.int64), s.neighs.astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
    assert not np.any(rows == idx)
    fwd = rows * n + idx
    assert np.all(np.diff(fwd) > 0)                       # rows ascending, no duplicates
    assert np.array_equal(np.sort(idx * n + rows), fwd)   # symmetric
    assert abs(len(idx) - p * n * (n - 1)) < 6 * np.sqrt(p * n * n)
    pf = float(np.float32(p))
    for v in (0, 1, 4567, 500000, 999_998):
        k0 = v * n - v * (v - 1) // 2                     # draws before row v of the upper triangle
        O.set_glibc_window(M.GlibcRand(1, k0).window)
        draws = np.asarray(O.rand(n - v), dtype=np.float64)
        upper = v + np.nonzero(draws / 2147483647.0 < pf)[0]
        upper = upper[upper > v]                          # the diagonal draw is consumed, then cleared
        got = idx[off[v]:off[v + 1]]
        assert np.array_equal(got[got > v], upper), v


TAILCUT = [
    # n, p, nCol, seed, maxRip, tailcut
    (1000, 0.1, 0, 1, 250, True),     # configs[0] with --tailcut: one pass repairs the rest
    (2500, 0.02, 24, 1, 250, True),   # nCol > 16: histogram order by libstdc++'s introsort
    (600, 0.03, 10, 1, 250, True),    # the repair oscillates: runs to the 1000-pass bound
    (500, 0.02, 7, 1, 250, True),
    (250, 0.2, 5, 3, 30, False),      # too few colours: loop cap, then 1000 passes
    (200, 0.01, 16, 4, 250, True),    # initial colouring within z: no accepted sweep
    (300, 0.1, 40, 5, 3, False),      # z = 0: identity colour order
]


@pytest.mark.parametrize("gather", ["tiled", "tiled::::0", "tiled:6:2:7", "lds", "global", "blocked:8"])
@pytest.mark.parametrize("n,p,ncol,seed,maxrip,tailcut", TAILCUT)
def test_tailcut_repair_matches_oracle(M, monkeypatch, gather, n, p, ncol, seed, maxrip, tailcut):
    """Corrected tail cut (coloringMCMC_CPU.cpp:272-311, k++) after the device loop == the oracle's
    tail_cut(): colouring, repaired Cviol and pass count; the trajectory stays the loop's. Every
    sweep kernel keeps the violation flags the first pass needs (those of the colouring before the
    last accepted sweep)."""
    set_gather(monkeypatch, gather)
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=maxrip, tailcut=tailcut, tailcutRepair=True)
    g = M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=nc, maxRip=maxrip, tailcut=tailcut, tailcutRepair=1000)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1, n * (n + 1) // 2)), params)
    st = col.run(0)
    assert_same(col, st, r)
    assert st.tailcutPasses == r.res.tailcutPasses


def test_tailcut_repair_generated_graph(M):
    """Tail cut on a generated graph (no CSR on the device: rows read through the tiled layout,
    several 2^16-column blocks) == the oracle on the restated CSR."""
    n, p, ncol, seed = 140000, 0.0004, 120, 9
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, tailcut=True, tailcutRepair=True, nthreads=8)
    assert r.res.tailcutPasses >= 1
    g = M.Graph.er_fast(n, p, seed)
    params = M.ColoringMCMCParams(nCol=ncol, tailcut=True, tailcutRepair=1000)
    col = M.ColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1)), params)
    st = col.run(0)
    assert_same(col, st, r)
    assert st.tailcutPasses == r.res.tailcutPasses


@pytest.mark.parametrize("drain,rows,stream", [("0", "200", "1"), ("256", "200", "1"), ("256", "64", "0"),
                                               ("48", "300", "1")])
def test_early_exit_drain_matches_oracle(M, monkeypatch, drain, rows, stream):
    """The early-exit scan (a row stops once its mask holds every colour; a group skips its
    remaining blocks once all rows are full) and its drain (a group's last few open rows finish
    every remaining block from the global layout and replica): 5 column blocks, small groups so
    every group drains after its first block; the full scan and the oracle agree bit for bit."""
    n, p, ncol, seed = 300000, 0.0006, 16, 12
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=5, nthreads=8)
    monkeypatch.setenv("MCMC_DRAIN_ROWS", drain)
    monkeypatch.setenv("MCMC_GROUP_ROWS", rows)
    monkeypatch.setenv("MCMC_TILE_STREAM", stream)
    col, st, _ = gpu_run(M, off, idx, ncol, seed, 0, maxRip=5)
    assert_same(col, st, r)
    monkeypatch.setenv("MCMC_FULL_SCAN", "1")
    col2, st2, _ = gpu_run(M, off, idx, ncol, seed, 0, maxRip=5)
    assert_same(col2, st2, r)

