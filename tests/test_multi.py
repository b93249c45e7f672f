"""The native multi-GPU path (csrc/multi.hip; VERDICT r1 "next" #5).

GPU (one MI355X): the partitioned colorer run inside one C call (mcmc_part_run) --
  * the loopback transport (every rank in this process on the one GPU, exchanged by device copies,
    otherwise the exact sequence of the RCCL path) for worlds 1..8: equal-row and arc-balanced
    plans, the wide sweep (nCol > 256), per-rank generated graphs, and sweeps whose overflow events
    outgrow a rank's footer (the spill exchange); the default delta exchange (changed vertices
    only), its overflow fallback (full ranges, then delta again), the full-range exchange
    (MCMC_EXCHANGE=p2p), and the corrected tail cut run rank by rank;
  * RCCL at world 1 through the C ABI: mcmc_comm_init_all and mcmc_comm_unique_id +
    mcmc_comm_init_rank, and the torch.distributed front end (NativePartitionedColoringMCMC);
  * the Python-exchanged protocol (HipRank in lock-step) on arc-balanced plans and spills.
All against the oracle, bit-exact. The N-rank RCCL exchange itself needs N GPUs: it is the same
driver with ncclSend/ncclRecv in place of the loopback copies; scaling stays unmeasured until the
round-end 8-GPU run.
CPU: the partition plans (host-only entry points).
"""
import numpy as np
import pytest

import oracle_ref as O
from test_gpu_parity import _lockstep, circulant, oracle_case


def skewed_csr(n, seed=3):
    """Hubs at low ids (degree falls with the id): equal-row plans balance it badly."""
    rng = np.random.default_rng(seed)
    E = set()
    for v in range(n):
        for _ in range(max(1, 40 * (n - v) // n)):
            w = int(rng.integers(0, n))
            if w != v:
                E.add((min(v, w), max(v, w)))
    rows = [[] for _ in range(n)]
    for a, b in E:
        rows[a].append(b)
        rows[b].append(a)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    return off, np.concatenate([np.sort(np.array(r, dtype=np.uint32)) for r in rows])


# ---- CPU: plans ---------------------------------------------------------------------------------
@pytest.mark.parametrize("n,world", [(1, 1), (100, 3), (1000, 8), (10_000_000, 8), (65, 2), (64, 64)])
def test_plan_rows(n, world):
    from mcmc_colorer_amd.distributed import plan_rows

    b = plan_rows(n, world).tolist()
    assert b[0] == 0 and b[-1] == n and b == sorted(b)
    assert all(x % 64 == 0 for x in b[1:-1] if x < n)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_plan_csr_balances_arcs(world):
    from mcmc_colorer_amd.distributed import plan_csr, plan_rows

    off, _ = skewed_csr(6000)
    b = plan_csr(off, world).tolist()
    assert b[0] == 0 and b[-1] == 6000 and b == sorted(b) and all(x % 64 == 0 for x in b[1:-1])
    deg = np.diff(off.astype(np.int64)) + 16
    load = [int(deg[b[r]:b[r + 1]].sum()) for r in range(world)]
    eq = plan_rows(6000, world).tolist()
    load_eq = [int(deg[eq[r]:eq[r + 1]].sum()) for r in range(world)]
    assert max(load) < 1.1 * sum(load) / world < max(load_eq)


# ---- GPU ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def loopback(M, off, idx, ncol, seed, bounds, draws, graphs=None, **kw):
    from mcmc_colorer_amd.distributed import LoopbackPartition

    g = graphs if graphs is not None else M.Graph.from_csr(off, idx)
    params = M.ColoringMCMCParams(nCol=ncol, **kw)
    lp = LoopbackPartition(g, params, seed, bounds)
    glibc = M.GlibcRand(1, draws)
    st = lp.run(glibc)
    return lp, st, glibc


def assert_native(lp, st, r, world):
    for k in range(world):
        assert lp.coloring(k).tolist() == r.colors.tolist(), k
        assert lp.trajectory(k).tolist() == r.traj.tolist(), k
        assert (st[k].iter, bool(st[k].maxIterReached), st[k].finalViol, st[k].glibcDraws) == (
            r.res.iter, bool(r.res.maxIterReached), r.res.finalViol, r.res.glibcDraws)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip", [(3000, 0.02, 16, 41, 1e-8, 0, 40),
                                                            (1500, 0.3, 5, 42, 3.3e6, 2, 12)])
def test_native_loopback_matches_oracle(M, world, n, p, ncol, seed, eps, taboo, maxrip):
    from mcmc_colorer_amd.distributed import plan_rows

    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    lp, st, glibc = loopback(M, off, idx, nc, seed, plan_rows(n, world), n * (n + 1) // 2, epsilon=eps,
                             tabooIteration=taboo, maxRip=maxrip)
    assert_native(lp, st, r, world)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_native_loopback_arc_balanced(M, world):
    from mcmc_colorer_amd.distributed import plan

    off, idx = skewed_csr(6000)
    O.srand(1)
    r = O.mcmc_run(off, idx, 14, 5, maxRip=30)
    g = M.Graph.from_csr(off, idx)
    b = plan(g, world, balance=True)
    assert b.tolist() != [min(k * ((6000 + world - 1) // world + 63) // 64 * 64, 6000) for k in range(world)] + [6000]
    lp, st, _ = loopback(M, off, idx, 14, 5, b, 0, graphs=g, maxRip=30)
    assert_native(lp, st, r, world)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_native_loopback_spill(M, world):
    """~20000 overflow events in sweep 0 (eps = 3e7, colour-0 vertices): every rank's list outgrows
    its 1020-event footer, the loop pauses, the full lists are all-gathered and committed."""
    off, idx = circulant(60000, 4)
    O.srand(1)
    r = O.mcmc_run(off, idx, 3, 21, epsilon=3e7, maxRip=4, nthreads=8)
    assert r.res.glibcDraws > 16384
    from mcmc_colorer_amd.distributed import plan_rows

    lp, st, _ = loopback(M, off, idx, 3, 21, plan_rows(60000, world), 0, epsilon=3e7, maxRip=4)
    assert_native(lp, st, r, world)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("inc", ["1", "2"])
@pytest.mark.parametrize("world", [2, 3])
def test_native_loopback_wide(M, monkeypatch, world, inc):
    """nCol > 256: the wide sweep's uint16 replicas over the native driver (configs[4]'s shape)."""
    import oracle_np as NP

    from mcmc_colorer_amd.distributed import plan_csr

    monkeypatch.setenv("MCMC_WIDE_INC", inc)   # 2: every sweep after a full one incremental
    off, idx = NP.rmat(11, 8, 0.5, 0.2, 0.2, 3)
    ncol = int(np.diff(off.astype(np.int64)).max())
    for nc, mr in ((ncol, 6), (max(257, ncol // 4), 12)):
        O.srand(1)
        r = O.mcmc_run(off, idx, nc, 1, maxRip=mr)
        lp, st, _ = loopback(M, off, idx, nc, 1, plan_csr(off, world), 0, maxRip=mr)
        assert_native(lp, st, r, world)
        # the delta exchange (changed vertices only) and the incremental violation counts, per rank
        import ctypes

        from mcmc_colorer_amd._lib import check, lib

        for k in range(world):
            xs = [ctypes.c_uint64() for _ in range(4)]
            check(lib().mcmc_part_exchange_stats(lp._ctx[k], *[ctypes.byref(x) for x in xs]))
            assert xs[0].value > 0, (k, [x.value for x in xs])
            ist = (ctypes.c_uint64 * 5)()
            check(lib().mcmc_get_wide_inc_stats(lp._ctx[k], ist))
            assert ist[0] == 1, (k, list(ist))
            if inc == "2" and r.res.iter >= 2:
                assert ist[1] > 0, (k, list(ist))
        lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("enter", ["-1", "1000000000"])
def test_native_loopback_wide_world1(M, monkeypatch, enter):
    """A world-1 partition of the wide sweep takes the one-GPU run's launches through the driver:
    its 8-step batches go through the persistent wide sweep (every batch, or from the second batch
    on, MCMC_WS_ENTER), equal to the oracle."""
    import oracle_np as NP

    from mcmc_colorer_amd.distributed import plan_csr

    monkeypatch.setenv("MCMC_WS_ENTER", enter)
    off, idx = NP.rmat(11, 8, 0.5, 0.2, 0.2, 3)
    ncol = int(np.diff(off.astype(np.int64)).max())
    for nc, mr in ((ncol, 6), (300, 30)):
        O.srand(1)
        r = O.mcmc_run(off, idx, nc, 1, maxRip=mr)
        lp, st, _ = loopback(M, off, idx, nc, 1, plan_csr(off, 1), 0, maxRip=mr)
        assert_native(lp, st, r, 1)
        import ctypes

        from mcmc_colorer_amd._lib import check, lib

        ws = (ctypes.c_uint64 * 30)()
        check(lib().mcmc_get_wide_solo_stats(lp._ctx[0], ws))
        assert ws[0] == 1, list(ws)[:10]
        if enter == "-1" or r.res.iter > 9:
            assert ws[2] > 0, list(ws)[:10]   # persistent sweeps run
        lp.close()


@pytest.mark.gpu
def test_native_loopback_er_fast_rows(M):
    """Each rank generates only its rows of an uneven plan (mcmc_graph_er_fast_rows)."""
    n, p, ncol, seed = 150000, 0.003, 16, 8
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=8, nthreads=8)
    b = np.array([0, 40000, 64000 * 2, n], dtype=np.uint32)
    graphs = [M.Graph.er_fast(n, p, seed, rows=(int(b[k]), int(b[k + 1]))) for k in range(3)]
    assert sum(gr.nEdges for gr in graphs) == len(idx)
    lp, st, _ = loopback(M, off, idx, ncol, seed, b, 0, graphs=graphs, maxRip=8)
    assert_native(lp, st, r, 3)
    lp.close()


@pytest.mark.gpu
def test_native_loopback_wide_er_fast_rows(M):
    """configs[3]'s shape at the reference's default nCol = maxDeg (> 256): every rank generates
    only its rows (mcmc_graph_er_fast_rows), the wide sweep materialises each rank's row-partial
    CSR from its layout, and the native driver's run equals the oracle's whole-graph run."""
    n, p, seed = 8000, 0.06, 5
    off, idx = O.er_fast(n, p, seed)
    ncol = O.max_deg(off)
    assert ncol > 256
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, maxRip=10)
    b = np.array([0, 2560, 5120, n], dtype=np.uint32)
    graphs = [M.Graph.er_fast(n, p, seed, rows=(int(b[k]), int(b[k + 1]))) for k in range(3)]
    lp, st, _ = loopback(M, off, idx, ncol, seed, b, 0, graphs=graphs, maxRip=10)
    assert_native(lp, st, r, 3)
    lp.close()


def _rccl_world1(M, off, idx, nc, seed, draws, use_id):
    import ctypes

    from mcmc_colorer_amd._lib import MCMCRunStats, check, lib, u32ptr

    comm = ctypes.c_void_p()
    if use_id:
        uid = (ctypes.c_uint8 * 128)()
        check(lib().mcmc_comm_unique_id(uid))
        check(lib().mcmc_comm_init_rank(uid, 1, 0, 0, ctypes.byref(comm)))
    else:
        devs = (ctypes.c_int * 1)(0)
        comms = (ctypes.c_void_p * 1)()
        check(lib().mcmc_comm_init_all(devs, 1, comms))
        comm = ctypes.c_void_p(comms[0])
    g = M.Graph.from_csr(off, idx)
    prm = M.ColoringMCMCParams(nCol=nc).to_c(seed)
    b = np.array([0, len(off) - 1], dtype=np.uint32)
    ctx = ctypes.c_void_p()
    check(lib().mcmc_part_create(g.handle, ctypes.byref(prm), 1, 0, u32ptr(b), comm, ctypes.byref(ctx)))
    w = M.GlibcRand(1, draws).window
    check(lib().mcmc_set_glibc_window(ctx, u32ptr(w)))
    check(lib().mcmc_init_coloring(ctx, None))
    st = (MCMCRunStats * 1)()
    check(lib().mcmc_part_run((ctypes.c_void_p * 1)(ctx.value), 1, 0, st))
    col = np.zeros(len(off) - 1, dtype=np.uint32)
    check(lib().mcmc_get_coloring(ctx, u32ptr(col)))
    k = ctypes.c_uint64()
    check(lib().mcmc_get_trajectory(ctx, None, 0, ctypes.byref(k)))
    traj = np.zeros(k.value, dtype=np.uint64)
    check(lib().mcmc_get_trajectory(ctx, traj.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), k.value,
                                    ctypes.byref(k)))
    lib().mcmc_destroy(ctx)
    lib().mcmc_comm_destroy(comm)
    return col, traj, st[0]


@pytest.mark.gpu
@pytest.mark.parametrize("use_id", [False, True])
def test_native_rccl_world1(M, use_id):
    """RCCL through the C ABI at world 1 (the footers' all-gather is the one collective)."""
    n, p, ncol, seed = 2000, 0.05, 12, 43
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=250)
    col, traj, st = _rccl_world1(M, off, idx, nc, seed, n * (n + 1) // 2, use_id)
    assert col.tolist() == r.colors.tolist() and traj.tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)


@pytest.mark.gpu
def test_native_driver_torch_frontend_world1(M):
    """NativePartitionedColoringMCMC: the unique id over torch.distributed (gloo), RCCL inside."""
    import os

    import torch.distributed as dist

    from mcmc_colorer_amd.distributed import NativePartitionedColoringMCMC, plan_rows

    n, p, ncol, seed = 1500, 0.05, 10, 44
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=250)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29519"
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        g = M.Graph.from_csr(off, idx)
        drv = NativePartitionedColoringMCMC(g, M.GPURand(n, seed, M.GlibcRand(1, n * (n + 1) // 2)),
                                            M.ColoringMCMCParams(nCol=nc), plan_rows(n, 1))
        st = drv.run(0)
        assert drv.coloring().tolist() == r.colors.tolist()
        assert drv.trajectory().tolist() == r.traj.tolist() and st.iter == r.res.iter
        drv.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_lockstep_arc_balanced_and_spill(M, world):
    """The Python-exchanged protocol (HipRank in lock-step) on an arc-balanced plan, then on a run
    whose sweep-0 lists outgrow the footers (spill exchange)."""
    from mcmc_colorer_amd.distributed import plan_csr

    off, idx = skewed_csr(6000)
    O.srand(1)
    r = O.mcmc_run(off, idx, 14, 5, maxRip=30)
    ranks = _lockstep(M, off, idx, 14, 5, world, maxRip=30, draws=0, bounds=plan_csr(off, world))
    for b in ranks:
        assert b.coloring().tolist() == r.colors.tolist() and b.trajectory().tolist() == r.traj.tolist()
    off, idx = circulant(60000, 4)
    O.srand(1)
    r = O.mcmc_run(off, idx, 3, 21, epsilon=3e7, maxRip=4, nthreads=8)
    ranks = _lockstep(M, off, idx, 3, 21, world, eps=3e7, maxRip=4, draws=0)
    assert ranks[0].spills >= 1
    for b in ranks:
        assert b.coloring().tolist() == r.colors.tolist() and b.trajectory().tolist() == r.traj.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["delta", "p2p"])
@pytest.mark.parametrize("world", [2, 5])
def test_native_loopback_exchange_modes(M, monkeypatch, exchange, world):
    """Both exchange forms give the oracle's run: delta (a rank sends the vertices whose colour
    changed; replicas kept equal off its rows) and p2p (whole row ranges every sweep)."""
    from mcmc_colorer_amd.distributed import plan_rows

    monkeypatch.setenv("MCMC_EXCHANGE", exchange)
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 41, maxRip=40)
    lp, st, _ = loopback(M, off, idx, nc, 41, plan_rows(3000, world), 3000 * 3001 // 2, maxRip=40)
    assert_native(lp, st, r, world)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_native_loopback_delta_overflow(M, world):
    """A sparse graph with few colours: thousands of vertices change colour per rank in the first
    sweeps, more than a delta slot holds (2047 pairs) -- those sweeps pause, travel as full row
    ranges, 16 full-mode steps follow, then delta mode resumes (after syncing the replicas); the
    run still equals the oracle's. Events (eps 0.05) ride along."""
    from mcmc_colorer_amd.distributed import plan_rows

    off, idx = circulant(60000, 4)
    O.srand(1)
    r = O.mcmc_run(off, idx, 5, 17, epsilon=0.05, maxRip=60, nthreads=8)
    lp, st, _ = loopback(M, off, idx, 5, 17, plan_rows(60000, world), 0, epsilon=0.05, maxRip=60)
    assert_native(lp, st, r, world)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("ncol,maxrip,tailcut", [(24, 250, True), (40, 3, False), (16, 6, False)])
def test_native_loopback_tailcut(M, world, ncol, maxrip, tailcut):
    """The corrected tail cut (coloringMCMC_CPU.cpp:272-311, k++) on a partitioned run: rank by rank
    in ascending order (each rank's repaired rows broadcast before the next rank's turn), recount
    summed over the ranks -- colouring, final Cviol and pass count equal the oracle's (the last
    case cannot repair: every pass up to the 1000-pass cap)."""
    from mcmc_colorer_amd.distributed import plan_rows

    n, p, seed = 2500, 0.02, 1
    off, idx, nc, r = oracle_case(n, p, ncol, seed, maxRip=maxrip, tailcut=tailcut, tailcutRepair=True)
    assert r.res.tailcutPasses >= 1
    lp, st, _ = loopback(M, off, idx, nc, seed, plan_rows(n, world), n * (n + 1) // 2, maxRip=maxrip,
                         tailcut=tailcut, tailcutRepair=1000)
    assert_native(lp, st, r, world)
    assert all(s.tailcutPasses == r.res.tailcutPasses for s in st)
    lp.close()


@pytest.mark.gpu
def test_native_loopback_tailcut_generated_rows(M):
    """Tail cut over per-rank generated layouts (no CSR: rows through each rank's tiled layout)."""
    n, p, ncol, seed = 140000, 0.0004, 120, 9
    off, idx = O.er_fast(n, p, seed)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, seed, tailcut=True, tailcutRepair=True, nthreads=8)
    assert r.res.tailcutPasses >= 1
    b = np.array([0, 50048, 90048, n], dtype=np.uint32)
    graphs = [M.Graph.er_fast(n, p, seed, rows=(int(b[k]), int(b[k + 1]))) for k in range(3)]
    lp, st, _ = loopback(M, off, idx, ncol, seed, b, 0, graphs=graphs, tailcut=True, tailcutRepair=1000)
    assert_native(lp, st, r, 3)
    assert all(s.tailcutPasses == r.res.tailcutPasses for s in st)
    lp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 8])
def test_part_bench_rank_stub(M, world):
    """mcmc_part_bench_rank (bench.py --rank-share): rank 0 of a world-K partition over its own
    generated rows, the exchange stubbed. Sweep 0 changes most colours, so its delta slot
    overflows and the driver runs full-mode steps after it; once the colouring settles (mean degree
    400, 32 colours: full masks) every step runs in delta mode (sweep + delta packing + footer +
    part_commit) and none overflows."""
    import ctypes

    from mcmc_colorer_amd._lib import MCMCRunStats, check, lib, u32ptr
    from mcmc_colorer_amd.distributed import plan_rows

    n, p, steps = 40000, 0.01, 12
    bounds = plan_rows(n, world)
    g = M.Graph.er_fast(n, p, 3, rows=(0, int(bounds[1])))
    prm = M.ColoringMCMCParams(nCol=32, maxRip=1000).to_c(3)
    ctx = ctypes.c_void_p()
    check(lib().mcmc_part_create(g.handle, ctypes.byref(prm), world, 0, u32ptr(bounds), None, ctypes.byref(ctx)))
    try:
        check(lib().mcmc_set_glibc_window(ctx, u32ptr(M.GlibcRand(1).window)))
        check(lib().mcmc_init_coloring(ctx, None))
        check(lib().mcmc_set_bench_mode(ctx, 1))
        st = MCMCRunStats()
        xs = [ctypes.c_uint64() for _ in range(4)]
        check(lib().mcmc_part_bench_rank(ctx, 24, ctypes.byref(st)))   # warm-up: overflow, full mode
        check(lib().mcmc_part_exchange_stats(ctx, *[ctypes.byref(x) for x in xs]))
        assert xs[0].value + xs[1].value == 24 and xs[2].value <= 1
        check(lib().mcmc_part_bench_rank(ctx, steps, ctypes.byref(st)))
        check(lib().mcmc_part_exchange_stats(ctx, *[ctypes.byref(x) for x in xs]))
        assert (xs[0].value, xs[1].value, xs[2].value) == (steps, 0, 0)
        assert st.loopMs > 0.0
    finally:
        lib().mcmc_destroy(ctx)
