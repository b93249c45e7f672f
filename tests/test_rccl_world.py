"""The native RCCL driver (csrc/multi.hip, mcmc_part_run over mcmc_comm_init_rank) at world 2 and 4,
every rank a process on the ONE GPU of the test box.

RCCL refuses two ranks of one communicator on the same device ("Duplicate GPU detected") unless the
ranks look like different hosts: each rank sets its own NCCL_HOSTID, so RCCL connects them through
its network transport (TCP sockets over the loopback interface) instead of xGMI P2P. That runs every
RCCL call of the data path at N > 1 -- the grouped ncclSend/ncclRecv of the row ranges (or the
in-place all-gather), the footer all-gather, the spill all-gather -- with exactly the message sizes
and buffer offsets of an 8-GPU run; what it does not exercise is the xGMI transport itself, whose
speed stays unmeasured until the driver's 8-GPU run. Results must equal the oracle bit for bit.
"""
import os
import socket

import numpy as np
import pytest

import oracle_ref as O

CASES = [
    # name, n, p, nCol, seed, eps, maxRip, plan, exchange
    ("er-rows-p2p", 3000, 0.02, 16, 41, 1e-8, 40, "rows", "p2p"),
    ("er-rows-allgather", 3000, 0.02, 16, 41, 1e-8, 40, "rows", "allgather"),
    ("skewed-arcs", 6000, 0.0, 14, 5, 1e-8, 30, "arcs", "p2p"),
    ("circulant-spill", 60000, 0.0, 3, 21, 3e7, 4, "rows", "p2p"),
    # the wide sweep (nCol = maxDeg > 256) with the delta exchange and incremental counts
    ("rmat-wide-delta", 2048, 0.0, 0, 1, 1e-8, 6, "arcs", "delta"),
    ("rmat-wide-quarter", 2048, 0.0, -4, 2, 1e-8, 10, "arcs", "delta"),
]


def _graph(kind, n, p):
    if kind.startswith("er"):
        O.srand(1)
        return O.setup_rnd2(n, p), n * (n + 1) // 2
    if kind.startswith("rmat"):
        import oracle_np as NP

        return NP.rmat(11, 8, 0.5, 0.2, 0.2, 3), 0
    if kind.startswith("circulant"):
        from test_gpu_parity import circulant

        return circulant(n, 4), 0
    from test_multi import skewed_csr

    return skewed_csr(n), 0


def _ncol(off, ncol):
    """0: maxDeg (main.cu:162's default); -k: maxDeg / k (at least 257: the wide sweep)."""
    if ncol > 0:
        return ncol
    md = int(np.diff(off.astype(np.int64)).max())
    return md if ncol == 0 else max(257, md // -ncol)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    # before anything initialises RCCL: a host id of its own per rank (see the module docstring)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"mcmc-test-rank{rank}",
                      NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", MCMC_EXCHANGE=case[8])
    import torch

    torch.cuda.init()
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd.distributed import NativePartitionedColoringMCMC, plan_csr, plan_rows

        name, n, p, ncol, seed, eps, maxrip, pl, _ = case
        (off, idx), draws = _graph(name, n, p)
        ncol = _ncol(off, ncol)
        bounds = plan_csr(off, world) if pl == "arcs" else plan_rows(n, world)
        g = M.Graph.from_csr(off, idx)
        rs = M.GPURand(n, seed, M.GlibcRand(1, draws))
        drv = NativePartitionedColoringMCMC(g, rs, M.ColoringMCMCParams(nCol=ncol, epsilon=eps, maxRip=maxrip),
                                            bounds, device=0)
        st = drv.run(0)
        q.put((rank, drv.coloring().tolist(), drv.trajectory().tolist(),
               (int(st.iter), int(st.finalViol), int(st.glibcDraws)), bounds.tolist()))
        drv.close()
        g.close()
    except Exception as e:   # report instead of hanging the parent on q.get
        q.put((rank, None, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_native_rccl_multiprocess_one_gpu(hip_lib, world, case):
    import torch.multiprocessing as mp

    name, n, p, ncol, seed, eps, maxrip, pl, ex = case
    (off, idx), draws = _graph(name, n, p)
    ncol = _ncol(off, ncol)
    O.srand(1)
    if draws:
        O.setup_rnd2(n, p)
    r = O.mcmc_run(off, idx, ncol, seed, epsilon=eps, maxRip=maxrip, nthreads=8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, world, port, case, q)) for k in range(world)]
    for pr in procs:
        pr.start()
    try:
        res = dict((x[0], x[1:]) for x in (q.get(timeout=240) for _ in range(world)))
    finally:
        for pr in procs:
            pr.join(timeout=60)
            if pr.is_alive():
                pr.kill()
    for k in range(world):
        colors, traj, stats, _ = res[k]
        assert colors is not None, (k, traj)
        assert colors == r.colors.tolist(), k
        assert traj == r.traj.tolist(), k
        assert stats == (r.res.iter, r.res.finalViol, r.res.glibcDraws), k
    for pr in procs:
        assert pr.exitcode == 0


def _c3_worker(rank, world, port, eps, e3_path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"mcmc-c3-rank{rank}",
                      NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    import ctypes

    import torch

    torch.cuda.init()
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import c3_expect as X
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd._lib import check, lib
        from mcmc_colorer_amd.distributed import NativePartitionedColoringMCMC, plan_rows

        b = plan_rows(X.N, world)
        g = M.Graph.er_fast(X.N, X.P, X.SEED, rows=(int(b[rank]), int(b[rank + 1])))
        drv = NativePartitionedColoringMCMC(g, M.GPURand(X.N, X.SEED, M.GlibcRand(1)),
                                            M.ColoringMCMCParams(nCol=X.NCOL, epsilon=eps), b, device=0)
        st = drv.run(0, max_sweeps=3)
        xs = [ctypes.c_uint64() for _ in range(4)]
        check(lib().mcmc_part_exchange_stats(drv._ctx, *[ctypes.byref(x) for x in xs]))
        bad = int((drv.coloring() != np.load(e3_path)).sum())
        q.put((rank, bad, drv.trajectory().tolist(), int(st.glibcDraws), [x.value for x in xs]))
        drv.close()
        g.close()
    except Exception as e:
        q.put((rank, None, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("eps", [1e-8, 1e-3])
def test_native_rccl_c3_world2(hip_lib, tmp_path, eps):
    """configs[3]'s data path over real RCCL at real sizes: the C3 graph (1e7 rows, 1e11 arcs) over 2
    processes on the one GPU (socket transport), each generating its 5e6 rows; 3 sweeps; every rank's
    replica equals C_3 of tests/c3_expect.py on EVERY vertex. eps 1e-8: delta slots only; eps 1e-3:
    ~150 000 changes per rank and sweep overflow the slots and the rows travel in full."""
    import torch.multiprocessing as mp

    import c3_expect as X

    E, k0, evs = X.expected(3, eps)
    e3 = tmp_path / "e3.npy"
    np.save(e3, E[3])
    del E
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c3_worker, args=(k, 2, port, eps, str(e3), q)) for k in range(2)]
    for pr in procs:
        pr.start()
    try:
        res = dict((x[0], x[1:]) for x in (q.get(timeout=900) for _ in range(2)))
    finally:
        for pr in procs:
            pr.join(timeout=120)
            if pr.is_alive():
                pr.kill()
    for k in range(2):
        bad, traj, draws, xs = res[k]
        assert bad == 0, (k, traj)
        assert traj == [X.N] * 3, k
        assert draws == sum(evs), k
        print(f"\nrank {k}: exchange stats (delta steps, full steps, overflows, bytes sent) {xs}", flush=True)
        if eps == 1e-8:
            assert xs[0] == 3 and xs[2] == 0, xs
        else:
            assert xs[2] >= 1, xs
    for pr in procs:
        assert pr.exitcode == 0
