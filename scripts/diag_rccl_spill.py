"""Diagnostic: the RCCL world-N circulant spill case (tests/test_rccl_world.py) under each exchange
mode, plus the loopback transport in the same modes; prints every rank's trajectory and whether its
initial colouring equals the others'. Usage: python scripts/diag_rccl_spill.py WORLD"""
import os
import socket
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, mode, max_sweeps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"diag-rank{rank}",
                      NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", MCMC_EXCHANGE=mode)
    import torch

    torch.cuda.init()
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_gpu_parity import circulant
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd.distributed import NativePartitionedColoringMCMC, plan_rows

        off, idx = circulant(60000, 4)
        g = M.Graph.from_csr(off, idx)
        rs = M.GPURand(60000, 21, M.GlibcRand(1, 0))
        drv = NativePartitionedColoringMCMC(g, rs, M.ColoringMCMCParams(nCol=3, epsilon=3e7, maxRip=4),
                                            plan_rows(60000, world), device=0)
        drv.init(0)
        c0 = drv.coloring()
        st = drv.run(0, max_sweeps)
        q.put((rank, drv.trajectory().tolist(), int(np.int64(c0.sum())), int(st.iter), drv.coloring().tolist()[:8]))
        drv.close()
        g.close()
    except Exception as e:
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import oracle_ref as O
    from test_gpu_parity import circulant

    off, idx = circulant(60000, 4)
    O.srand(1)
    r = O.mcmc_run(off, idx, 3, 21, epsilon=3e7, maxRip=4, nthreads=8)
    print("oracle", r.traj.tolist(), flush=True)
    for mode in ("p2p", "delta", "allgather"):
        for ms in (1, 0):
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            port = _free_port()
            procs = [ctx.Process(target=worker, args=(k, world, port, mode, ms, q)) for k in range(world)]
            for p in procs:
                p.start()
            res = sorted(q.get(timeout=120) for _ in range(world))
            for p in procs:
                p.join(timeout=60)
            for x in res:
                print(f"rccl world={world} mode={mode} max_sweeps={ms}", x, flush=True)
    # loopback, same modes
    from mcmc_colorer_amd import colorer as M
    from mcmc_colorer_amd.distributed import LoopbackPartition, plan_rows

    g = M.Graph.from_csr(off, idx)
    for mode in ("p2p", "delta", "allgather"):
        os.environ["MCMC_EXCHANGE"] = mode
        lp = LoopbackPartition(g, M.ColoringMCMCParams(nCol=3, epsilon=3e7, maxRip=4), 21, plan_rows(60000, world))
        lp.run(M.GlibcRand(1, 0))
        print(f"loopback world={world} mode={mode}", [lp.trajectory(k).tolist() for k in range(world)], flush=True)
        lp.close()


if __name__ == "__main__":
    main()
