"""Multi-rank path on CPU (gloo): the product's PartitionedColoringMCMC driver with the numpy rank
backend (tests/partition_ref.py), world sizes 2 and 3, against the unpartitioned oracle."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ref as O

CASES = [
    # n, p, nCol, seed, eps, taboo, maxRip
    (90, 0.2, 6, 4, 1e-8, 0, 30),
    (120, 0.3, 7, 9, 3.3e6, 1, 12),     # CDF-overflow events on every rank
    (80, 0.3, 300, 5, 1e-3, 0, 6),      # nCol > 256: the wide sweep's 2-byte colour regions
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import partition_ref as PR
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd.distributed import PartitionedColoringMCMC

        n, p, ncol, seed, eps, taboo, maxrip = case
        O.srand(1)
        off, idx = O.setup_rnd2(n, p)
        backend = PR.NumpyRank(off, idx, ncol, world, rank, eps=eps, maxRip=maxrip, taboo=taboo)
        rs = M.GPURand(n, seed, M.GlibcRand(1, n * (n + 1) // 2))

        class _G:   # only nNodes/maxDeg are read by the driver when nCol is given
            nNodes = n

        params = M.ColoringMCMCParams(nCol=ncol, epsilon=eps, maxRip=maxrip, tabooIteration=taboo)
        drv = PartitionedColoringMCMC(_G(), rs, params, backend=backend, check_every=3)
        out = []
        for it in range(2):                    # two repetitions: seed + i, shared glibc stream
            drv.run(it)
            out.append((drv.coloring().tolist(), drv.trajectory().tolist(), backend.iter,
                        rs.glibc.window.tolist()))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES)
def test_partitioned_driver_gloo_matches_oracle(world, case):
    n, p, ncol, seed, eps, taboo, maxrip = case
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    refs = [O.mcmc_run(off, idx, ncol, seed + i, epsilon=eps, tabooIteration=taboo, maxRip=maxrip) for i in range(2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = dict(q.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank in range(world):
        for i, ref in enumerate(refs):
            colors, traj, it, _ = results[rank][i]
            assert colors == ref.colors.tolist(), (rank, i)
            assert traj == ref.traj.tolist(), (rank, i)
            assert it == ref.res.iter
    assert refs[0].res.glibcDraws + refs[1].res.glibcDraws > 0 or eps < 1
    # replicas leave the glibc stream at the same position
    assert len({tuple(results[r][1][3]) for r in range(world)}) == 1
