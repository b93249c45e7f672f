"""Multi-rank path on CPU (gloo): the product's PartitionedColoringMCMC driver with the numpy rank
backend (tests/partition_ref.py), world sizes 2 and 3, against the unpartitioned oracle: equal-row
and arc-balanced plans (mcmc_part_plan_csr), events on every rank, and more events per rank than a
footer holds (the spill exchange) -- with the full-range exchange and with the delta exchange
(changed vertices only; a slot that overflows pauses the sweep, which then travels in full)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ref as O

CASES = [
    # graph, n, p, nCol, seed, eps, taboo, maxRip, plan
    ("simulate", 90, 0.2, 6, 4, 1e-8, 0, 30, "rows"),
    ("simulate", 120, 0.3, 7, 9, 3.3e6, 1, 12, "rows"),     # CDF-overflow events on every rank
    ("simulate", 80, 0.3, 300, 5, 1e-3, 0, 6, "rows"),      # nCol > 256: the wide sweep's 2-byte colours
    ("skewed", 2000, 0.0, 12, 6, 1e-8, 0, 12, "arcs"),      # arc-balanced plan of a skewed graph
    ("circulant", 10500, 0.0, 3, 21, 3e7, 0, 3, "rows"),    # > 1020 events per rank in sweep 0: spill
    ("circulant", 20000, 0.0, 5, 17, 0.05, 0, 20, "rows"),  # > 2047 changed vertices per rank: delta overflow
]


def make_graph(kind, n, p):
    if kind == "simulate":
        O.srand(1)
        return O.setup_rnd2(n, p)
    if kind == "circulant":
        from test_gpu_parity import circulant

        return circulant(n, 4)
    # skewed: low ids are hubs (degree falls with the id), the shape equal-row plans balance badly
    rng = np.random.default_rng(n)
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q, exchange="full"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import partition_ref as PR
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd.distributed import PartitionedColoringMCMC, plan_csr, plan_rows

        kind, n, p, ncol, seed, eps, taboo, maxrip, pl = case
        off, idx = make_graph(kind, n, p)
        bounds = plan_csr(off, world) if pl == "arcs" else plan_rows(n, world)
        backend = PR.NumpyRank(off, idx, ncol, world, rank, eps=eps, maxRip=maxrip, taboo=taboo, bounds=bounds)
        draws = n * (n + 1) // 2 if kind == "simulate" else 0
        rs = M.GPURand(n, seed, M.GlibcRand(1, draws))

        class _G:   # only nNodes/maxDeg are read by the driver when nCol is given
            nNodes = n

        params = M.ColoringMCMCParams(nCol=ncol, epsilon=eps, maxRip=maxrip, tabooIteration=taboo)
        drv = PartitionedColoringMCMC(_G(), rs, params, backend=backend, check_every=3, exchange=exchange)
        out = []
        for it in range(2):                    # two repetitions: seed + i, shared glibc stream
            drv.run(it)
            out.append((drv.coloring().tolist(), drv.trajectory().tolist(), backend.iter,
                        rs.glibc.window.tolist(), drv.spills, bounds.tolist(), drv.overflows))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["full", "delta"])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{c[1]}-{c[8]}")
def test_partitioned_driver_gloo_matches_oracle(world, case, exchange):
    kind, n, p, ncol, seed, eps, taboo, maxrip, pl = case
    off, idx = make_graph(kind, n, p)
    O.srand(1)
    if kind == "simulate":
        O.setup_rnd2(n, p)   # the glibc stream position after the generator
    refs = [O.mcmc_run(off, idx, ncol, seed + i, epsilon=eps, tabooIteration=taboo, maxRip=maxrip, nthreads=4)
            for i in range(2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q, exchange)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = dict(q.get(timeout=600) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank in range(world):
        for i, ref in enumerate(refs):
            colors, traj, it, _, spills, bounds, _ = results[rank][i]
            assert colors == ref.colors.tolist(), (rank, i)
            assert traj == ref.traj.tolist(), (rank, i)
            assert it == ref.res.iter
    assert refs[0].res.glibcDraws + refs[1].res.glibcDraws > 0 or eps < 1
    # replicas leave the glibc stream at the same position
    assert len({tuple(results[r][1][3]) for r in range(world)}) == 1
    if kind == "circulant" and n == 10500:
        assert results[0][0][4] >= 1, "the case must exercise the spill exchange"
    if kind == "circulant" and n == 20000 and exchange == "delta":
        assert results[0][0][6] >= 2, "the case must overflow delta slots (and return to delta mode)"
    if pl == "arcs":
        b = results[0][0][5]
        deg = np.diff(off.astype(np.int64))
        loads = [int(deg[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert b != plan_rows_py(n, world) and max(loads) < 1.25 * sum(loads) / world, (b, loads)


def plan_rows_py(n, world):
    S = ((n + world - 1) // world + 63) // 64 * 64
    return [min(r * S, n) for r in range(world)] + [n]


def _ncol_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mcmc_colorer_amd import colorer as M
        from mcmc_colorer_amd.distributed import group_default_ncol

        class _Rows:   # a rank's row-partial graph: its own rows' max degree only
            def getMaxNodeDeg(self):
                return [37, 120, 64][rank]

        q.put((rank, group_default_ncol(_Rows(), M.ColoringMCMCParams(nCol=0)),
               group_default_ncol(_Rows(), M.ColoringMCMCParams(nCol=0, numColorRatio=0.5))))
    finally:
        dist.destroy_process_group()


def test_default_ncol_uses_whole_graph_max_degree():
    """with per-rank graphs (Graph.er_fast(rows=...)) every rank must take main.cu:162's
    nCol from the WHOLE graph's max degree, not its own rows'."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ncol_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict((x[0], x[1:]) for x in (q.get(timeout=300) for _ in range(world)))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(res[r] == (120, 60) for r in range(world)), res
