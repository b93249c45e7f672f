"""configs[3] (C4) at full size on ONE GPU: the C3 graph (1e7 rows, ~1e11 arcs) vertex-partitioned
over 8 ranks, every rank generating only its own rows (mcmc_graph_er_fast_rows), the native driver
(mcmc_part_run) over the loopback transport -- the exact sequence of the RCCL path with device
copies in place of ncclSend/ncclRecv (the RCCL leg itself stays unmeasured until an 8-GPU run).
After 3 sweeps every rank's replica equals C_3 of tests/c3_expect.py for EVERY vertex (the
restatement that tests/test_c3_full.py checks the one-GPU run against), and every rank's trajectory
is [n, n, n]. Plans: equal rows (the bench's), and an unequal one; exchanges: the default delta
exchange (few changed vertices at eps 1e-8) and, at eps 1e-3 (~37 000 changes per rank and sweep,
past a delta slot's 2047), the overflow fallback to full row ranges."""
import time

import numpy as np
import pytest

import c3_expect as X

N, P, SEED, NCOL = X.N, X.P, X.SEED, X.NCOL


def _bounds(kind):
    from mcmc_colorer_amd.distributed import plan_rows

    if kind == "equal":
        return plan_rows(N, 8)
    # unequal: ranks of 0.5x .. 1.5x the mean, multiples of 64 rows
    w = np.array([0.5, 1.5, 0.8, 1.2, 1.0, 0.7, 1.3, 1.0])
    cut = np.concatenate([[0], np.cumsum(w) / w.sum()])
    b = (np.round(cut * N / 64) * 64).astype(np.int64)
    b[-1] = N
    return b.astype(np.uint32)


@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("plan,eps", [("equal", 1e-8), ("unequal", 1e-8), ("equal", 1e-3)])
def test_c4_full_size_loopback_world8(hip_lib, plan, eps):
    import torch

    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd.distributed import LoopbackPartition

    E, k0, evs = X.expected(3, eps)
    b = _bounds(plan)
    free0 = torch.cuda.mem_get_info()[0]
    t0 = time.perf_counter()
    graphs = [M.Graph.er_fast(N, P, SEED, rows=(int(b[r]), int(b[r + 1]))) for r in range(8)]
    tg = time.perf_counter() - t0
    assert sum(gr.nEdges for gr in graphs) > 9.9e10
    lp = LoopbackPartition(graphs, M.ColoringMCMCParams(nCol=NCOL, epsilon=eps, maxRip=250), SEED, b)
    st = lp.run(M.GlibcRand(1), max_sweeps=3)
    used = free0 - torch.cuda.mem_get_info()[0]
    infos = [lp.info(r) for r in range(8)]
    print(f"\nC4 loopback world 8, {plan} plan {b.tolist()}, eps {eps}: graphs {tg:.1f} s, device memory "
          f"{used / 1e9:.1f} GB; per-rank layout GB " +
          " ".join(f"{i['layout_bytes'] / 1e9:.1f}" for i in infos) +
          f"; loop {st[0].loopMs:.1f} ms for 3 sweeps; overflow events {evs}", flush=True)
    for r in range(8):
        got = lp.coloring(r)
        bad = np.nonzero(got != E[3])[0]
        assert len(bad) == 0, f"rank {r}: {len(bad)} vertices differ from C_3, first {bad[:5].tolist()}"
        assert lp.trajectory(r).tolist() == [N, N, N], r
        assert st[r].glibcDraws == sum(evs)
    lp.close()
    for gr in graphs:
        gr.close()
