"""Every MCMC_* setting the library reads, against the oracle (a default-off variant is
product code and needs a parity test).

Knobs covered here (the others have their own tests: MCMC_GATHER / MCMC_BLOCK_LOG2 / MCMC_SUB_LOG2 /
MCMC_GROUP_ROWS / MCMC_TILE_STREAM in test_gpu_parity.py::test_all_gather_variants, MCMC_DRAIN_ROWS
and MCMC_FULL_SCAN there too, MCMC_EXCHANGE in test_multi.py, MCMC_WIDE_INC / MCMC_WIDE_SCAN /
MCMC_SPLIT_ARCS in test_wide.py, the persistent wide sweep's MCMC_WIDE_SOLO / MCMC_WS_ENTER /
MCMC_WS_LEAD_ARCS / MCMC_WS_LEAD_HEAVY / MCMC_WS_LIGHT / MCMC_WS_MAX / MCMC_WS_POLL / MCMC_WS_POLL_IDLE /
MCMC_WS_DEBUG in
test_wide.py::test_wide_persistent* and test_multi.py::test_native_loopback_wide_world1,
MCMC_DENSE / MCMC_DENSE_ROWS / MCMC_DENSE_MULTI / MCMC_DENSE_CHG_CAP / MCMC_DCM_BS in test_dense.py, MCMC_DC_POLL
(the dense helpers' poll interval) in test_dense.py::test_dense_poll_interval, MCMC_WT_INC / MCMC_WT_ARCS_DIV / MCMC_WT_RC in
test_wide.py::test_wide_tiled_incremental):
  tiled scan sweep (MCMC_DENSE=0): MCMC_LATE_STAGE, MCMC_NO_OLIST, MCMC_NO_EWALK, MCMC_TQ_DENSE,
  MCMC_PHASE_DUMP, MCMC_PAIR_TRACE (diagnostics: results unchanged);
  partitioned: MCMC_PART_SOLO_OFF;
  wide sweep: MCMC_WALK_LIGHT, MCMC_WALK_TIE, MCMC_WIDE_INC_DIV, MCMC_WIDE_INC_HUB, MCMC_WIDE_INC_SLOT,
  MCMC_TSCAN_PLAN;
  persistent launches: MCMC_PERSIST_CHECK_GRID (the co-residency check; test only).
The count rebuild's MCMC_DENSE_RB is in test_dense.py::test_dense_rebuild_*.
"""
import numpy as np
import pytest

import oracle_ref as O
from test_gpu_parity import assert_same, gpu_run, oracle_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


TILED = [
    {"MCMC_LATE_STAGE": "0"}, {"MCMC_LATE_STAGE": "1"}, {"MCMC_NO_OLIST": "1"}, {"MCMC_NO_EWALK": "1"},
    {"MCMC_TQ_DENSE": "0"}, {"MCMC_TQ_DENSE": "1"}, {"MCMC_TQ_DENSE": "3"},
    {"MCMC_PHASE_DUMP": "@phase"}, {"MCMC_PAIR_TRACE": "@pairs"},
]


@pytest.mark.parametrize("env", TILED, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("n,p,ncol,seed,eps,taboo,maxrip", [(6000, 0.02, 16, 51, 1e-8, 0, 30),
                                                            (3000, 0.05, 40, 52, 1e-3, 2, 20)])
def test_tiled_scan_knobs(M, monkeypatch, tmp_path, env, n, p, ncol, seed, eps, taboo, maxrip):
    """The tiled scan sweep (MCMC_DENSE=0) with 1024-id column blocks (MCMC_BLOCK_LOG2=10: several
    blocks, so tail queues, listed pairs and drains all run) under each setting."""
    monkeypatch.setenv("MCMC_DENSE", "0")
    monkeypatch.setenv("MCMC_GATHER", "tiled")
    monkeypatch.setenv("MCMC_BLOCK_LOG2", "10")
    for k, v in env.items():
        monkeypatch.setenv(k, str(tmp_path / v[1:]) if v.startswith("@") else v)
    off, idx, nc, r = oracle_case(n, p, ncol, seed, epsilon=eps, tabooIteration=taboo, maxRip=maxrip)
    col, st, _ = gpu_run(M, off, idx, nc, seed, n * (n + 1) // 2, eps=eps, maxRip=maxrip, taboo=taboo)
    assert_same(col, st, r)
    assert col.info()["variant"] == "tiled"


def test_part_solo_off(M, monkeypatch):
    """A world-1 partition through the footer + commit launch instead of the fused one-GPU step."""
    from mcmc_colorer_amd.distributed import LoopbackPartition, plan_rows

    monkeypatch.setenv("MCMC_PART_SOLO_OFF", "1")
    off, idx, nc, r = oracle_case(3000, 0.02, 16, 53, epsilon=1e-8, maxRip=30)
    g = M.Graph.from_csr(off, idx)
    lp = LoopbackPartition(g, M.ColoringMCMCParams(nCol=nc, maxRip=30), 53, plan_rows(3000, 1))
    st = lp.run(M.GlibcRand(1, 3000 * 3001 // 2))
    assert lp.coloring(0).tolist() == r.colors.tolist()
    assert lp.trajectory(0).tolist() == r.traj.tolist()
    assert (st[0].iter, st[0].finalViol, st[0].glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
    lp.close()


WIDE = [
    {"MCMC_WALK_LIGHT": "0"}, {"MCMC_WALK_LIGHT": "64"}, {"MCMC_WALK_TIE": "0"}, {"MCMC_WIDE_INC_DIV": "1"},
    {"MCMC_WIDE_INC_DIV": "100000"}, {"MCMC_WIDE_INC_HUB": "8"}, {"MCMC_WIDE_INC_SLOT": "1"},
    {"MCMC_TSCAN_PLAN": "lpt"},
]


@pytest.mark.parametrize("env", WIDE, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("ncol_div,eps,taboo", [(1, 1e-8, 0), (4, 1e-8, 2), (4, 1e-3, 0)])
def test_wide_knobs(M, monkeypatch, env, ncol_div, eps, taboo):
    """The wide sweep on an R-MAT graph (hub rows, nCol = maxDeg and maxDeg / 4: violators walked
    every sweep) under each setting."""
    import oracle_np as NP

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 5)
    ncol = max(257, int(np.diff(off.astype(np.int64)).max()) // ncol_div)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, 3, epsilon=eps, tabooIteration=taboo, maxRip=15)
    g = M.Graph.from_csr(off, idx)
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 3, M.GlibcRand(1)),
                         M.ColoringMCMCParams(nCol=ncol, epsilon=eps, tabooIteration=taboo, maxRip=15))
    st = col.run(0)
    assert col.info()["variant"] == "wide"
    assert_same(col, st, r)


@pytest.mark.parametrize("kind", ["dense", "wide"])
def test_persistent_needs_coresident_grid(M, monkeypatch, kind):
    """The persistent launches (dc_multi_kernel, ws_kernel) spin on flags their leader posts, so a
    context takes them only when the whole grid can be resident at once (hipOccupancy x CUs >= the
    grid). MCMC_PERSIST_CHECK_GRID makes the check ask for more workgroups than the device holds:
    the context then runs the per-sweep path -- the same results as the oracle, the persistent
    launch off in the statistics. Without the knob the same case takes the persistent path."""
    import oracle_np as NP

    def run(check_grid):
        if check_grid:
            monkeypatch.setenv("MCMC_PERSIST_CHECK_GRID", "100000000")
        else:
            monkeypatch.delenv("MCMC_PERSIST_CHECK_GRID", raising=False)
        if kind == "dense":
            off, idx, nc, r = oracle_case(3000, 0.3, 16, 57, epsilon=1e-8, maxRip=40)
            col, st, _ = gpu_run(M, off, idx, nc, 57, 3000 * 3001 // 2, maxRip=40)
            assert_same(col, st, r)
            return col.dense_stats()["persistent"]
        monkeypatch.setenv("MCMC_WS_ENTER", "-1")
        off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
        ncol = int(np.diff(off.astype(np.int64)).max())
        O.srand(1)
        r = O.mcmc_run(off, idx, ncol, 1, maxRip=20)
        g = M.Graph.from_csr(off, idx)
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=20))
        st = col.run(0)
        assert_same(col, st, r)
        return col.wide_solo_stats()["enabled"]

    assert run(False)
    assert not run(True)
