"""configs[4] stand-in at its own size: R-MAT scale 22 (4.19M vertices, ~8.4e7 arcs, the bench's C5
graph), the wide sweep from the initial colouring, with nCol = maxDeg (main.cu:162's default: 2 852
violators in sweep 0, converged after one) and nCol = maxDeg / 4 (violators in three sweeps, the
bench's `violators` record). EVERY vertex of every colouring equals tests/c5_expect.py (non-violators by the
oracle-pinned vectorised case (iii) walk, violators -- hubs included -- by the oracle's one-vertex
update on their rows, overflow events from glibc in vertex order); the fused Cviol trajectory equals
the host's violation count; and the arc-balanced loopback world 8 (the native partitioned driver,
uint16 replicas) gives the same replicas and trajectory on every rank."""
import time

import numpy as np
import pytest

import c5_expect as X


@pytest.fixture(scope="module", params=[1, 4], ids=["nCol=maxDeg", "nCol=maxDeg/4"])
def c5(hip_lib, request):
    import mcmc_colorer_amd.colorer as M

    t0 = time.perf_counter()
    g = M.Graph.rmat(22, 10, 0.5, 0.2, 0.2, 1)
    s = g.getStruct()
    ncol = max(257, g.getMaxNodeDeg() // request.param)
    X.pin(ncol, 1e-8)
    C, traj, events, k0 = X.expected(s.cumulDegs, s.neighs, ncol, 3)
    print(f"\nC5 stand-in: n={g.nNodes} m={g.nEdges} nCol=maxDeg={ncol}; host expectation of 3 sweeps "
          f"{time.perf_counter() - t0:.1f} s: Cviol {traj}, overflow events {events}, changed "
          f"{[int((C[t + 1] != C[t]).sum()) for t in range(len(C) - 1)]}", flush=True)
    yield M, g, ncol, C, traj, events, k0
    g.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c5_full_size_every_vertex(c5):
    M, g, ncol, C, traj, events, k0 = c5
    assert traj[0] > 1000, "the initial colouring must have violators (case (ii) walks)"
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol))
    col.init(0)
    got = [col.coloring()]
    counts = [col.count_violations()]
    for _ in range(len(C) - 1):
        st = col.step(1)
        got.append(col.coloring())
        counts.append(col.count_violations())
    assert st.initDraws == k0
    for t in range(len(C)):
        bad = np.nonzero(got[t] != C[t])[0]
        assert len(bad) == 0, f"C_{t}: {len(bad)} vertices differ, first {bad[:5].tolist()}"
    assert counts == traj[:len(C)], (counts, traj)
    if traj[-1] == 0:   # converged: the device loop stopped with the same trajectory
        st = col.step(1)
        assert st.iter == len(C) - 1 and st.finalViol == 0
        assert col.trajectory().tolist() == traj
    else:
        assert col.trajectory().tolist() == traj[:len(C) - 1]
    assert st.glibcDraws == sum(events)
    print(f"every vertex of C_1..C_3 equals the host expectation; recount {counts}", flush=True)
    col.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c5_full_size_loopback_world8_arc_balanced(c5):
    M, g, ncol, C, traj, events, k0 = c5
    from mcmc_colorer_amd.distributed import LoopbackPartition, plan

    b = plan(g, 8, balance=True)
    lp = LoopbackPartition(g, M.ColoringMCMCParams(nCol=ncol, maxRip=len(C) - 2 if traj[-1] else 250), 1, b)
    st = lp.run(M.GlibcRand(1))
    print(f"\nC5 loopback world 8, arc-balanced plan {b.tolist()}: loop {st[0].loopMs:.1f} ms for 3 sweeps", flush=True)
    for r in range(8):
        bad = np.nonzero(lp.coloring(r) != C[-1])[0]
        assert len(bad) == 0, f"rank {r}: {len(bad)} vertices differ from C_{len(C) - 1}"
        assert lp.trajectory(r).tolist() == traj, r
        assert st[r].glibcDraws == sum(events)
    lp.close()
