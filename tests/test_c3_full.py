"""configs[2] (C3) at full size: `--mcmcgpu --simulate 0.001 -n 10000000`, 32 colours, one MI355X.

The only other GPU runs of this path are reduced (tests/test_gpu_parity.py::test_er_fast_*, n <= 2e5).
Here the real graph is built (the build's G(n, p), csrc/er_gen.h, seed 1: 1e7 rows, ~1e11 arcs, 153
column blocks, layout indices far past 2^32) and checked against the oracle without enumerating it:

  * rows: ~1000 sampled rows of three column blocks (first, middle, last) read back from the tiled
    layout (mcmc_graph_rows) equal the oracle's per-row restatement of the generator
    (oracle_er_rows: the rows' own streams plus every stream into their blocks);
  * C_0 equals ColoringMCMC_CPU's initial colouring (uniform_int from default_random_engine(seed),
    coloringMCMC_CPU.cpp:53-61) on all 1e7 vertices;
  * sweeps 0..2: for every sampled vertex, C_{t+1}[v] equals the oracle's one-vertex update
    (count_free_colors / fill_p / extract_new_color, coloringMCMC_CPU.cpp:361-528) from C_t on its
    regenerated row and u_v = engine draw K0 + t n + v + 1 (:139); the per-vertex violation flags
    of the tail cut's recount kernel (a second code path over the layout) equal the oracle's for
    the sampled rows; the recount's total equals the sweep's fused Cviol_t (the trajectory);
  * sweeps 0..2, EVERY vertex: C_1..C_3 equal tests/c3_expect.py's restatement of the all-full case
    (pinned against the oracle's one-vertex update), overflow events replayed from glibc in vertex
    order -- at the default eps and at eps = 1e-3 (about 3% of the vertices change colour per sweep).
"""
import time

import numpy as np
import pytest

import c3_expect as C3X
import oracle_ref as O

N, P, SEED, NCOL, EPS = 10_000_000, 0.001, 1, 32, 1e-8
T = 65536


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c3_full_size_rows_and_sweeps(hip_lib):
    import mcmc_colorer_amd.colorer as M

    t0 = time.perf_counter()
    g = M.Graph.er_fast(N, P, SEED)
    print(f"\nC3 graph: n={g.nNodes} m={g.nEdges} maxDeg={g.maxDeg} ({time.perf_counter() - t0:.1f} s)", flush=True)
    assert g.nNodes == N and g.nEdges > 9.9e10
    rng = np.random.default_rng(2026)
    rows = []
    for X in (0, 76, (N - 1) // T):
        lo, hi = X * T, min(N, (X + 1) * T)
        rows += [lo, lo + 1, hi - 1] + rng.integers(lo, hi, 330).tolist()
    rows = np.unique(np.array(rows, dtype=np.uint32))
    got, pos = g.rows(rows)
    t1 = time.perf_counter()
    ref = O.er_rows(N, P, SEED, rows)
    print(f"oracle rows: {len(rows)} rows in {time.perf_counter() - t1:.1f} s; layout index of the first id "
          f"(sample): " + ", ".join(f"row {int(v)} @ {int(q)}" for v, q in list(zip(rows, pos))[::150]), flush=True)
    for v, a, b in zip(rows, got, ref):
        assert np.array_equal(np.sort(a), b), f"row {v}"
    assert int((pos >= 2**32).sum()) >= 600, "sampled rows must reach layout indices past 2^32"

    col = M.ColoringMCMC(g, M.GPURand(N, SEED, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=NCOL))
    col.init(0)
    C = [col.coloring()]
    exp0 = np.zeros(N, dtype=np.uint32)
    k0 = int(O.lib().oracle_uniform_int_seq(SEED, NCOL, N, O._p(exp0)))
    assert np.array_equal(C[0], exp0), "initial colouring"
    counts, flags = [], []
    for t in range(3):
        c, f = col.count_violations(flags=True)
        counts.append(c)
        flags.append(f[rows])
        st = col.step(1)
        C.append(col.coloring())
    assert st.initDraws == k0
    traj = col.trajectory()
    print(f"Cviol trajectory {traj.tolist()}, recount {counts}", flush=True)
    assert traj.tolist() == counts, "fused Cviol_t != recount of C_t"
    checked = events = 0
    for t in range(3):
        u = O.canonical_at(SEED, k0 + t * N + rows.astype(np.uint64) + 1)
        for i, v in enumerate(rows.tolist()):
            c, viol = O.vertex_update(NCOL, EPS, int(C[t][v]), C[t][ref[i]], float(u[i]))
            assert bool(flags[t][i]) == viol, f"violation flag of {v} at sweep {t}"
            if c is None:
                events += 1
            else:
                assert int(C[t + 1][v]) == c, f"C_{t + 1}[{v}]"
                checked += 1
    print(f"checked {checked} vertex updates ({events} CDF overflows skipped)", flush=True)
    assert checked >= 2900
    t1 = time.perf_counter()
    C3X.pin_walk(NCOL, EPS)
    E, k0e, evs = C3X.expected(3, EPS)
    assert k0e == k0
    for t in range(4):
        bad = np.nonzero(C[t] != E[t])[0]
        assert len(bad) == 0, f"C_{t}: {len(bad)} vertices differ, first {bad[:5].tolist()}"
    print(f"every vertex of C_1..C_3 equals the all-full restatement ({evs} overflow events; "
          f"{time.perf_counter() - t1:.1f} s)", flush=True)
    col.close()
    g.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c3_full_size_every_vertex_eps_1e3(hip_lib):
    """eps = 1e-3: about 3% of the vertices leave their colour each sweep (u < own colour x eps walks
    to a lower colour), so the walk's every branch position is exercised on all 1e7 vertices."""
    import mcmc_colorer_amd.colorer as M

    eps = 1e-3
    C3X.pin_walk(NCOL, eps)
    E, k0, evs = C3X.expected(3, eps)
    g = M.Graph.er_fast(N, P, SEED)
    col = M.ColoringMCMC(g, M.GPURand(N, SEED, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=NCOL, epsilon=eps))
    col.init(0)
    got = [col.coloring()]
    for _ in range(3):
        col.step(1)
        got.append(col.coloring())
    changed = [int((E[t + 1] != E[t]).sum()) for t in range(3)]
    print(f"\nchanged colours per sweep {changed}, overflow events {evs}", flush=True)
    assert min(changed) > 100_000
    for t in range(4):
        bad = np.nonzero(got[t] != E[t])[0]
        assert len(bad) == 0, f"C_{t}: {len(bad)} vertices differ, first {bad[:5].tolist()}"
    assert col.trajectory().tolist()[:3] == [N, N, N]
    col.close()
    g.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c3_full_size_reference_loop_every_vertex(hip_lib):
    """The bench's exact reference loop at full C3 size -- run() from the initial colouring to its
    maxRip cap (251 accepted sweeps + the count-only pass, coloringMCMC_CPU.cpp:136-270) -- at the
    default eps (the persistent dense sweep: discrete-log candidate rows, solo sweeps, move phases
    for the ~60 vertices of the dense range that change over the run) and at eps = 1e-3 (no
    closed-form walk: one dense sweep per launch, ~13 000 vertices of the dense range moving per
    sweep, incremental count updates over hundreds of sweeps). Every vertex of the final colouring
    C_251, the glibc draws and the whole Cviol trajectory equal tests/c3_expect.py's streamed
    restatement of the all-full case."""
    import mcmc_colorer_amd.colorer as M

    g = M.Graph.er_fast(N, P, SEED)
    for eps in (EPS, 1e-3):
        t0 = time.perf_counter()
        col = M.ColoringMCMC(g, M.GPURand(N, SEED, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=NCOL, epsilon=eps))
        st = col.run(0)
        got = col.coloring()
        traj = col.trajectory()
        ds = col.dense_stats()
        t1 = time.perf_counter()
        C3X.pin_walk(NCOL, eps)
        E, k0, evs = C3X.expected_final(251, eps)
        print(f"\neps {eps}: loop {st.loopMs:.1f} ms ({t1 - t0:.1f} s with set-up), restatement "
              f"{time.perf_counter() - t1:.1f} s; glibc draws {st.glibcDraws}, events {sum(evs)}; dense {ds}", flush=True)
        assert (st.iter, bool(st.maxIterReached), st.sweepsRun) == (251, True, 252)
        assert st.initDraws == k0
        assert st.glibcDraws == sum(evs)
        assert traj.tolist() == [N] * 252
        bad = np.nonzero(got != E)[0]
        assert len(bad) == 0, f"eps {eps}: {len(bad)} vertices of C_251 differ, first {bad[:5].tolist()}"
        assert ds["incremental_sweeps"] >= 200 and ds["moved_vertices"] > 0
        if eps == EPS:
            assert ds["solo_sweeps"] >= 240, ds
        col.close()
    g.close()


@pytest.mark.gpu
@pytest.mark.timeout(1100)
def test_c3_default_ncol_maxdeg_sampled_rows(hip_lib):
    """C3 at the reference's default colour count (`--mcmcgpu --simulate-fast 0.001 -n 10000000
    --seed 1`: nCol = maxDeg, main.cu:162 -- about 10 400 colours): no CSR fits beside the 2.2e11 B
    layout, so the wide sweep runs over the layout itself (csrc/wide_tiled.h). C_0 is checked on every
    vertex; for sweeps 0..2 every one of ~1000 sampled rows (three column blocks) equals the oracle's
    one-vertex update on its regenerated row, and so do the recount's violation flags; the fused
    Cviol_t equals the recount of C_t. r06: the same checks on sweeps 3..9, which run from the
    incremental violation counts (wide_tiled.h wt_*) once the changed rows thin out."""
    import mcmc_colorer_amd.colorer as M

    g = M.Graph.er_fast(N, P, SEED)
    ncol = M.default_ncol(g, M.ColoringMCMCParams(nCol=0))
    assert ncol == g.maxDeg > 256
    rng = np.random.default_rng(77)
    rows = []
    for X in (0, 76, (N - 1) // T):
        lo, hi = X * T, min(N, (X + 1) * T)
        rows += [lo, lo + 1, hi - 1] + rng.integers(lo, hi, 330).tolist()
    rows = np.unique(np.array(rows, dtype=np.uint32))
    t0 = time.perf_counter()
    ref = O.er_rows(N, P, SEED, rows)
    print(f"\nnCol = maxDeg = {ncol}; oracle rows: {len(rows)} in {time.perf_counter() - t0:.1f} s", flush=True)
    col = M.ColoringMCMC(g, M.GPURand(N, SEED, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol))
    assert col.info()["variant"] == "wide-tiled"
    col.init(0)
    C = [col.coloring()]
    exp0 = np.zeros(N, dtype=np.uint32)
    k0 = int(O.lib().oracle_uniform_int_seq(SEED, ncol, N, O._p(exp0)))
    assert np.array_equal(C[0], exp0), "initial colouring"
    counts, flags, ms = [], [], []
    SW = 10
    for t in range(SW):
        c, f = col.count_violations(flags=True)
        counts.append(c)
        flags.append(f[rows])
        t1 = time.perf_counter()
        st = col.step(1)
        ms.append((time.perf_counter() - t1) * 1e3)
        C.append(col.coloring())
    assert st.initDraws == k0
    traj = col.trajectory()
    print(f"Cviol trajectory {traj.tolist()}, recount {counts}; step wall ms {[round(x, 1) for x in ms]}", flush=True)
    assert traj.tolist() == counts, "fused Cviol_t != recount of C_t"
    ws = col.wide_inc_stats()
    print(f"wide tiled counts: {ws}", flush=True)
    assert ws["enabled"] and ws["incremental_sweeps"] >= 4, ws
    checked = events = moved = 0
    for t in range(SW):
        u = O.canonical_at(SEED, k0 + t * N + rows.astype(np.uint64) + 1)
        for i, v in enumerate(rows.tolist()):
            c, viol = O.vertex_update(ncol, EPS, int(C[t][v]), C[t][ref[i]], float(u[i]))
            assert bool(flags[t][i]) == viol, f"violation flag of {v} at sweep {t}"
            if c is None:
                events += 1
            else:
                assert int(C[t + 1][v]) == c, f"C_{t + 1}[{v}]"
                checked += 1
                moved += int(c != int(C[t][v]))
    print(f"checked {checked} vertex updates ({moved} moved, {events} CDF overflows skipped)", flush=True)
    assert checked >= 2900 * SW // 3 and moved > 500
    col.close()
    g.close()
