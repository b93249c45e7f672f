"""GPU parity of the reference-GPU-semantics mode against the oracle.

The HIP path (tiled REF sweep through the C ABI: mcmc_gpurand_*, mcmc_ref_create/run) and
oracle/mcmc_gpu_ref.cpp -- pinned by tests/test_xorwow.py (rocRAND engine, Python restatement) --
must agree bit-for-bit: final colouring, per-sweep conflicting-edge counts, rip, the
max-iteration flag, sweeps, tail-cut passes and counts, and the XORWOW states after the run
(which the next repetition continues from). Against CUDA itself parity is unpinned (no CUDA here).
"""
import numpy as np
import pytest

import oracle_ref as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def set_gather(monkeypatch, spec):
    parts = spec.split(":")
    monkeypatch.setenv("MCMC_GATHER", parts[0])
    for key, v in zip(("MCMC_BLOCK_LOG2", "MCMC_SUB_LOG2", "MCMC_GROUP_ROWS", "MCMC_TILE_STREAM"), parts[1:]):
        if v:
            monkeypatch.setenv(key, v)


def compare(M, off, idx, g, nc, seed, *, maxrip=250, taboo=0, tailcut=False, reps=1):
    n = len(off) - 1
    st = O.gpurand_init(n, seed)
    states = M.CurandStates(n, seed)
    assert np.array_equal(states.states(), st)
    params = M.ColoringMCMCParams(nCol=nc, maxRip=maxrip, tabooIteration=taboo, tailcut=tailcut)
    for _ in range(reps):
        r = O.mcmc_gpu_run(off, idx, nc, st, maxRip=maxrip, tabooIteration=taboo, tailcut=tailcut)
        col = M.ColoringMCMCGpuRef(g, states, params)
        s = col.run()
        assert col.coloring().tolist() == r.colors.tolist()
        assert col.trajectory().tolist() == r.traj.tolist()
        assert (s.iter, bool(s.maxIterReached), s.sweepsRun, s.tailcutPasses, s.finalViol) == (
            r.res.rip, bool(r.res.maxIterReached), r.res.sweeps, r.res.tailcutPasses, r.res.finalConflicts)
        assert col.tail_trajectory().tolist() == r.tail_traj.tolist()
        assert np.array_equal(states.states(), st)
        col.close()
    return r


CASES = [
    # n, p, nCol, seed, maxRip, taboo, tailcut
    (1000, 0.1, 0, 1, 250, 0, False),    # configs[0]: nCol = maxDeg (137), converges
    (1000, 0.1, 0, 1, 250, 0, True),     # ... stops within z = 50, the GPU tail cut resolves
    (2000, 0.02, 12, 2, 40, 0, False),   # too few colours: runs to maxRip
    (1500, 0.05, 20, 3, 30, 2, False),   # taboo
    (900, 0.1, 31, 4, 30, 0, True),
    (900, 0.1, 32, 5, 20, 1, False),     # one mask word, and a colour 32 (u = 1.0f) would set none
    (3000, 0.01, 8, 6, 25, 1, True),     # tail cut after the cap (stale conflictCounter), bounded
]


@pytest.mark.parametrize("gather", ["tiled", "tiled::::0", "tiled:8:1:50", "tiled:6:2:7:0", "tiled:10:5:1"])
@pytest.mark.parametrize("n,p,ncol,seed,maxrip,taboo,tailcut", CASES)
def test_ref_mode_matches_oracle(M, monkeypatch, gather, n, p, ncol, seed, maxrip, taboo, tailcut):
    """Streamed slices and the resident replica, 256- to 1024-vertex blocks (dozens of blocks,
    own colours of odd-sized groups straddling 16-byte boundaries), 1..32 lanes per segment."""
    set_gather(monkeypatch, gather)
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    nc = ncol or O.max_deg(off)
    g = M.Graph.from_csr(off, idx)
    compare(M, off, idx, g, nc, seed, maxrip=maxrip, taboo=taboo, tailcut=tailcut)


def test_ref_mode_repetitions_continue_the_states(M):
    """main.cu:80,193: one GPURand for all repetitions -- run 2 starts from run 1's states."""
    O.srand(1)
    off, idx = O.setup_rnd2(1200, 0.05)
    compare(M, off, idx, M.Graph.from_csr(off, idx), 9, 7, maxrip=20, taboo=1, tailcut=True, reps=3)


def test_ref_mode_self_loops(M):
    """Self-loops occupy the vertex's own colour; the reference's edge count (v < w) never counts
    them."""
    n, K = 500, 3
    nb = sorted([d for k in range(1, K + 1) for d in (k, -k)])
    rows = [sorted({(v + d) % n for d in nb} | ({v} if v % 7 == 0 else set())) for v in range(n)]
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    idx = np.array([w for r in rows for w in r], dtype=np.uint32)
    compare(M, off, idx, M.Graph.from_csr(off, idx), 5, 3, maxrip=30, tailcut=True)


def test_ref_mode_generated_graph(M):
    """A generated graph (no CSR on the device, three 2^16-column blocks) == the oracle on the
    restated CSR."""
    n, p, ncol, seed = 140000, 0.0004, 60, 9
    off, idx = O.er_fast(n, p, seed)
    g = M.Graph.er_fast(n, p, seed)
    compare(M, off, idx, g, ncol, seed, maxrip=15, tailcut=True)


def test_ref_mode_multigraph_unsorted_rows(M):
    """Repeated neighbours count once per arc (conflictCounter walks every arc), unsorted rows; the
    scan tells padding from real ids by the segment table's padding counts, not by id order."""
    rng = np.random.default_rng(11)
    n = 800
    rows = [[] for _ in range(n)]
    for _ in range(6000):
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b:
            rows[a].append(b)
            rows[b].append(a)
    for r in rows:
        rng.shuffle(r)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    idx = np.array([w for r in rows for w in r], dtype=np.uint32)
    compare(M, off, idx, M.Graph.from_csr(off, idx), 7, 5, maxrip=25, tailcut=True)


def hub_graph(n, hubs, hub_deg, extra, seed):
    """Symmetric CSR: `hubs` vertices joined to hub_deg random others each, plus `extra` random
    edges (rows of every size class of the wide REF sweep: lane, wave and workgroup rows)."""
    rng = np.random.default_rng(seed)
    edges = set()
    for h in range(hubs):
        for w in rng.choice(n, size=hub_deg, replace=False):
            if int(w) != h:
                edges.add((min(h, int(w)), max(h, int(w))))
    for _ in range(extra):
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b:
            edges.add((min(a, b), max(a, b)))
    rows = [[] for _ in range(n)]
    for a, b in edges:
        rows[a].append(b)
        rows[b].append(a)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    idx = np.array([w for r in rows for w in sorted(r)], dtype=np.uint32)
    return off, idx


WIDE_CASES = [
    # graph, nCol (0: maxDeg), seed, maxRip, taboo, tailcut
    ("rnd2", 0, 1, 40, 0, False),       # setupRnd2 G(1500, 0.3): nCol = maxDeg (~500), wave rows
    ("rnd2", 256, 2, 25, 2, True),      # the first colour count past the uint8 replicas; taboo
    ("hubs", 300, 3, 20, 0, False),     # 2500-arc hubs: workgroup rows and workgroup violator walks
    ("hubs", 0, 4, 15, 1, True),        # nCol = maxDeg, taboo, the tail cut on uint16 colours
    ("hubs", 4000, 5, 10, 0, False),    # more colours than any row has neighbours
]


@pytest.mark.parametrize("graph,ncol,seed,maxrip,taboo,tailcut", WIDE_CASES)
def test_ref_mode_wide_matches_oracle(M, graph, ncol, seed, maxrip, taboo, tailcut):
    """--mcmcgpu-ref past 255 colours (uint16 replicas, csrc/ref_wide.h): colouring, per-sweep
    conflicting-edge counts, rip, sweeps, tail cut and the XORWOW states equal the oracle's."""
    if graph == "rnd2":
        O.srand(1)
        off, idx = O.setup_rnd2(1500, 0.3)
    else:
        off, idx = hub_graph(6000, 6, 2500, 30000, seed)
    nc = ncol or O.max_deg(off)
    g = M.Graph.from_csr(off, idx)
    compare(M, off, idx, g, nc, seed, maxrip=maxrip, taboo=taboo, tailcut=tailcut)
