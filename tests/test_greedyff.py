"""The reference's parallel greedy first-fit colorer (ColoringGreedyFF, `--grdffgpu`;
graph_coloring/coloringGreedyFF.cu).

CPU: the vectorised restatement (oracle/oracle_np.py::greedy_ff) against a literal per-thread
restatement of the four kernels below (tentative_coloring :88-129 with its uint32 forbidden rows
flagged by the node's id, conflict_detection :134-163, update_coloring_GPU, check_uncolored_nodes).
GPU: the HIP colorer (csrc/greedyff.hip) against the restatement -- colours, colour count, rounds --
on --simulate, skewed and power-law graphs, and the CLI's -GFF- files. The reference publishes no
outputs for this colorer: parity is pinned by the two restatements, not by reference runs.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O

ROOT = Path(__file__).resolve().parent.parent


def literal_greedy_ff(off, idx):
    """The kernels as written: thread idx of each launch reads the launch's input array only."""
    n = len(off) - 1
    max_colors = int(np.diff(off.astype(np.int64)).max()) + 1
    coloring = [0] * n                                   # cudaMemset(coloring_device, 0)
    temp = [0] * n
    forbidden = [[0] * max_colors for _ in range(n)]     # cudaMalloc'ed rows, taken as zero
    rounds = 0
    uncolored = True
    while uncolored:
        rounds += 1
        out = list(temp)
        for i in range(n):                               # tentative_coloring
            if i == 0:
                out[i] = 1
            if coloring[i] != 0:
                continue
            for k in range(int(off[i]), int(off[i + 1])):
                forbidden[i][coloring[int(idx[k])]] = i
            for c in range(1, max_colors):
                if forbidden[i][c] != i:
                    out[i] = c
                    break
        temp = out
        coloring = list(temp)                            # update_coloring_GPU
        out = list(temp)
        for i in range(n):                               # conflict_detection
            if coloring[i] == 0:
                continue
            for k in range(int(off[i]), int(off[i + 1])):
                w = int(idx[k])
                if coloring[i] == coloring[w] and i > w:
                    out[i] = 0
                    break
        temp = out
        coloring = list(temp)                            # update_coloring_GPU
        uncolored = any(c == 0 for c in coloring)        # check_uncolored_nodes
        if uncolored and rounds > 4 * max_colors + 64:
            raise RuntimeError("no progress")
    return np.array(coloring, dtype=np.uint32), rounds


def small_graphs():
    out = []
    for n, p in [(1, 0.5), (6, 0.9), (40, 0.3), (120, 0.1), (200, 0.5)]:
        O.srand(1)
        out.append(O.setup_rnd2(n, p))
    return out


@pytest.mark.parametrize("k", range(5))
def test_restatement_matches_literal_kernels(k):
    off, idx = small_graphs()[k]
    a, ra = NP.greedy_ff(off, idx)
    b, rb = literal_greedy_ff(off, idx)
    assert a.tolist() == b.tolist() and ra == rb


def test_full_forbidden_set_is_reported():
    """K2: colours stop at maxDeg = 1, so node 1 can never be coloured -- the reference loops
    forever (coloringGreedyFF.cu:17, :122-127); the restatements stop and say so."""
    off, idx = np.array([0, 1, 2], dtype=np.uint64), np.array([1, 0], dtype=np.uint32)
    with pytest.raises(RuntimeError):
        NP.greedy_ff(off, idx)
    with pytest.raises(RuntimeError):
        literal_greedy_ff(off, idx)


def asymmetric_graph(n=400, arcs=2400, seed=5):
    """Directed arcs without their reverse (mcmc_graph_upload accepts any CSR), rows ascending."""
    rng = np.random.default_rng(seed)
    E = set()
    while len(E) < arcs:
        a, b = (int(x) for x in rng.integers(0, n, 2))
        if a != b:
            E.add((a, b))
    E = sorted(E)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.add.at(off, np.array([a for a, _ in E]) + 1, 1)
    return np.cumsum(off).astype(np.uint64), np.array([b for _, b in E], dtype=np.uint32)


def test_restatement_matches_literal_kernels_asymmetric():
    """On an asymmetric CSR an older node can lose to a fresh smaller neighbour whose row lacks it."""
    off, idx = asymmetric_graph()
    a, ra = NP.greedy_ff(off, idx)
    b, rb = literal_greedy_ff(off, idx)
    assert a.tolist() == b.tolist() and ra == rb


def test_restatement_is_a_proper_colouring():
    O.srand(1)
    off, idx = O.setup_rnd2(1500, 0.05)
    c, r = NP.greedy_ff(off, idx)
    rows = np.repeat(np.arange(len(off) - 1), np.diff(off.astype(np.int64)))
    assert not np.any(c[rows] == c[idx]) and c.min() >= 1 and c[0] == 1
    assert c.max() <= np.diff(off.astype(np.int64)).max() + 1 and r >= 1


# ---------------------------------------------------------------------------------------------
# GPU


def _gpu(off, idx):
    import mcmc_colorer_amd.colorer as M

    g = M.Graph.from_csr(off, idx)
    col = M.ColoringGreedyFF(g)
    col.run()
    return col


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1, 0.5), (300, 0.1), (2000, 0.02), (1200, 0.6)])
def test_gpu_greedyff_simulate(hip_lib, n, p):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    col = _gpu(off, idx)
    c, r = NP.greedy_ff(off, idx)
    assert col.colors.tolist() == c.tolist()
    assert col.rounds == r and col.numColors == len(set(c.tolist()))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6, 7])
def test_gpu_greedyff_asymmetric_csr(hip_lib, seed):
    """the fresh-only conflict scan is valid on symmetric CSRs only; an asymmetric one
    scans every coloured row, as conflict_detection (coloringGreedyFF.cu:134-163) does."""
    off, idx = asymmetric_graph(seed=seed)
    col = _gpu(off, idx)
    c, r = NP.greedy_ff(off, idx)
    assert col.colors.tolist() == c.tolist() and col.rounds == r


@pytest.mark.gpu
def test_gpu_vff_asymmetric_csr(hip_lib):
    import mcmc_colorer_amd.colorer as M

    off, idx = asymmetric_graph(seed=8)
    col = M.ColoringVFF(M.Graph.from_csr(off, idx))
    col.run()
    c, K, it, valid = NP.vff(off, idx)
    assert col.colors.tolist() == c.tolist() and (col.numColors, col.iterations, col.valid) == (K, it, valid)


@pytest.mark.gpu
def test_gpu_greedyff_full_forbidden_set_fails_loudly(hip_lib):
    import mcmc_colorer_amd.colorer as M

    off, idx = np.array([0, 1, 2], dtype=np.uint64), np.array([1, 0], dtype=np.uint32)
    with pytest.raises(Exception, match="no progress"):
        M.ColoringGreedyFF(M.Graph.from_csr(off, idx)).run()


@pytest.mark.gpu
def test_gpu_greedyff_power_law(hip_lib):
    off, idx = NP.rmat(13, 8, 0.5, 0.2, 0.2, 3)   # hubs: wide forbidden sets, many rounds
    col = _gpu(off, idx)
    c, r = NP.greedy_ff(off, idx)
    assert col.colors.tolist() == c.tolist() and col.rounds == r


@pytest.mark.gpu
def test_cli_grdffgpu_files(hip_lib, tmp_path):
    """--grdffgpu writes <graph>-GFF-<i>.log / -colors.txt (main.cu:111-132) with the restated colours."""
    exe = ROOT / "mcmc_colorer_amd" / "mcmc_colorer"
    r = subprocess.run([str(exe), "--grdffgpu", "--simulate", "0.1", "-n", "300", "--seed", "1",
                        "--outDir", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    O.srand(1)
    off, idx = O.setup_rnd2(300, 0.1)
    c, _ = NP.greedy_ff(off, idx)
    name = "300_0.100000_1.000000"
    lines = (tmp_path / f"{name}-GFF-0-colors.txt").read_text().split("\n")
    assert [int(x.split()[1]) for x in lines if x] == c.tolist()
    log = (tmp_path / f"{name}-GFF-0.log").read_text()
    assert f"Number of colors: {len(set(c.tolist()))}" in log
    assert f"Parallel Greedy First Fit - number of colors: {len(set(c.tolist()))}" in r.stdout
