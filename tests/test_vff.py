"""The reference's greedy colorer with vertex-first-fit rebalancing (ColoringVFF, `--vffgpu`;
graph_coloring/coloringVFF.cu).

CPU: the vectorised restatement (oracle/oracle_np.py::vff) against a literal per-thread
restatement of run_balancing and its kernels with the reference's own data structures (forbidden
rows flagged with the node id over a zero memset, cumulative bin sizes read through BIN_SIZE,
update_bins + inclusive scan, the ten-row unbalanced history shifted every iteration and
ensure_not_looping over it). The greedy phase is greedy_ff (tests/test_greedyff.py pins it).
GPU: the HIP colorer (csrc/greedyff.hip, mcmc_vff_run) against the restatement -- colours, colour
count, iterations, valid -- and the CLI's -VFF- files. The reference publishes no outputs for this
colorer: parity is pinned by the two restatements, not by reference runs.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O

ROOT = Path(__file__).resolve().parent.parent
HIST = 10   # UNBALANCED_HISTORY


def literal_balancing(off, idx, coloring):
    """run_balancing (:101-228) from the greedy colouring, thread idx of each launch in turn."""
    n = len(off) - 1
    coloring = [int(c) for c in coloring]
    K = len(set(coloring))
    cumul = [0] * (K + 1)                                    # convert_to_standard_notation
    for c in range(1, K + 1):
        cumul[c] = coloring.count(c)
    for c in range(2, K + 1):
        cumul[c] += cumul[c - 1]
    bsize = lambda i: cumul[i] - cumul[i - 1]                # BIN_SIZE
    gamma = n // K
    unb = [[False] * n for _ in range(HIST)]
    temp = list(coloring)
    for i in range(n):                                       # detect_unbalanced_nodes
        if gamma < bsize(coloring[i]):
            unb[0][i] = True
    unbalanced, not_looping, it = any(unb[0]), True, 0
    while unbalanced and not_looping:
        it += 1
        forb = [[0] * (K + 1) for _ in range(n)]             # cudaMemset(forbiddenColors, 0)
        for i in range(n):                                   # tentative_rebalancing
            if not unb[0][i]:
                continue
            forb[i][coloring[i]] = i
            for k in range(int(off[i]), int(off[i + 1])):
                forb[i][coloring[int(idx[k])]] = i
            for c in range(1, K + 1):
                if forb[i][c] != i and gamma < bsize(c):
                    temp[i] = c
                    break
        for c in range(1, K + 1):                            # update_bins
            cumul[c] = sum(1 for i in range(n) if temp[i] == c)
        for i in range(n):                                   # solve_conflicts
            if not unb[0][i]:
                continue
            if not any(temp[int(idx[k])] == temp[i] and i > int(idx[k]) for k in range(int(off[i]), int(off[i + 1]))):
                unb[0][i] = False
        for c in range(1, K + 1):                            # thrust::inclusive_scan
            cumul[c] += cumul[c - 1]
        coloring = list(temp)                                # update_coloring_GPU
        unbalanced = any(unb[0])                             # is_unbalanced
        for r in range(HIST - 1, 0, -1):                     # the history shift
            unb[r] = list(unb[r - 1])
        if all(unb[0][v] == unb[o][v] for v in range(n) for o in range(1, HIST)):   # ensure_not_looping
            not_looping = False
    return coloring, K, it, not_looping


def small_graphs():
    out = []
    for n, p in [(1, 0.5), (6, 0.9), (40, 0.3), (120, 0.1), (300, 0.1)]:
        O.srand(1)
        out.append(O.setup_rnd2(n, p))
    return out


@pytest.mark.parametrize("k", range(5))
def test_restatement_matches_literal_kernels(k):
    off, idx = small_graphs()[k]
    c, K, it, valid = NP.vff(off, idx)
    g, _ = NP.greedy_ff(off, idx)
    lc, lK, lit, lvalid = literal_balancing(off, idx, g)
    assert (K, it, valid) == (lK, lit, lvalid)
    assert c.tolist() == (lc if lvalid else g.tolist())


def test_restatement_outcomes():
    """Both endings occur: a balanced result (valid) and a detected loop (greedy colours back)."""
    seen = set()
    for n, p in [(40, 0.3), (300, 0.1)]:
        O.srand(1)
        off, idx = O.setup_rnd2(n, p)
        c, K, it, valid = NP.vff(off, idx)
        seen.add(valid)
        if not valid:
            assert c.tolist() == NP.greedy_ff(off, idx)[0].tolist()
        assert c.min() >= 1 and c.max() <= K
    assert seen == {True, False}


# ---------------------------------------------------------------------------------------------
# GPU


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1, 0.5), (6, 0.9), (40, 0.3), (300, 0.1), (2000, 0.02), (1200, 0.6)])
def test_gpu_vff_simulate(hip_lib, n, p):
    import mcmc_colorer_amd.colorer as M

    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    col = M.ColoringVFF(M.Graph.from_csr(off, idx))
    col.run()
    c, K, it, valid = NP.vff(off, idx)
    assert col.colors.tolist() == c.tolist()
    assert (col.numColors, col.iterations, col.valid) == (K, it, valid)


@pytest.mark.gpu
def test_gpu_vff_power_law(hip_lib):
    import mcmc_colorer_amd.colorer as M

    off, idx = NP.rmat(13, 8, 0.5, 0.2, 0.2, 3)
    col = M.ColoringVFF(M.Graph.from_csr(off, idx))
    col.run()
    c, K, it, valid = NP.vff(off, idx)
    assert col.colors.tolist() == c.tolist() and (col.numColors, col.iterations, col.valid) == (K, it, valid)


@pytest.mark.gpu
def test_cli_vffgpu_files(hip_lib, tmp_path):
    """--vffgpu writes <graph>-VFF-<i>.log / -colors.txt (main.cu:134-158)."""
    exe = ROOT / "mcmc_colorer_amd" / "mcmc_colorer"
    r = subprocess.run([str(exe), "--vffgpu", "--simulate", "0.3", "-n", "40", "--seed", "1",
                        "--outDir", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    O.srand(1)
    off, idx = O.setup_rnd2(40, 0.3)
    c, K, _, valid = NP.vff(off, idx)
    name = "40_0.300000_1.000000"
    lines = (tmp_path / f"{name}-VFF-0-colors.txt").read_text().split("\n")
    assert [int(x.split()[1]) for x in lines if x] == c.tolist()
    log = (tmp_path / f"{name}-VFF-0.log").read_text()
    assert f"Valid result? (boolean) {int(valid)}" in log and f"Number of colors: {K}" in log
    hist = np.bincount(c, minlength=K + 1)[1:]
    assert all(f"{i + 1}\t: {h}" in log for i, h in enumerate(hist))
    assert f"Vertex-centric First Fit rebalancing after Greedy FF coloring - number of colors: {K}" in r.stdout
