"""The reference's Luby colorer (ColoringLuby::run_fast, `--lubygpu`;
graph_coloring/coloringLubyFast.cu, coloringLuby.cu).

CPU: the vectorised restatement (oracle/oracle_np.py::luby) against a literal per-thread
restatement of the kernels (set_initial_distr_k, check_conflicts_fast_k, update_eligible_fast_k,
check_finished_k, add_color_and_check_uncolored_k, prune_eligible_clear_is), both from the XORWOW
states of curand_init(seed, v, 0) (tests/test_xorwow.py pins them). The reference's conflict kernel
clears flags in place, so its result depends on thread timing; both restatements take the
schedule in which every read precedes every write (the snapshot), as the HIP colorer does.
GPU: the HIP colorer (csrc/luby.hip) against the restatement -- colours, colour count, inner
rounds and the advanced states -- on --simulate and power-law graphs, repetitions sharing the
states, and the CLI's -LUBY- files. The reference publishes no outputs for this colorer and its
result is timing-dependent: parity is pinned by the two restatements, not by reference runs.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O

ROOT = Path(__file__).resolve().parent.parent


def init_states(n, seed):
    return np.stack([O.xorwow_init(seed, v) for v in range(n)]).astype(np.uint32)


def literal_luby(off, idx, states):
    """The kernels as written, thread idx of each launch in turn; check_conflicts reads the draw's
    flags (i_i_in) and writes a copy (i_i)."""
    n = len(off) - 1
    deg = [int(off[i + 1]) - int(off[i]) for i in range(n)]
    coloring = [0] * n
    cands = [1] * n                                   # run_fast :30-33
    is_ = [0] * n
    num = rounds = 0
    uncolored = True
    while uncolored:
        for i in range(n):                            # prune_eligible_clear_is
            cands[i] = 1 if coloring[i] == 0 else 0
            is_[i] = 0
        node_left = True
        while node_left:
            rounds += 1
            i_i_in = [0] * n
            for i in range(n):                        # set_initial_distr_k
                u = NP.curand_uniform(NP.xorwow_step(states[i:i + 1]))[0]
                i_i_in[i] = (1 if cands[i] else 0) if u < 0.5 else 0
            i_i = list(i_i_in)
            for i in range(n):                        # check_conflicts_fast_k
                if i_i_in[i] == 0:
                    continue
                for j in range(deg[i]):
                    nb = int(idx[int(off[i]) + j])
                    if i_i_in[nb] == 1:
                        if deg[i] <= deg[nb]:
                            i_i[i] = 0
                        else:
                            i_i[nb] = 0
            for i in range(n):                        # update_eligible_fast_k
                is_[i] |= i_i[i]
                if i_i[i] == 0:
                    continue
                cands[i] = 0
                for j in range(deg[i]):
                    cands[int(idx[int(off[i]) + j])] = 0
            node_left = any(cands)                    # check_finished_k
        num += 1
        uncolored = False
        for i in range(n):                            # add_color_and_check_uncolored_k
            if is_[i] == 1:
                coloring[i] = num
            if coloring[i] == 0:
                uncolored = True
    return np.array(coloring, dtype=np.uint32), num, rounds


def small_graphs():
    out = []
    for n, p in [(1, 0.5), (2, 1.0), (7, 0.9), (60, 0.2), (150, 0.05)]:
        O.srand(1)
        out.append(O.setup_rnd2(n, p))
    return out


@pytest.mark.parametrize("k", range(5))
def test_restatement_matches_literal_kernels(k):
    off, idx = small_graphs()[k]
    n = len(off) - 1
    s1, s2 = init_states(n, 3), init_states(n, 3)
    a = NP.luby(off, idx, s1)
    b = literal_luby(off, idx, s2)
    assert a[0].tolist() == b[0].tolist() and a[1:] == b[1:]
    assert np.array_equal(s1, s2)


def test_restatement_is_a_proper_colouring():
    O.srand(1)
    off, idx = O.setup_rnd2(800, 0.05)
    c, k, r = NP.luby(off, idx, init_states(800, 1))
    rows = np.repeat(np.arange(800), np.diff(off.astype(np.int64)))
    assert not np.any(c[rows] == c[idx]) and c.min() == 1 and c.max() == k and r >= k


def test_self_loop_is_reported():
    """A node adjacent to itself is dropped by its own conflict check every time it is selected
    (deg <= deg): the reference spins; the restatement stops and says so."""
    off, idx = np.array([0, 1], dtype=np.uint64), np.array([0], dtype=np.uint32)
    with pytest.raises(RuntimeError):
        NP.luby(off, idx, init_states(1, 1), max_stale=50)


# ---------------------------------------------------------------------------------------------
# GPU


@pytest.fixture
def M(hip_lib):
    import mcmc_colorer_amd.colorer as M

    return M


def _check(M, off, idx, seed, reps=1):
    g = M.Graph.from_csr(off, idx)
    states = M.CurandStates(g.nNodes, seed)
    ref = states.states()
    for _ in range(reps):
        col = M.ColoringLuby(g, states)
        col.run_fast()
        c, k, r = NP.luby(off, idx, ref)
        assert col.colors.tolist() == c.tolist()
        assert col.numOfColors == k and col.rounds == r
        assert np.array_equal(states.states(), ref)
    states.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1, 0.5), (2, 1.0), (300, 0.1), (2000, 0.02), (1200, 0.6)])
def test_gpu_luby_simulate(M, n, p):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    _check(M, off, idx, 1)


@pytest.mark.gpu
def test_gpu_luby_repetitions_share_states(M):
    """main.cu:80,91: every repetition's colorer draws from the same, advanced GPURand states."""
    O.srand(2)
    off, idx = O.setup_rnd2(500, 0.05)
    _check(M, off, idx, 7, reps=3)


@pytest.mark.gpu
def test_gpu_luby_power_law(M):
    off, idx = NP.rmat(13, 8, 0.5, 0.2, 0.2, 3)   # hubs: long rows in the conflict and update waves
    _check(M, off, idx, 5)


@pytest.mark.gpu
def test_gpu_luby_self_loop_fails_loudly(M):
    off, idx = np.array([0, 1, 2], dtype=np.uint64), np.array([0, 0], dtype=np.uint32)
    g = M.Graph.from_csr(off, idx)
    states = M.CurandStates(2, 1)
    with pytest.raises(Exception, match="no progress"):
        M.ColoringLuby(g, states).run_fast()


@pytest.mark.gpu
def test_cli_lubygpu_files(hip_lib, tmp_path):
    """--lubygpu writes <graph>-LUBY-<i>.log / -colors.txt (main.cu:89-109); two repetitions draw
    from the same states (the second continues where the first stopped)."""
    exe = ROOT / "mcmc_colorer_amd" / "mcmc_colorer"
    r = subprocess.run([str(exe), "--lubygpu", "--simulate", "0.1", "-n", "300", "--seed", "1", "--repet", "2",
                        "--outDir", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    O.srand(1)
    off, idx = O.setup_rnd2(300, 0.1)
    st = init_states(300, 1)
    name = "300_0.100000_1.000000"
    for i in range(2):
        c, k, _ = NP.luby(off, idx, st)
        lines = (tmp_path / f"{name}-LUBY-{i}-colors.txt").read_text().split("\n")
        assert [int(x.split()[1]) for x in lines if x] == c.tolist()
        log = (tmp_path / f"{name}-LUBY-{i}.log").read_text()
        assert log.startswith("Luby Colorer - GPU version - Report")
        assert f"Number of colors: {k}" in log
        assert f"LubyGPU - number of colors: {k}" in r.stdout
