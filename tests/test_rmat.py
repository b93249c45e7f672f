"""R-MAT power-law stand-in for configs[4] (csrc/er_gen.h rmat_edge).

SNAP LiveJournal / Reddit are not in the container, so C5 runs on this generator. CPU: the numpy
restatement (oracle/oracle_np.rmat) is pinned by the Philox4x32-10 known-answer vectors of its
authors (Random123, SC'11) and by structural properties of the output. GPU: the device generator
(mcmc_graph_rmat) reproduces the restatement's CSR exactly, and the colorer matches the oracle on it
with the reference's default nCol = maxDeg (wide sweep).
"""
import numpy as np
import pytest

import oracle_np as NP
import oracle_ref as O

M32 = 0xFFFFFFFF


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((M32, M32, M32, M32), (M32, M32), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, out):
    r = NP._philox4x32_10(*[np.array([c], dtype=np.uint64) for c in ctr], key[0], key[1])
    assert tuple(int(x[0]) for x in r) == out


@pytest.mark.parametrize("scale,ef", [(1, 4), (6, 8), (12, 10)])
def test_rmat_restatement_structure(scale, ef):
    off, idx = NP.rmat(scale, ef, 0.5, 0.2, 0.2, 3)
    n = 1 << scale
    assert len(off) == n + 1 and off[0] == 0 and off[-1] == len(idx)
    rows = np.repeat(np.arange(n), np.diff(off.astype(np.int64)))
    assert not np.any(rows == idx)                              # no self-loops
    keys = rows.astype(np.int64) * n + idx
    assert np.all(np.diff(keys) > 0)                            # ascending rows, no duplicates
    rev = np.sort(idx.astype(np.int64) * n + rows)
    assert np.array_equal(rev, keys)                            # symmetric
    assert len(idx) <= 2 * ef * n


def test_rmat_is_power_law_like():
    off, idx = NP.rmat(14, 10, 0.5, 0.2, 0.2, 1)
    d = np.diff(off.astype(np.int64))
    assert d.max() > 20 * d.mean()                              # hubs
    assert np.median(d) < d.mean()                              # heavy tail
    off2, _ = NP.rmat(14, 10, 0.5, 0.2, 0.2, 2)
    assert not np.array_equal(off, off2)                        # the seed matters


@pytest.mark.gpu
@pytest.mark.parametrize("scale,ef,seed", [(0, 4, 1), (3, 2, 1), (9, 16, 5), (15, 10, 1)])
def test_gpu_rmat_matches_restatement(hip_lib, scale, ef, seed):
    import mcmc_colorer_amd.colorer as M

    g = M.Graph.rmat(scale, ef, 0.5, 0.2, 0.2, seed)
    s = g.getStruct()
    off, idx = NP.rmat(scale, ef, 0.5, 0.2, 0.2, seed)
    assert np.array_equal(s.cumulDegs, off)
    assert np.array_equal(s.neighs[: len(idx)], idx)
    assert g.getMaxNodeDeg() == (int(np.diff(off.astype(np.int64)).max()) if len(off) > 1 else 0)


@pytest.mark.gpu
def test_gpu_colorer_on_rmat_default_ncol(hip_lib):
    """configs[4] in miniature: power-law graph, nCol = maxDeg (main.cu:162), convergent run."""
    import mcmc_colorer_amd.colorer as M

    off, idx = NP.rmat(13, 10, 0.5, 0.2, 0.2, 1)
    g = M.Graph.from_csr(off, idx)
    ncol = g.getMaxNodeDeg()
    assert ncol > 256
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol))
    st = col.run(0)
    O.srand(1)
    r = O.mcmc_run(off, idx, ncol, 1)
    assert col.coloring().tolist() == r.colors.tolist()
    assert col.trajectory().tolist() == r.traj.tolist()
    assert (st.iter, st.finalViol, st.glibcDraws) == (r.res.iter, r.res.finalViol, r.res.glibcDraws)
