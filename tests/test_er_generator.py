"""The build's counter-based G(n, p) (mcmc_colorer_amd/csrc/er_gen.h) for C3/C4-scale runs.

Not a reference function (setupRnd2 is infeasible at n = 1e7; "parity is
GPU-vs-restatement on the same graph"). CPU: the C oracle's restatement (oracle_er_fast) is pinned
by an independent numpy restatement (oracle/oracle_np.er_fast) and by the G(n, p) statistics.
"""
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as O

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import oracle_np as NP  # noqa: E402

CASES = [(1000, 0.05, 7), (70000, 0.0005, 3), (131073, 0.0002, 11), (300, 1.0, 1), (500, 0.0, 1), (2, 0.5, 9),
         (65537, 0.001, 2)]


def csr_from_edges(n, E):
    deg = np.zeros(n + 1, np.int64)
    np.add.at(deg, E[:, 0] + 1, 1)
    np.add.at(deg, E[:, 1] + 1, 1)
    src = np.concatenate([E[:, 0], E[:, 1]])
    dst = np.concatenate([E[:, 1], E[:, 0]])
    return np.cumsum(deg), dst[np.lexsort((dst, src))]


@pytest.mark.parametrize("n,p,seed", CASES)
def test_oracle_generator_matches_numpy_restatement(n, p, seed):
    off, idx = O.er_fast(n, p, seed)
    offn, idxn = csr_from_edges(n, NP.er_fast(n, p, seed))
    assert np.array_equal(off.astype(np.int64), offn)
    assert np.array_equal(idx.astype(np.int64), idxn)


def test_generator_statistics():
    """G(n, p): arc count within 5 sigma of p n (n-1); simple graph (no loops, no duplicates);
    degrees across the 65536-column block boundary show no seam; seeds give different graphs."""
    n, p = 131073, 0.0002
    off, idx = O.er_fast(n, p, 11)
    m = len(idx)
    mean = p * n * (n - 1)
    assert abs(m - mean) < 5 * np.sqrt(2 * mean)
    rows = np.repeat(np.arange(n), np.diff(off.astype(np.int64)))
    assert not np.any(rows == idx)
    pairs = rows.astype(np.int64) * n + idx
    assert len(np.unique(pairs)) == m
    deg = np.diff(off.astype(np.int64))
    assert abs(deg[:65536].mean() - deg[65536:].mean()) < 5 * np.sqrt(p * n / 65536)
    off2, idx2 = O.er_fast(n, p, 12)
    assert not (len(idx2) == m and np.array_equal(idx2, idx))
