"""Generates tests/golden/*.json from the oracle (oracle/mcmc_cpu_ref.cpp) -- TEST INFRASTRUCTURE.

The reference ships no golden vectors and executing it was refused, so these
fixtures are the oracle restatement's own outputs on BASELINE.json's configs (C1 in full; C2 as
hashes + trajectory) and on small hand-sized cases. The oracle itself is pinned by KATs and by
the independent numpy restatement (tests/test_oracle.py).

    python tests/golden/make_golden.py [--c2]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle_ref as O  # noqa: E402

SMALL_CASES = [
    # name, n, p, nCol (0 = maxDeg), seed, epsilon, maxRip, taboo, tailcut
    ("k_small_a", 200, 0.05, 0, 3, 1e-8, 250, 0, False),
    ("k_small_b", 300, 0.2, 12, 5, 1e-8, 40, 0, False),
    ("k_taboo", 250, 0.1, 0, 9, 1e-8, 250, 3, False),
    ("k_tailcut", 400, 0.05, 6, 2, 1e-8, 60, 0, True),
    ("k_events", 300, 0.3, 7, 11, 3.3e6, 30, 0, False),
    ("k_events_taboo", 500, 0.02, 5, 13, 3.3e6, 40, 2, False),
    ("k_ncol2", 150, 0.01, 2, 17, 1e-8, 30, 0, False),
    ("k_ncol_gt64", 500, 0.3, 90, 4, 1e-8, 20, 2, False),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case(name, n, p, ncol, seed, eps, maxrip, taboo, tailcut, full=True):
    O.srand(1)                            # --seed given: glibc stays unseeded (ArgHandle.cpp:272-276)
    off, idx = O.setup_rnd2(n, p)
    nc = ncol or O.max_deg(off)
    r = O.mcmc_run(off, idx, nc, seed, epsilon=eps, maxRip=maxrip, tabooIteration=taboo, tailcut=tailcut,
                   nthreads=1 if n <= 5000 else 8)
    d = dict(name=name, n=n, prob=p, nCol=nc, seed=seed, epsilon=eps, maxRip=maxrip, tabooIteration=taboo,
             tailcut=tailcut, m=int(len(idx)), maxDeg=O.max_deg(off),
             row_off_sha256=sha(off.astype(np.uint64)), col_idx_sha256=sha(idx.astype(np.uint32)),
             init_sha256=sha(r.init), colors_sha256=sha(r.colors), traj=[int(x) for x in r.traj],
             iter=int(r.res.iter), maxIterReached=bool(r.res.maxIterReached), finalViol=int(r.res.finalViol),
             glibcDraws=int(r.res.glibcDraws), initDraws=int(r.res.initDraws))
    if full:
        d["colors"] = [int(x) for x in r.colors]
    return d


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", action="store_true", help="also the n=1e5 C2 fixture (~2 min)")
    a = ap.parse_args()
    out = {"c1": case("c1", 1000, 0.1, 0, 1, 1e-8, 250, 0, False)}
    for c in SMALL_CASES:
        out[c[0]] = case(*c)
    (HERE / "small.json").write_text(json.dumps(out, indent=1))
    print("wrote small.json")
    if a.c2:
        t = time.time()
        d = case("c2", 100000, 0.01, 16, 1, 1e-8, 250, 0, False, full=False)
        d["seconds"] = time.time() - t
        (HERE / "c2.json").write_text(json.dumps(d, indent=1))
        print("wrote c2.json", d["seconds"])


if __name__ == "__main__":
    main()
