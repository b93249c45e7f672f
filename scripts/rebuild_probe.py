"""The dense sweep's count rebuild at C3 (configs[2]: n 1e7, p 0.001, 32 colours): first-sweep minus
second-sweep device time of a fresh colouring, per rebuild form (the lane rebuild kernel over the
tile-transposed ids, the same over the layout with MCMC_DC_TID=0, MCMC_DENSE_RB=1 the chunk rebuild
inside the sweep), and the forms' counts compared on sampled rows. Usage:
    python scripts/rebuild_probe.py [reps]"""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import mcmc_colorer_amd.colorer as M  # noqa: E402
from mcmc_colorer_amd._lib import check, lib, u32ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = 10_000_000
t0 = time.perf_counter()
g = M.Graph.er_fast(n, 0.001, 1)
print(f"graph {time.perf_counter() - t0:.1f} s, {g.nEdges} arcs", flush=True)
rows = np.unique(np.concatenate([np.arange(0, 70000), np.arange(n - 5000, n),
                                 np.random.default_rng(1).integers(0, n, 50000)])).astype(np.uint32)
out = {}
counts = {}
FORMS = {"transposed": {}, "lanes": {"MCMC_DC_TID": "0"}, "chunks": {"MCMC_DENSE_RB": "1"}}
for form, env in FORMS.items():
    for k in ("MCMC_DENSE_RB", "MCMC_DC_TID"):
        os.environ.pop(k, None)
    os.environ.update(env)
    t1 = time.perf_counter()
    col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32))
    print(form, f"context set-up {time.perf_counter() - t1:.2f} s", col.dense_stats()["transposed_ids"], flush=True)
    res = []
    for r in range(reps):
        col.init(r)
        s1 = col.step(1)
        s2 = col.step(1)
        res.append((s1.loopMs, s2.loopMs))
        print(form, r, f"first {s1.loopMs:.3f} ms second {s2.loopMs:.3f} ms rebuild {s1.loopMs - s2.loopMs:.3f} ms",
              flush=True)
    col.init(0)
    col.step(1)
    cnt = np.zeros((len(rows), 32), dtype=np.uint32)
    buf = np.zeros(32, dtype=np.uint32)
    # rows one at a time would be slow: contiguous runs
    runs = np.split(rows, np.nonzero(np.diff(rows) != 1)[0] + 1)
    k = 0
    for run in runs:
        b = np.zeros((len(run), 32), dtype=np.uint32)
        check(lib().mcmc_get_dense_counts(col._ctx, int(run[0]), len(run), u32ptr(b), None))
        cnt[k:k + len(run)] = b
        k += len(run)
    counts[form] = cnt
    out[form] = {"rebuild_ms": [a - b for a, b in res], "first_ms": [a for a, _ in res], "second_ms": [b for _, b in res],
                 "dense": col.dense_stats()}
    col.close()
same = all(bool(np.array_equal(counts[f], counts["chunks"])) for f in FORMS)
out["sampled_rows"] = int(len(rows))
out["counts_equal"] = same
out["mean_s_count"] = float(counts["lanes"].sum(axis=1).mean())
print(json.dumps(out), flush=True)
sys.exit(0 if same else 1)
