"""C3 at the reference's default colour count (nCol = maxDeg ~ 10 500, the wide sweep over the tiled
layout): device time and Cviol of each sweep from C_0, and which sweeps ran from the incremental
violation counts (MCMC_WT_INC, wide_tiled.h). Usage: python scripts/wt_probe.py [sweeps]"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import mcmc_colorer_amd.colorer as M  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 10_000_000
t0 = time.perf_counter()
g = M.Graph.er_fast(n, 0.001, 1)
ncol = g.maxDeg
print(f"graph {time.perf_counter() - t0:.1f} s, nCol = maxDeg = {ncol}", flush=True)
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol))
col.init(0)
rows = []
for t in range(K):
    st = col.step(1)
    ws = col.wide_inc_stats()
    rows.append({"sweep": t, "ms": st.loopMs, "sweeps_run": int(st.sweepsRun), "inc": ws["incremental_sweeps"],
                 "full": ws["full_sweeps"], "changed": ws["changed_rows"], "walked": ws["changed_arcs"]})
    print(json.dumps(rows[-1]), flush=True)
    if st.sweepsRun == 0:
        break
traj = [int(x) for x in col.trajectory()]
print(json.dumps({"variant": col.info()["variant"], "nCol": ncol, "trajectory": traj, "per_sweep": rows}), flush=True)
