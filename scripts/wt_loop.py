"""C3 at the reference's default colour count (nCol = maxDeg): the reference's whole loop from C_0
(run(), maxRip 250) on the wide sweep over the tiled layout -- device time, sweeps, the final Cviol and
how many sweeps ran from the incremental counts. Usage: python scripts/wt_loop.py"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import mcmc_colorer_amd.colorer as M  # noqa: E402

n = 10_000_000
t0 = time.perf_counter()
g = M.Graph.er_fast(n, 0.001, 1)
print(f"graph {time.perf_counter() - t0:.1f} s, nCol = maxDeg = {g.maxDeg}", flush=True)
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.maxDeg))
col.init(0)
st = col.run(0)
traj = [int(x) for x in col.trajectory()]
ws = col.wide_inc_stats()
print(json.dumps({"loop_ms": st.loopMs, "sweeps_run": int(st.sweepsRun), "iter": int(st.iter),
                  "final_Cviol": int(st.finalViol), "max_iter_reached": bool(st.maxIterReached),
                  "incremental_sweeps": ws["incremental_sweeps"], "full_sweeps": ws["full_sweeps"],
                  "trajectory_head": traj[:8], "trajectory_tail": traj[-4:]}), flush=True)
