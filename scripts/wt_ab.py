"""A/B of the wide tiled sweep's block rotation (MCMC_WT_ROTATE) at C3 with nCol = maxDeg."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import mcmc_colorer_amd.colorer as M  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001
g = M.Graph.er_fast(n, p, 1)
ncol = M.default_ncol(g, M.ColoringMCMCParams(nCol=0))
print(f"n={n} m={g.nEdges} nCol={ncol}", flush=True)
for rot in ("1", "0", "1"):
    os.environ["MCMC_WT_ROTATE"] = rot
    col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol))
    col.init(0)
    ms = []
    for _ in range(4):
        t0 = time.perf_counter()
        col.step(1)
        ms.append((time.perf_counter() - t0) * 1e3)
    print(f"rotate={rot} variant={col.info()['variant']} step ms {[round(x, 1) for x in ms]} traj {col.trajectory().tolist()}", flush=True)
    col.close()
