"""The C3 count rebuild (dc_rebuild_kernel over the tile-transposed ids) twice, for rocprofv3 counter
passes: python scripts/rb_sq_probe.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import mcmc_colorer_amd.colorer as M  # noqa: E402

n = 10_000_000
g = M.Graph.er_fast(n, 0.001, 1)
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32))
for r in range(2):
    col.init(r)
    s1 = col.step(1)
    print(r, s1.loopMs, flush=True)
col.close()
