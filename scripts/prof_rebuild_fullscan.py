"""C3 (configs[2]: n 1e7, p 0.001, 32 colours) under rocprofv3: the count rebuild of a fresh colouring
(dc_rebuild_kernel, 2 colourings) and the full-scan sweep (MCMC_FULL_SCAN=1: sweep_tiled_kernel over
every arc, 2 warm-up + 5 timed sweeps), each with its host-timed figure printed beside. Run under
`rocprofv3 --kernel-trace --stats` and, separately, `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
(scripts/gpu_prof_r06.sh)."""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import mcmc_colorer_amd.colorer as M  # noqa: E402
from mcmc_colorer_amd._lib import check, lib  # noqa: E402

n = 10_000_000
t0 = time.perf_counter()
g = M.Graph.er_fast(n, 0.001, 1)
print(f"graph {time.perf_counter() - t0:.1f} s", flush=True)
out = {"rebuild_ms": []}
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32))
for r in range(2):
    col.init(r)
    s1 = col.step(1)
    s2 = col.step(1)
    out["rebuild_ms"].append(s1.loopMs - s2.loopMs)
ds = col.dense_stats()
out["dense_range"] = [ds["s0"], ds["s1"]]
col.close()
os.environ["MCMC_FULL_SCAN"] = "1"
os.environ["MCMC_DENSE"] = "0"
cf = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=32, maxRip=0x7FFFFFF0))
cf.init(0)
tot, ker = ctypes.c_double(), ctypes.c_double()
check(lib().mcmc_bench_sweeps(cf._ctx, 2, ctypes.byref(tot), ctypes.byref(ker)))
check(lib().mcmc_bench_sweeps(cf._ctx, 5, ctypes.byref(tot), ctypes.byref(ker)))
info = cf.info()
out["full_scan"] = {"ms_per_sweep": ker.value, "layout_bytes": info["sweep_bytes"],
                    "frac_of_8TBs": info["sweep_bytes"] / (ker.value * 1e-3) / 8e12}
cf.close()
print(json.dumps(out), flush=True)
