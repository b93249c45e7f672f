"""Early-exit scan probe: sweep time and scanned bytes of the tiled sweep with the exact early exit
(default) and with MCMC_FULL_SCAN=1, on configs[1] (C2) and configs[2] (C3). One JSON line per run."""
import ctypes
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    import torch

    torch.cuda.init()
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    if cfg == "c3":
        g = M.Graph.er_fast(10_000_000, 0.001, 1)
        ncol, steps = 32, 20
    else:
        g = M.Graph.simulate(100000, 0.01, M.GlibcRand(1))
        ncol, steps = 16, 200
    for full in os.environ.get("MCMC_PROBE_MODES", "0,1").split(","):
        os.environ["MCMC_FULL_SCAN"] = full
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=0x7FFFFFF0))
        col.init(0)
        tot, ker = ctypes.c_double(), ctypes.c_double()
        check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot), ctypes.byref(ker)))
        check(lib().mcmc_bench_sweeps(col._ctx, steps, ctypes.byref(tot), ctypes.byref(ker)))
        ms = ker.value
        check(lib().mcmc_set_scan_stats(col._ctx, 1))
        check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot), ctypes.byref(ker)))
        q, p = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().mcmc_get_scan_stats(col._ctx, ctypes.byref(q), ctypes.byref(p)))
        info = col.info()
        print(json.dumps({"config": cfg, "full_scan": full == "1", "ms_per_sweep": ms,
                          "vu_per_s": g.nNodes / (ms * 1e-3), "quads_per_sweep": q.value / 3,
                          "pairs_per_sweep": p.value / 3, "id_bytes_per_sweep": 16 * q.value / 3,
                          "layout_bytes": info["layout_bytes"], "ngroups": info["ngroups"], "nblocks": info["nblocks"]}),
              flush=True)
        col.close()


if __name__ == "__main__":
    main()
