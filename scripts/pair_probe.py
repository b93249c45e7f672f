"""Per-pair trace of the tiled early-exit sweep (MCMC_PAIR_TRACE, the diagnostics instantiation):
C3 (configs[2]) or C2 (configs[1]); writes <out>.trace (summarise with pair_trace_summary.py) and
prints the sweep time of the traced instantiation and of the plain one."""
import ctypes
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    cfg, out = sys.argv[1], sys.argv[2]
    import torch

    torch.cuda.init()
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    if cfg == "c3":
        g = M.Graph.er_fast(10_000_000, 0.001, 1)
        ncol = 32
    else:
        g = M.Graph.simulate(100000, 0.01, M.GlibcRand(1))
        ncol = 16
    res = {"config": cfg}
    for mode in ("plain", "trace"):
        if mode == "trace":
            os.environ["MCMC_PAIR_TRACE"] = out + ".trace"
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=0x7FFFFFF0))
        col.init(0)
        tot, ker = ctypes.c_double(), ctypes.c_double()
        check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot), ctypes.byref(ker)))
        check(lib().mcmc_bench_sweeps(col._ctx, 10, ctypes.byref(tot), ctypes.byref(ker)))
        res[mode + "_ms"] = ker.value
        col.close()
        os.environ.pop("MCMC_PAIR_TRACE", None)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
