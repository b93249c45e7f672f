"""Column-block / group-size probe for the early-exit tiled sweep: a G(n, p) with C3's per-block
density (65 arcs per row and 2^16-column block) small enough for a CSR, swept with several
(MCMC_BLOCK_LOG2, MCMC_GROUP_ROWS) layouts. Every variant must give the same trajectory and
colouring; one JSON line per variant (ms/sweep, pairs, quads)."""
import ctypes
import hashlib
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    n = int(os.environ.get("PROBE_N", "2000000"))
    p = float(os.environ.get("PROBE_P", "0.001"))
    ncol = int(os.environ.get("PROBE_NCOL", "32"))
    variants = os.environ.get("PROBE_VARIANTS", "16:,16:1563,15:,14:").split(",")
    import torch

    torch.cuda.init()
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    g = M.Graph.er_fast(n, p, 1)
    check(lib().mcmc_graph_materialize_csr(g.handle))
    ref = None
    for var in variants:
        bl, rows = var.split(":")
        for k, v in (("MCMC_BLOCK_LOG2", bl), ("MCMC_GROUP_ROWS", rows)):
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=0x7FFFFFF0))
        col.init(0)
        tot, ker = ctypes.c_double(), ctypes.c_double()
        check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot), ctypes.byref(ker)))
        h = hashlib.sha1(col.coloring().tobytes()).hexdigest()[:12]
        check(lib().mcmc_bench_sweeps(col._ctx, 20, ctypes.byref(tot), ctypes.byref(ker)))
        ms = ker.value
        check(lib().mcmc_set_scan_stats(col._ctx, 1))
        check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot), ctypes.byref(ker)))
        q, pr = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().mcmc_get_scan_stats(col._ctx, ctypes.byref(q), ctypes.byref(pr)))
        info = col.info()
        same = ref is None or ref == h
        ref = ref or h
        print(json.dumps({"variant": var, "ms_per_sweep": ms, "vu_per_s": g.nNodes / (ms * 1e-3),
                          "quads": q.value / 3, "pairs": pr.value / 3, "grp_rows": info["grp_rows"],
                          "ngroups": info["ngroups"], "nblocks": info["nblocks"], "sub_log2": info["sub_log2"],
                          "lds": info["lds_bytes"], "C3_hash": h, "same_as_first": same}), flush=True)
        col.close()
        if not same:
            sys.exit(3)


if __name__ == "__main__":
    main()
