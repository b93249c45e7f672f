"""Per-rank sweep time of the partitioned C3/C4 run, measured on ONE GPU (no exchange).

Generates only rank r's rows of the C3 graph (mcmc_graph_er_fast_part) and times that rank's sweep
kernel alone (mcmc_bench_sweeps on a context over its rows). The sweep is the part of a C4 step
that must shrink 1/N for strong scaling; the exchange (one all-gather of n + 4 KiB per rank) and
the commit launch come on top. Usage: python scripts/rank_probe.py [world ...]
"""
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import mcmc_colorer_amd.colorer as M  # noqa: E402
from mcmc_colorer_amd._lib import MCMCCtxInfo, check, lib, u32ptr  # noqa: E402

N, P = 10_000_000, 0.001


def probe(world: int, rank: int, steps: int = 10) -> None:
    t0 = time.perf_counter()
    g = M.Graph.er_fast(N, P, 1, world=world, rank=rank)
    gen = time.perf_counter() - t0
    S = ((N + world - 1) // world + 15) // 16 * 16
    vb, ve = min(rank * S, N), min((rank + 1) * S, N)
    params = M.ColoringMCMCParams(nCol=32, maxRip=0x7FFFFFF0).to_c(1)
    ctx = ctypes.c_void_p()
    check(lib().mcmc_create(g.handle, ctypes.byref(params), vb, ve, ctypes.byref(ctx)))
    check(lib().mcmc_set_glibc_window(ctx, u32ptr(M.GlibcRand(1).window)))
    check(lib().mcmc_init_coloring(ctx, None))
    tot, ker = ctypes.c_double(), ctypes.c_double()
    check(lib().mcmc_bench_sweeps(ctx, 2, ctypes.byref(tot), ctypes.byref(ker)))
    check(lib().mcmc_bench_sweeps(ctx, steps, ctypes.byref(tot), ctypes.byref(ker)))
    info = MCMCCtxInfo()
    check(lib().mcmc_get_info(ctx, ctypes.byref(info)))
    print(f"world {world} rank {rank}: rows {ve - vb} arcs {g.nEdges} groups {info.ngroups} R {info.grp_rows} "
          f"sweep {ker.value:.3f} ms  ({info.sweep_bytes / ker.value / 1e6:.0f} GB/s)  gen {gen:.1f} s", flush=True)
    lib().mcmc_destroy(ctx)
    g.close()


if __name__ == "__main__":
    for w in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]:
        for r in sorted({0, w - 1}):
            probe(w, r)
