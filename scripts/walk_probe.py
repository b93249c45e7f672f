"""Per-workgroup walk timings of the violator-heavy C5 sweep (nCol = maxDeg / 4, sweep 0 from C_0):
MCMC_PHASE_DUMP stamps of the wide evaluation launch's walk workgroups (start, end, tasks, split tasks)."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    out = sys.argv[1]
    os.environ["MCMC_PHASE_DUMP"] = out
    import torch

    torch.cuda.init()
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    g = M.Graph.rmat(22, 10, 0.5, 0.2, 0.2, 1)
    nc = max(257, g.getMaxNodeDeg() // 4)
    col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=nc, maxRip=0x7FFFFFF0))
    col.init(0)
    # C_0's violators and their degrees (host count over the downloaded CSR)
    S = g.getStruct()
    C0 = col.coloring().astype(np.int64)
    deg = np.diff(S.cumulDegs.astype(np.int64))
    src = np.repeat(np.arange(g.nNodes), deg)
    bad = np.zeros(g.nNodes, dtype=bool)
    bad[src[C0[src] == C0[S.neighs.astype(np.int64)]]] = True
    vd = deg[bad]
    light = int(os.environ.get("MCMC_WALK_LIGHT", "512"))
    print(f"violators {bad.sum()}: degree med {np.median(vd):.0f} p90 {np.percentile(vd, 90):.0f} max {vd.max()}; "
          f"light (<= {light}) {(vd <= light).sum()} ({vd[vd <= light].sum()} arcs), heavy {(vd > light).sum()} "
          f"({vd[vd > light].sum()} arcs), > 2048: {(vd > 2048).sum()}", flush=True)
    tot, ker = ctypes.c_double(), ctypes.c_double()
    check(lib().mcmc_bench_sweeps(col._ctx, 1, ctypes.byref(tot), ctypes.byref(ker)))
    print(f"sweep 0: {ker.value * 1e3:.1f} us (phase stamps on)")
    t = np.fromfile(out, dtype=np.uint64).reshape(-1, 8).astype(np.int64)[:1024]
    live = t[t[:, 0] > 0]
    d = (live[:, 1] - live[:, 0]) / 100.0
    print(f"walk workgroups with tasks: {len(live)}; duration us: min {d.min():.1f} med {np.median(d):.1f} "
          f"p90 {np.percentile(d, 90):.1f} max {d.max():.1f}; tasks per wg med {np.median(live[:, 2]):.0f} max {live[:, 2].max()}; "
          f"split tasks total {live[:, 3].sum()}")
    st = (live[:, 0] - live[:, 0].min()) / 100.0
    print(f"start spread: max {st.max():.1f} us")
    i = np.argsort(-d)[:8]
    for k in i:
        print(f"  wg {k}: {d[k]:.1f} us, tasks {live[k, 2]}, split {live[k, 3]}, start +{st[k]:.1f}")
    # per-task stamps (walk_task_stamp): gather | walk ticks (10 ns), arcs | kind
    rec = np.fromfile(out, dtype=np.uint64)[8 * 4096:].reshape(-1, 2)
    rec = rec[rec[:, 1] > 0]
    gat = (rec[:, 0] & 0xFFFFFFFF).astype(np.int64) / 100.0
    wlk = (rec[:, 0] >> np.uint64(32)).astype(np.int64) / 100.0
    dg = (rec[:, 1] & 0xFFFFFFFF).astype(np.int64)
    kind = (rec[:, 1] >> np.uint64(32)).astype(np.int64)
    for k, name in enumerate(["light (wave)", "heavy row (workgroup)", "split chunk", "split chunk + walk"]):
        m = kind == k
        if m.any():
            print(f"{name:22s} n {m.sum():5d}  gather us med {np.median(gat[m]):6.1f} p90 {np.percentile(gat[m], 90):6.1f} "
                  f"max {gat[m].max():6.1f} | walk us med {np.median(wlk[m]):6.1f} p90 {np.percentile(wlk[m], 90):6.1f} "
                  f"max {wlk[m].max():6.1f} | arcs med {np.median(dg[m]):.0f} max {dg[m].max()}")
    top = np.argsort(-(gat + wlk))[:6]
    for i in top:
        print(f"  slow task: kind {kind[i]} arcs {dg[i]} gather {gat[i]:.1f} walk {wlk[i]:.1f} us")
    col.close()


if __name__ == "__main__":
    main()
