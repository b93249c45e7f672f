"""C5 stand-in, nCol = maxDeg / 4 (violators in the first sweeps): the reference loop with the
persistent wide sweep on and off, its per-step times (MCMC_WIDE_SOLO is read at context creation)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import mcmc_colorer_amd.colorer as M  # noqa: E402

g = M.Graph.rmat(22, 10, 0.5, 0.2, 0.2, 1, device=0)
nc4 = max(257, g.maxDeg // 4)
for ws in ("1", "0", "1"):
    os.environ["MCMC_WIDE_SOLO"] = ws
    cv = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=nc4, maxRip=20))
    st = cv.run(0)
    s = cv.wide_solo_stats()
    print(f"ws={ws} loop {st.loopMs:.3f} ms, {st.sweepsRun} sweeps, traj {cv.trajectory().tolist()[:6]}", flush=True)
    if s["enabled"]:
        print("   ", {k: s[k] for k in ("sweeps", "phases", "leader_walks", "walk_phases", "delta_phases", "collects",
                                     "changed_rows")}, flush=True)
        print("    step us (sum)", {k: round(v, 1) for k, v in s["step_us"].items()}, flush=True)
    cv.close()
