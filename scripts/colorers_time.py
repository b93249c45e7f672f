"""Wall time of the other colorers (GreedyFF, Luby, VFF) on the GPU: C2's graph size from the
build's G(n,p) generator and the C5 stand-in R-MAT graph. One JSON line per (graph, colorer)."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402  (torch's HIP runtime first, as in the tests)

if torch.cuda.is_available():
    torch.cuda.init()
import mcmc_colorer_amd.colorer as M  # noqa: E402

graphs = [("rmat scale 20 ef 10", lambda: M.Graph.rmat(20, 10)),
          ("--simulate 0.01 -n 100000 (setupRnd2 replay)", lambda: M.Graph.simulate(100000, 0.01, M.GlibcRand(1)))]
for name, make in graphs:
    g = make()
    for cname in ("GreedyFF", "Luby", "VFF"):
        states = M.CurandStates(g.nNodes, 1) if cname == "Luby" else None
        col = {"GreedyFF": lambda: M.ColoringGreedyFF(g), "Luby": lambda: M.ColoringLuby(g, states),
               "VFF": lambda: M.ColoringVFF(g)}[cname]()
        t0 = time.perf_counter()
        col.run()
        dt = time.perf_counter() - t0
        k = {"GreedyFF": lambda: col.numColors, "Luby": lambda: col.numOfColors, "VFF": lambda: col.numColors}[cname]()
        extra = {"rounds": getattr(col, "rounds", None), "iterations": getattr(col, "iterations", None),
                 "valid": getattr(col, "valid", None)}
        print(json.dumps({"graph": name, "n": g.nNodes, "colorer": cname, "seconds": round(dt, 4), "colors": k, **extra}),
              flush=True)
