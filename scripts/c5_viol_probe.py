"""C5 stand-in with violators in every sweep (nCol = maxDeg / 4, the bench's `violators` record): the
reference loop to convergence, for a kernel trace of the violator-heavy first sweeps."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch

    torch.cuda.init()
    import mcmc_colorer_amd.colorer as M

    g = M.Graph.rmat(22, 10, 0.5, 0.2, 0.2, 1)
    nc = max(257, g.getMaxNodeDeg() // 4)
    for rep in range(2):
        col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=nc, maxRip=20))
        st = col.run(0)
        print(f"rep {rep}: nCol {nc} sweeps {st.sweepsRun} loop_ms {st.loopMs:.3f} traj {col.trajectory().tolist()}",
              flush=True)
        col.close()


if __name__ == "__main__":
    main()
