"""Persistent wide sweep probe: one R-MAT case, its result vs the oracle, the sweep statistics.
MCMC_WS_DEBUG=1: the run goes on a thread while this one prints the kernel's progress words."""
import collections
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle_np as NP  # noqa: E402
import oracle_ref as O  # noqa: E402

import mcmc_colorer_amd.colorer as M  # noqa: E402
from mcmc_colorer_amd import _lib  # noqa: E402

ncol = int(sys.argv[1]) if len(sys.argv) > 1 else 300
maxrip = int(sys.argv[2]) if len(sys.argv) > 2 else 25
off, idx = NP.rmat(12, 8, 0.5, 0.2, 0.2, 4)
g = M.Graph.from_csr(off, idx)
col = M.ColoringMCMC(g, M.GPURand(g.nNodes, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=ncol, maxRip=maxrip))
out = {}


def run():
    try:
        out["st"] = col.run(0)
    except Exception as e:  # noqa: BLE001
        out["err"] = str(e)


th = threading.Thread(target=run, daemon=True)
t0 = time.time()
th.start()
L = _lib.lib()
L.mcmc_ws_debug.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
buf = (ctypes.c_uint32 * 1024)()
for i in range(40):
    th.join(0.5)
    if not th.is_alive():
        break
    if i % 4 == 3:
        L.mcmc_ws_debug(col._ctx, buf, 1024)
        hs = collections.Counter(buf[64 + b] & 15 for b in range(1, 256))
        gens = collections.Counter(buf[64 + b] >> 4 for b in range(1, 256))
        print(f"t={time.time() - t0:.1f}s leader k={buf[0]} step={buf[1]} seq={buf[2]} done={buf[3]} exp={buf[4]}; "
              f"helper states {dict(hs)} gens {dict(gens.most_common(4))}", flush=True)
        for b in range(1, 4):
            print(f"   wg {b} waves", [hex(buf[512 + b * 16 + k]) for k in range(16)], flush=True)
if th.is_alive():
    print("HUNG: leaving", flush=True)
    sys.stdout.flush()
    os._exit(3)
print("run", out, time.time() - t0, flush=True)
print("ws", col.wide_solo_stats(), flush=True)
O.srand(1)
r = O.mcmc_run(off, idx, ncol, 1, maxRip=maxrip)
print("oracle", r.res.iter, r.res.finalViol, r.res.glibcDraws, "traj", r.traj.tolist()[:8], flush=True)
print("gpu   traj", col.trajectory().tolist()[:8], flush=True)
print("colours equal", col.coloring().tolist() == r.colors.tolist(), flush=True)
