"""Library loaded before torch, one colouring, a torch op, exit: which variant of teardown aborts
(tests/test_runtime.py saw 'double free or corruption' at exit on the r05 box)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BODY = """
import sys
sys.path.insert(0, {root!r})
from mcmc_colorer_amd import _lib
_lib.lib()
import torch
import mcmc_colorer_amd.colorer as M
n = 300
g = M.Graph.simulate(n, 0.1, M.GlibcRand(1), device=0)
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.getMaxNodeDeg()))
st = col.run(0)
x = torch.arange(1000, device="cuda", dtype=torch.float32).sum().item()
print("ran", st.sweepsRun, x, flush=True)
{tail}
"""
for name, tail in (("implicit", ""), ("close", "col.close(); g.close()"), ("no_torch_op", ""),
                   ("no_torch_first", "")):
    body = BODY.format(root=str(ROOT), tail=tail)
    if name == "no_torch_op":
        body = body.replace('x = torch.arange(1000, device="cuda", dtype=torch.float32).sum().item()', "x = 0")
    env = dict(__import__("os").environ, **({"MCMC_NO_TORCH_FIRST": "1"} if name == "no_torch_first" else {}))
    r = subprocess.run([sys.executable, "-c", body], capture_output=True, text=True, timeout=300, env=env)
    print(name, r.returncode, r.stdout.strip()[-80:], r.stderr.strip()[-200:], flush=True)
