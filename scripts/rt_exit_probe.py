"""Which teardown aborts when libmcmc_hip.so is loaded before torch ('double free or corruption' at
exit, r05 box: gpurun_out/r05final/rt.log). Each variant is a fresh child; a SIGABRT handler
(scripts/abrt_trace.so, diagnostic) prints a stack scan of the abort.
r06 findings: no ROCm library was mapped twice; the abort came from librocm_smi64's static
std::map destructor (gpurun_out/r06c) and only when _lib preloaded torch's runtime and RCCL
RTLD_GLOBAL; with RTLD_LOCAL every order exited with status 0 (gpurun_out/r06d). _lib now always
preloads RTLD_LOCAL and no longer imports torch, so the MCMC_NO_TORCH_FIRST / MCMC_PRELOAD_MODE
knobs the variants set are no longer read: every variant runs the fixed loader."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
TRACE = ROOT / "scripts" / "abrt_trace.so"
HEAD = """
import sys, os, ctypes, atexit
ctypes.CDLL({trace!r})
sys.path.insert(0, {root!r})
def _maps():
    keys = ("amdhip64", "hsa-runtime", "comgr", "rocprofiler", "rccl", "libdrm", "numa", "libelf", "rocm_smi",
            "roctx", "roctracer", "mcmc_hip", "torch_hip", "c10_hip")
    seen = {{}}
    for ln in open("/proc/self/maps"):
        p = ln.split()[-1]
        if p.startswith("/") and any(k in p for k in keys):
            seen[p] = 1
    print("MAPS", *sorted(seen), sep="\\n  ", flush=True)
"""
RUN = """
import mcmc_colorer_amd.colorer as M
n = 300
g = M.Graph.simulate(n, 0.1, M.GlibcRand(1), device=0)
col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.getMaxNodeDeg()))
st = col.run(0)
print("ran", st.sweepsRun, flush=True)
"""
TORCH_OP = """
import torch
x = torch.arange(1000, device="cuda", dtype=torch.float32).sum().item()
print("torch", x, flush=True)
"""
VARIANTS = {
    # the r05 failure: library (torch's runtime preloaded), a run, then torch and a torch op
    "lib_run_torch": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + TORCH_OP, {"MCMC_NO_TORCH_FIRST": "1"}),
    # the same without importing torch at all
    "lib_run": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN, {"MCMC_NO_TORCH_FIRST": "1"}),
    # the library on its own /opt/rocm runtime, no torch
    "own_rt_run": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN,
                   {"MCMC_NO_TORCH_FIRST": "1", "MCMC_OWN_HIP_RUNTIME": "1"}),
    # torch imported (no op) after the run
    "lib_run_import": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + "import torch\n",
                       {"MCMC_NO_TORCH_FIRST": "1"}),
    # torch imported after loading but before the first HIP call
    "lib_torch_run": ("from mcmc_colorer_amd import _lib; _lib.lib()\nimport torch\n" + RUN + TORCH_OP,
                      {"MCMC_NO_TORCH_FIRST": "1"}),
    # handles closed before exit
    "lib_run_torch_close": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + TORCH_OP + "col.close(); g.close()\n",
                            {"MCMC_NO_TORCH_FIRST": "1"}),
    # the r05 failure with the runtime and RCCL preloaded RTLD_LOCAL instead of RTLD_GLOBAL
    "lib_run_import_local": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + "import torch\n",
                             {"MCMC_NO_TORCH_FIRST": "1", "MCMC_PRELOAD_MODE": "local"}),
    "lib_run_torch_local": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + TORCH_OP,
                            {"MCMC_NO_TORCH_FIRST": "1", "MCMC_PRELOAD_MODE": "local"}),
    "lib_torch_run_local": ("from mcmc_colorer_amd import _lib; _lib.lib()\nimport torch\n" + RUN + TORCH_OP,
                            {"MCMC_NO_TORCH_FIRST": "1", "MCMC_PRELOAD_MODE": "local"}),
    # the default order (torch first)
    "default": ("from mcmc_colorer_amd import _lib; _lib.lib()" + RUN + TORCH_OP, {}),
}
only = sys.argv[1:]
for name, (body, extra) in VARIANTS.items():
    if only and name not in only:
        continue
    src = HEAD.format(trace=str(TRACE), root=str(ROOT)) + body
    env = dict(os.environ, **extra)
    print(f"##### {name}", flush=True)
    try:
        r = subprocess.run([sys.executable, "-u", "-c", src], timeout=120, env=env)   # output streams to ours
        print(f"##### {name} rc={r.returncode}", flush=True)
    except subprocess.TimeoutExpired:
        print(f"##### {name} timed out", flush=True)
