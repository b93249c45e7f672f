"""One HIP runtime per process, whatever the import order.

torch bundles its own HIP and HSA runtimes (libamdhip64.so with the soname libamdhip64.so.7);
libmcmc_hip.so needs libamdhip64.so.7. mcmc_colorer_amd._lib loads the process's runtime (torch's
when torch is installed) before the library, so the library binds to it and a later `import torch`
finds it mapped. The child processes start fresh (nothing imported, no device touched)."""
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

LIB_FIRST = textwrap.dedent("""
    import sys
    sys.path.insert(0, {root!r})
    from mcmc_colorer_amd import _lib
    _lib.lib()
    first = _lib._hip_runtimes()
    import torch
    after = _lib._hip_runtimes()
    assert len(first) == 1 and after == first, (first, after)
    if {gpu}:
        import mcmc_colorer_amd.colorer as M
        n = 300
        g = M.Graph.simulate(n, 0.1, M.GlibcRand(1), device=0)
        col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.getMaxNodeDeg()))
        st = col.run(0)
        assert st.sweepsRun >= 1
        x = torch.arange(1000, device="cuda", dtype=torch.float32).sum().item()
        assert x == 499500.0, x
        assert _lib._hip_runtimes() == first
        print("sweeps", st.sweepsRun, "torch ok", x)
    print("runtimes", sorted(first))
""")


def _child(gpu: bool) -> str:
    r = subprocess.run([sys.executable, "-c", LIB_FIRST.format(root=str(ROOT), gpu=gpu)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_library_before_torch_one_runtime():
    out = _child(False)
    assert "runtimes" in out


@pytest.mark.gpu
def test_library_before_torch_runs_on_the_gpu():
    """The library loaded, a colouring run on the device, THEN torch imported and used: both on the
    same runtime (r04: hipSetDevice 'no ROCm-capable device is detected' in this order)."""
    out = _child(True)
    assert "torch ok" in out, out
