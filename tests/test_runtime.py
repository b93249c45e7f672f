"""One HIP runtime per process, whatever the import order.

torch bundles its own HIP and HSA runtimes (libamdhip64.so with the soname libamdhip64.so.7) and
RCCL (librccl.so.1, which pulls in librocm_smi64); libmcmc_hip.so needs libamdhip64.so.7 and
librccl.so.1. mcmc_colorer_amd._lib loads the process's runtime and RCCL (torch's when torch is
installed) RTLD_LOCAL before the library, so the library binds to them by soname and a later
`import torch` finds them mapped. r05 preloaded them RTLD_GLOBAL: a process that loaded the library
before torch then aborted at exit ("double free or corruption" in librocm_smi64's static destructors,
gpurun_out/r06c). The child processes start fresh (nothing imported, no device touched) and must
exit with status 0 in every order."""
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
    assert "torch" not in sys.modules   # loading the library does not import torch
    if {gpu} and {run_before}:
        import mcmc_colorer_amd.colorer as M
        n = 300
        g = M.Graph.simulate(n, 0.1, M.GlibcRand(1), device=0)
        col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.getMaxNodeDeg()))
        st = col.run(0)
        assert st.sweepsRun >= 1
        print("sweeps", st.sweepsRun)
    import torch
    after = _lib._hip_runtimes()
    assert len(first) <= 1 and (not first or after == first), (first, after)
    if {gpu}:
        if not {run_before}:
            import mcmc_colorer_amd.colorer as M
            n = 300
            g = M.Graph.simulate(n, 0.1, M.GlibcRand(1), device=0)
            col = M.ColoringMCMC(g, M.GPURand(n, 1, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=g.getMaxNodeDeg()))
            assert col.run(0).sweepsRun >= 1
        if {torch_op}:
            x = torch.arange(1000, device="cuda", dtype=torch.float32).sum().item()
            assert x == 499500.0, x
            print("torch ok", x)
        assert _lib._hip_runtimes() == first
    print("runtimes", sorted(first))
""")


def _child(gpu: bool, run_before: bool = True, torch_op: bool = True) -> str:
    src = LIB_FIRST.format(root=str(ROOT), gpu=gpu, run_before=run_before, torch_op=torch_op)
    r = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout + r.stderr)
    assert "double free" not in r.stderr
    return r.stdout


def test_library_before_torch_one_runtime():
    out = _child(False)
    assert "runtimes" in out


@pytest.mark.gpu
@pytest.mark.parametrize("run_before,torch_op", [(True, True), (True, False), (False, True)])
def test_library_before_torch_runs_on_the_gpu(run_before, torch_op):
    """The library loaded before torch, a colouring run on the device before or after `import torch`,
    a torch op or none: both on the same runtime (r04: hipSetDevice 'no ROCm-capable device is
    detected' in this order) and a clean exit (r05: rc -6 'double free or corruption')."""
    out = _child(True, run_before, torch_op)
    assert "runtimes" in out
    if torch_op:
        assert "torch ok" in out, out


@pytest.mark.gpu
def test_runtime_major_version_matches_build(hip_lib):
    """The runtime the library runs on (torch's bundled one) has the major version it was built for."""
    import ctypes

    from mcmc_colorer_amd._lib import check, lib

    built, rt = ctypes.c_int(), ctypes.c_int()
    check(lib().mcmc_hip_versions(ctypes.byref(built), ctypes.byref(rt)))
    assert built.value // 10_000_000 == rt.value // 10_000_000, (built.value, rt.value)
