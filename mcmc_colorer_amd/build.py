"""Builds libmcmc_hip.so (gfx950) in-tree, plus the oracle (test infrastructure) when asked.

    python -m mcmc_colorer_amd.build            # product library + CLI
    python -m mcmc_colorer_amd.build --oracle   # also oracle/build/*
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
LIB = PKG / "libmcmc_hip.so"
CLI = PKG / "mcmc_colorer"
ARCH = os.environ.get("MCMC_OFFLOAD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
# -ffp-contract=off: bit-exact fp32 with the reference's (non-FMA) host arithmetic.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          f"-I{ROOT / 'include'}", f"-I{CSRC}", "-Wall", "-Wno-unused-function"]
LIB_SOURCES = ["mcmc_sweep.hip", "graph.hip", "tiled_layout.hip", "refstruct.hip", "tailcut.hip", "refmode.hip", "rmat.hip",
               "greedyff.hip", "luby.hip", "multi.hip"]
# RCCL (multi.hip: the native multi-GPU path); torch's bundled librccl.so.1 satisfies the same soname
# when torch is loaded first
LINK = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def _run(cmd: list[str]) -> None:
    print(" ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build_lib(force: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h*"))
    objs = []
    jobs = []
    for src in LIB_SOURCES:
        s = CSRC / src
        o = BUILD / (src + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            jobs.append([HIPCC, *COMMON, "-c", s, "-o", o])
    if jobs:
        with ThreadPoolExecutor(max_workers=min(4, len(jobs))) as ex:
            list(ex.map(_run, jobs))
    if force or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, *LINK, "-o", LIB])
    return LIB


def build_cli(force: bool = False) -> Path | None:
    src = CSRC / "main.cpp"
    if not src.exists():
        return None
    headers = list(CSRC.glob("*.h*")) + list((ROOT / "include").glob("*.h*"))
    if force or _stale(CLI, [src, LIB] + headers):
        _run([HIPCC, "-O2", "-std=c++17", f"-I{ROOT / 'include'}", src, "-o", CLI,
              f"-L{PKG}", "-lmcmc_hip", f"-Wl,-rpath,$ORIGIN"])
    return CLI


def build_oracle() -> None:
    _run(["make", "-C", ROOT / "oracle", "-j4"])


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build_lib(a.force)
    build_cli(a.force)
    if a.oracle:
        build_oracle()
    return 0


if __name__ == "__main__":
    sys.exit(main())
