"""ColoringMCMC_CPU's per-vertex hooks (include/mcmc_colorer.hpp; reference coloringMCMC_CPU.h:20-28,
public "for integration with GoogleTest"): count_free_colors, fill_p, extract_new_color driven vertex
by vertex over loop 1 of run() (coloringMCMC_CPU.cpp:183-204) on host-only graphs -- K3, P4, C5 and a
random graph -- against the oracle's restatement of the same vertex update, with draws that land in
every branch (fill_p cases (i)-(iii), the strict > at a CDF step, the rand() % (nCol - 1) overflow
from the process-global glibc stream, srand(1)). CPU only: the hooks are host code."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as O

ROOT = Path(__file__).resolve().parent.parent
EXE = ROOT / "tests" / "build" / "hooks_main"


@pytest.fixture(scope="module")
def hooks_exe():
    from mcmc_colorer_amd import build as B

    B.build_lib()
    EXE.parent.mkdir(exist_ok=True)
    src = ROOT / "tests" / "hooks_main.cpp"
    hdr = ROOT / "include" / "mcmc_colorer.hpp"
    if not EXE.exists() or EXE.stat().st_mtime < max(src.stat().st_mtime, hdr.stat().st_mtime):
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include'}", str(src), "-o", str(EXE),
                        f"-L{ROOT / 'mcmc_colorer_amd'}", "-lmcmc_hip", f"-Wl,-rpath,{ROOT / 'mcmc_colorer_amd'}"],
                       check=True)
    return EXE


def graph(name):
    if name == "K3":
        E = [(0, 1), (0, 2), (1, 2)]
        n = 3
    elif name == "P4":
        E = [(0, 1), (1, 2), (2, 3)]
        n = 4
    elif name == "C5":
        E = [(i, (i + 1) % 5) for i in range(5)]
        n = 5
    else:
        O.srand(1)
        return O.setup_rnd2(60, 0.2)
    adj = [[] for _ in range(n)]
    for a, b in E:
        adj[a].append(b)
        adj[b].append(a)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in adj])
    return off, np.array([w for x in adj for w in sorted(x)], dtype=np.uint32)


def run(exe, off, idx, ncol, eps, seed, u, taboo=0):
    n = len(off) - 1
    inp = f"{n} {len(idx)} {ncol} {eps!r} {seed} {taboo}\n" + " ".join(map(str, off.tolist())) + "\n" + \
          " ".join(map(str, idx.tolist())) + "\n" + " ".join(repr(float(x)) for x in u) + "\n"
    r = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True)
    lines = r.stdout.split("\n")
    c0 = np.array(lines[0].split()[1:], dtype=np.uint32)
    rows = [list(map(int, ln.split())) for ln in lines[1:1 + n]]
    k = int(lines[1 + n].split()[1])
    return c0, rows, k


@pytest.mark.parametrize("name,ncol,eps", [("K3", 3, 1e-8), ("K3", 2, 1e-8), ("P4", 3, 1e-8), ("C5", 3, 1e-8),
                                           ("C5", 2, 0.2), ("P4", 5, 0.05), ("G", 0, 1e-8), ("G", 6, 1e-3)])
def test_hooks_match_oracle(hooks_exe, name, ncol, eps):
    off, idx = graph(name)
    n = len(off) - 1
    ncol = ncol or O.max_deg(off)
    seed = 11
    rng = np.random.default_rng(ncol * 7 + n)
    u = rng.random(n).astype(np.float32)
    u[0] = np.float32(1 - 2 ** -24)   # the largest draw: a CDF overflow in case (i)/(iii)
    if n > 2:
        u[1] = np.float32(0.0)
    c0, rows, k = run(hooks_exe, off, idx, ncol, eps, seed, u)
    # the initial colouring: ColoringMCMC_CPU's ctor (coloringMCMC_CPU.cpp:53-61)
    exp0 = np.zeros(n, dtype=np.uint32)
    O.lib().oracle_uniform_int_seq(seed, ncol, n, O._p(exp0))
    assert c0.tolist() == exp0.tolist()
    O.srand(1)   # the hooks' overflows draw the process stream from srand(1), in vertex order
    nviol = 0
    for v in range(n):
        nbr = c0[idx[off[v]:off[v + 1]]]
        c, viol = O.vertex_update(ncol, eps, int(c0[v]), nbr, float(u[v]))
        if c is None:
            c = O.rand(1)[0] % (ncol - 1)
        vv, rv, zv, newc, qb = rows[v][:5]
        assert vv == v and bool(rv) == viol, (v, rows[v][:5], viol)
        assert zv == ncol - len(set(nbr.tolist())), v
        assert newc == c, (name, v, newc, c)
        p = np.array(rows[v][5:], dtype=np.uint32).view(np.float32)
        assert len(p) == ncol and np.array_equal(np.array([qb], dtype=np.uint32).view(np.float32), p[newc:newc + 1])
        nviol += viol
    assert k == nviol
