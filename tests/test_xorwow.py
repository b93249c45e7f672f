"""Pins the reference-GPU-semantics pieces before the GPU is checked against them.

1. XORWOW: the build's jump-ahead (mcmc_xorwow_state, column-major GF(2) tables) and the oracle's
   (row-major, written separately) equal rocRAND's engine -- the same transition and 2^67
   subsequence jump as cuRAND, other salts -- run from tests/probes/rocrand_xorwow_probe.cpp.
   With cuRAND's salts (restated from cuRAND's published header; not in this image) the build and
   the oracle agree: parity there is unpinned against CUDA itself.
2. The oracle's restatement of the reference's GPU colorer (oracle/mcmc_gpu_ref.cpp) equals a
   second restatement in plain Python (below), written from the same reference source
   (coloringMCMC_main.cu:101-298, coloringMCMC_balance.cu:79-143, coloringMCMC_utils.cu:24-119).
"""
import ctypes
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as O

ROOT = Path(__file__).resolve().parent.parent
PROBE = ROOT / "tests" / "probes" / "rocrand_xorwow_probe.cpp"
CASES = [(1, 0), (1, 1), (1, 2), (0, 3), (5, 1_000_000), (7, 12345), (2**64 - 1, 2**32 - 1),
         (123456789, 65535), (42, 2**31 + 77)]


@pytest.fixture(scope="module")
def rocrand_probe(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists() or not Path("/opt/rocm/include/rocrand/rocrand_xorwow.h").exists():
        pytest.skip("hipcc / rocRAND headers not available")
    exe = tmp_path_factory.mktemp("probe") / "xwprobe"
    subprocess.run([hipcc, "-O1", "--offload-arch=gfx950", str(PROBE), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    return exe


def _product_state(seed, sub, flavor):
    from mcmc_colorer_amd._lib import lib

    out = (ctypes.c_uint32 * 6)()
    assert lib().mcmc_xorwow_state(ctypes.c_uint64(seed), ctypes.c_uint64(sub), flavor, out) == 0
    return list(out)


def test_jump_and_transition_equal_rocrand(rocrand_probe, hip_lib):
    r = subprocess.run([str(rocrand_probe)] + [f"{s}:{k}" for s, k in CASES], capture_output=True, text=True,
                       check=True, timeout=60)
    for (seed, sub), line in zip(CASES, r.stdout.strip().split("\n")):
        ref = [int(x) for x in line.split()]
        orc = O.xorwow_init(seed, sub, flavor=1)
        assert orc.tolist() == ref[:6], (seed, sub)
        assert O.xorwow_next(orc, 4).tolist() == ref[6:], (seed, sub)
        assert _product_state(seed, sub, 1) == ref[:6], (seed, sub)


def test_curand_flavour_build_equals_oracle(hip_lib):
    rng = np.random.default_rng(3)
    cases = CASES + [(int(rng.integers(0, 2**63)), int(rng.integers(0, 2**32))) for _ in range(20)]
    for seed, sub in cases:
        assert _product_state(seed, sub, 0) == O.xorwow_init(seed, sub, 0).tolist(), (seed, sub)
    # curand_init's salt for seed 0, subsequence 0 (no jump): the salted state itself
    t0 = (1099087573 * 0xAAD26B49) & 0xFFFFFFFF
    t1 = (2591861531 * 0xF7DCEFDD) & 0xFFFFFFFF
    assert O.xorwow_init(0, 0, 0).tolist() == [(123456789 + t0) & 0xFFFFFFFF, 362436069 ^ t0,
                                               (521288629 + t1) & 0xFFFFFFFF, 88675123 ^ t1,
                                               (5783321 + t0) & 0xFFFFFFFF, (6615241 + t1 + t0) & 0xFFFFFFFF]


# ---- second restatement of the reference GPU colorer, plain Python (small graphs only) --------
M32 = 0xFFFFFFFF
F = np.float32


def _next(s):
    t = (s[0] ^ (s[0] >> 2)) & M32
    s[0], s[1], s[2], s[3] = s[1], s[2], s[3], s[4]
    s[4] = ((s[4] ^ ((s[4] << 4) & M32)) ^ (t ^ ((t << 1) & M32))) & M32
    s[5] = (s[5] + 362437) & M32
    return (s[4] + s[5]) & M32


def _uniform(x):
    return F(F(x) * F(2.0**-32)) + F(2.0**-33)    # curand_uniform: x 2^-32 + 2^-33


def _edges(off, idx, C, v):
    return sum(1 for w in idx[off[v]:off[v + 1]] if C[w] == C[v] and v < w)


def py_gpu_run(off, idx, ncol, states, max_rip=250, taboo_iter=0, tailcut=False, eps=F(1e-8), tail_max=1000):
    n = len(off) - 1
    S = [list(map(int, s)) for s in states]
    C = [0] * n
    B = [0] * n
    taboo = [0] * n
    for v in range(n):                                       # initColoring
        C[v] = int(_uniform(_next(S[v])) * F(ncol))
    z = max(50, n // 2000) if tailcut else 0
    hi = F(1) - F(F(ncol - 1) * eps)                         # == the fused value for eps = 1e-8
    traj, rip, broke, cc = [], 0, False, 0
    while True:
        rip += 1
        cc = sum(_edges(off, idx, C, v) for v in range(n))
        traj.append(cc)
        if cc <= z:
            broke = True
            break
        hist = [0] * (ncol + 1)
        for c in C:
            hist[min(c, ncol)] += 1
        p = [F(F(1) - F(F(hist[c]) / F(n))) / F(ncol - 1) for c in range(ncol)]
        for v in range(n):
            if taboo[v] > 0:
                taboo[v] -= 1
                continue                                     # star keeps its stale value
            occ = [False] * ncol
            for w in idx[off[v]:off[v + 1]]:
                if C[w] < ncol:
                    occ[C[w]] = True
            rem, zn = F(0), 0
            for i in range(ncol):
                if occ[i]:
                    zn += 1
                    rem = F(rem + F(p[i] - eps))
            zp = ncol - zn
            if zp == 0:
                B[v] = C[v]
                continue
            u = _uniform(_next(S[v]))
            i, thr = 0, F(0)
            own = C[v] < ncol and occ[C[v]]
            r = F(rem / F(zp))
            while True:
                q = (eps if occ[i] else F(p[i] + r)) if own else (hi if i == C[v] else eps)
                thr = F(thr + q)
                i += 1
                if not (thr < u and i < ncol):
                    break
            B[v] = i - 1
            taboo[v] = taboo_iter if B[v] == C[v] else 0
        C, B = B, C
        if rip >= max_rip:
            break
    if not broke:
        traj.append(sum(_edges(off, idx, C, v) for v in range(n)))
    passes, tail = 0, []
    if tailcut:
        hist = [0] * (max(n, ncol) + 1)
        for c in C:
            hist[c] += 1
        order = sorted(range(ncol), key=lambda c: hist[c])   # stable == libstdc++ insertion sort (ncol <= 16)
        while cc > 0 and passes < tail_max:
            cnt = [_edges(off, idx, C, v) for v in range(n)]
            resolved = 0
            for v in range(n):
                if resolved >= cc:
                    break
                if not cnt[v]:
                    continue
                resolved += 1
                occ = [False] * ncol
                for w in idx[off[v]:off[v + 1]]:
                    if C[w] < ncol:
                        occ[C[w]] = True
                c, j = C[v], 0
                while c < ncol and occ[c] and j < ncol:
                    c = order[j]
                    j += 1
                C[v] = c
            cc = sum(_edges(off, idx, C, v) for v in range(n))
            tail.append(cc)
            passes += 1
    return C, traj, rip, rip == max_rip, passes, tail, S


GPU_CASES = [
    # n, p, nCol, seed, maxRip, taboo, tailcut
    (60, 0.2, 0, 1, 250, 0, False),      # nCol = maxDeg: converges
    (80, 0.15, 5, 2, 25, 0, False),      # too few colours: runs to the cap
    (70, 0.2, 6, 3, 30, 2, False),       # taboo
    (90, 0.1, 4, 4, 20, 1, True),        # tail cut after the cap (stale conflictCounter)
    (120, 0.05, 6, 5, 250, 0, True),     # stops within z = 50, tail cut resolves
    (50, 0.3, 12, 6, 40, 3, True),
]


@pytest.mark.parametrize("n,p,ncol,seed,maxrip,taboo,tailcut", GPU_CASES)
def test_oracle_gpu_semantics_equals_python_restatement(n, p, ncol, seed, maxrip, taboo, tailcut):
    O.srand(1)
    off, idx = O.setup_rnd2(n, p)
    nc = ncol or O.max_deg(off)
    st = O.gpurand_init(n, seed)
    C, traj, rip, maxr, passes, tail, S = py_gpu_run(off.tolist(), idx.tolist(), nc, st.tolist(), maxrip, taboo,
                                                     tailcut)
    for rep in range(2):   # two repetitions share the states (main.cu:80, 193)
        r = O.mcmc_gpu_run(off, idx, nc, st, maxRip=maxrip, tabooIteration=taboo, tailcut=tailcut)
        if rep == 0:
            assert r.colors.tolist() == C
            assert r.traj.tolist() == traj
            assert (r.res.rip, bool(r.res.maxIterReached), r.res.tailcutPasses) == (rip, maxr, passes)
            assert r.tail_traj.tolist() == tail
            assert st.tolist() == S
        else:
            C, traj, rip, maxr, passes, tail, S = py_gpu_run(off.tolist(), idx.tolist(), nc, S, maxrip, taboo,
                                                             tailcut)
            assert r.colors.tolist() == C and r.traj.tolist() == traj and st.tolist() == S
