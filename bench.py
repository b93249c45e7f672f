"""bench.py -- vertex-updates/s of the MCMC colour-resampling sweep on MI355X.

Default workload (--config c3): BASELINE.json configs[2], the configuration the north star's target
is quoted on -- `--mcmcgpu --simulate 0.001 -n 10000000`, 32 colours, one MI355X. setupRnd2 is
infeasible there (5e13 sequential glibc draws), so the graph is the build's documented counter-based
G(n, p) (mcmc_colorer_amd/csrc/er_gen.h, seed 1), generated on the GPU straight into
the sweep's tiled layout (1e11 arcs, 217 GB; no CSR could exist: 400 GB). Under torchrun (N > 1) it
is configs[3]: the same graph vertex-partitioned over N GPUs (strong scaling), every rank generating
only its own rows; the loop runs natively with the RCCL communicator inside libmcmc_hip.so
(mcmc_part_run, csrc/multi.hip: per sweep the row ranges travel by P2P sends over xGMI -- or one
all-gather for equal ranges -- plus one all-gather of the 4 KiB footers).
`--config c2`: configs[1], `--simulate 0.01 -n 100000 --nCol 16` with the reference's exact setupRnd2
graph (weak scaling at N > 1: N*1e5 rows, p 0.01/N).
`--config c5`: configs[4] (power-law, nCol = maxDeg). SNAP LiveJournal / Reddit are not available, so
the graph is the build's R-MAT stand-in of LiveJournal's size and skew (csrc/er_gen.h rmat_edge: scale
22 = 4.19M vertices, edge factor 10, (a,b,c) = (0.5,0.2,0.2), seed 1; about 82M arcs, maxDeg about 26K),
the wide sweep (uint16 colours); under torchrun the graph is vertex-partitioned (strong scaling). The run
converges, so the one-GPU line also carries the full --mcmcgpu run from the initial colouring:
sweeps-to-zero-conflict and its wall time.
`--semantics ref` (one GPU): the same sweep with the reference GPU colorer's own semantics
(--mcmcgpu-ref: balance-dynamic proposal, per-vertex cuRAND XORWOW, conflicts counted as edges);
its CPU leg times the oracle's restatement of those semantics.

A step is one sweep: all n vertices resampled. Inputs are resident in HBM before the timed region;
the timed region is K back-to-back sweeps (one hipGraph at N = 1) bracketed by barrier + synchronize,
max over ranks. Prints ONE JSON line (rank 0). Besides the driver contract fields it carries
  roofline     : the sweep kernel's bytes per launch in its layout (B_fmt; the
                 reference-layout B_alg beside it) / its average duration, measured with hipEvents on
                 the kernel's own stream, against the 8 TB/s HBM peak; traffic = PMC HBM bytes per
                 launch from the committed rocprofv3 summary (profiles/pmc_summary.json)
  refstruct    : the reference CUDA path's per-sweep structure re-expressed in HIP (the stand-in for
                 "the reference CUDA path's vertex-updates/sec", which cannot run on MI355X)
  cpu_baseline : the oracle (faithful single-thread restatement of --mcmccpu, kind "port") on this
                 host, a bounded number of sweeps
For c3 the CPU leg runs on `--simulate 0.1 -n 100000` (C3's mean degree, 1e4) and the refstruct leg on a
2e6-row graph of the same degree (full occupancy at thread-per-vertex): C3's own uint32 CSR (400 GB)
cannot exist on the host or one GPU. Every single-GPU line also carries `convergence`: the reference
loop run from the initial colouring (sweeps-to-zero-conflict, or not converged at 251 + final Cviol +
trajectory).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


KERNELS = {"dense": "dc_multi_kernel (persistent: the timed sweeps in one launch; solo sweeps on workgroup 0, "
                    "full sweeps on the grid)",
           "dense-part": "dc_eval_kernel (one sweep: update + evaluation + commit; world 1: dc_multi_kernel)",
           "wide-persistent": "ws_kernel (persistent wide sweep: the timed sweeps in one launch)", "lds": "sweep_kernel<NW,true>", "global": "sweep_kernel<NW,false>", "blocked": "sweep_blocked_kernel",
           "tiled": "sweep_tiled_kernel", "wide": "wide_tscan+wide_eval(+walks)+commit (one sweep)",
           "ref-wide": "refw_scan+refw_rows+refw_walk+refw_commit (one sweep)"}


def ctx_stats(ctx) -> tuple:
    """(dense, wide incremental, persistent wide) device statistics of a context handle -- a single
    context or a partitioned rank: the bench prices a sweep by what these count, on every line."""
    from mcmc_colorer_amd._lib import check, lib

    def q(fn, k):
        out = (ctypes.c_uint64 * k)()
        check(getattr(lib(), fn)(ctx, out))
        return [int(x) for x in out]
    d = q("mcmc_get_dense_stats_v2", 16)
    dense = {"enabled": bool(d[0]), "s0": d[1], "s1": d[2], "incremental_sweeps": d[3], "rebuilds": d[4],
             "moved_vertices": d[5], "open_rows": d[6], "rebuild_threshold": d[7], "changed_rows": d[8],
             "copy_sweeps": d[9], "solo_sweeps": d[10], "window_states": d[11], "persistent": bool(d[12]),
             "open_words": d[13], "solo_evaluated": d[14]}
    i = q("mcmc_get_wide_inc_stats", 5)
    inc = {"enabled": bool(i[0]), "incremental_sweeps": i[1], "full_sweeps": i[2], "changed_rows": i[3],
           "changed_arcs": i[4]}
    w = q("mcmc_get_wide_solo_stats", 30)
    keys = ("enabled", "window_states", "sweeps", "phases", "leader_walks", "walk_phases", "delta_phases",
            "collects", "candidates", "changed_rows")
    ws = {k: v for k, v in zip(keys, w)}
    steps = ("walks", "candidates", "walk_wait", "events", "changes", "count_moves", "violator_list", "sweep")
    ws["step_us"] = {k: w[14 + j] / 100.0 for j, k in enumerate(steps)}
    ws["probe_us"] = [w[22 + j] / 100.0 for j in range(8)]
    return dense, inc, ws


def load_traffic(key: str):
    """HBM bytes per sweep from the committed rocprofv3 PMC summary (or None): a persistent launch's
    bytes divided by the sweeps it ran (make_pmc_summary.py sweeps-per-launch)."""
    p = ROOT / "profiles" / "pmc_summary.json"
    if not p.exists():
        return None
    try:
        e = json.loads(p.read_text()).get(key, {})
        return e.get("hbm_bytes_per_sweep", e.get("hbm_bytes_per_launch"))
    except Exception:
        return None


def host_info() -> dict:
    """The GPU box's host: logical CPUs, the CPUs this process may use, the CPU model."""
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"nproc": os.cpu_count(), "usable_cpus": usable, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(off: np.ndarray, idx: np.ndarray, ncol: int, seed: int, window: np.ndarray, n: int,
                 max_seconds: float = 20.0):
    """Oracle (tests/oracle_ref.py) on this host, a bounded sample of sweeps: the faithful
    single-thread restatement of ColoringMCMC_CPU::run (the reference's --mcmccpu is single-threaded:
    the headline value, cores = 1), then its OpenMP variant (bit-identical colouring) on all the CPUs
    this process may use (OMP_NUM_THREADS, else the affinity mask) as `all_cores`."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as O

    def sample(threads: int, budget: float):
        O.set_glibc_window(window)
        r = O.mcmc_run(off, idx, ncol, seed, sweep_limit=1, nthreads=threads)
        one = r.res.loopSeconds
        k = max(1, min(30, int(budget / max(one, 1e-3))))
        O.set_glibc_window(window)
        r = O.mcmc_run(off, idx, ncol, seed, sweep_limit=k, nthreads=threads)
        return n * r.res.sweepsRun / r.res.loopSeconds, r.res.sweepsRun, r

    t0 = time.perf_counter()
    v1, k1, r1 = sample(1, max_seconds)
    w1 = time.perf_counter() - t0
    info = host_info()
    # The GPU pool gives one GPU's job a share of the host's CPUs (OMP_NUM_THREADS = 16 on the box;
    # the affinity mask still lists every CPU of the machine, which other jobs use): the OpenMP leg
    # runs on that share, and its per-thread rate scaled to every usable CPU is reported beside it
    # as an upper bound for the CPU path on the whole host (linear scaling assumed, not measured)
    threads = int(os.environ.get("OMP_NUM_THREADS") or info["usable_cpus"] or 1)
    t0 = time.perf_counter()
    vN, kN, rN = sample(threads, max_seconds / 2)
    wN = time.perf_counter() - t0
    return {
        "value": v1,
        "unit": "vertex-updates/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {k1} sweeps of the same graph/seed (oracle single-thread restatement of "
                  f"ColoringMCMC_CPU::run incl. its 4 arc passes/sweep, debugger hook excluded); {w1:.1f} s wall",
        "host": info,
        "all_cores": {"value": vN, "unit": "vertex-updates/s", "cores": threads, "kind": "port",
                      "sample": f"first {kN} sweeps, OpenMP variant of the oracle on {threads} threads (same "
                                f"colouring as the single-thread run; loop 2 / fill_qstar, output-dead, skipped); "
                                f"{wN:.1f} s wall",
                      "identical_trajectory_prefix": bool(np.array_equal(r1.traj[:min(k1, kN)], rN.traj[:min(k1, kN)])),
                      "cpu_share_note": "threads = the job's CPU share on the GPU box (OMP_NUM_THREADS); the "
                                        "pool's rules reserve the other CPUs of the machine for other jobs"},
        "all_usable_cpus_extrapolated": {
            "value": vN / threads * (info["usable_cpus"] or threads), "cores": info["usable_cpus"],
            "kind": "extrapolation",
            "note": f"all_cores' per-thread rate x {info['usable_cpus']} usable CPUs (linear scaling assumed, "
                    f"an upper bound for the CPU path on this host; not measured)"},
    }


def cpu_baseline_ref(off: np.ndarray, idx: np.ndarray, ncol: int, seed: int, n: int, max_seconds: float = 20.0):
    """Oracle restatement of the reference GPU colorer (oracle/mcmc_gpu_ref.cpp), single thread, a
    bounded number of sweeps (maxRip = k: k sweeps, a conflict count before each and after the last)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as O

    st0 = O.gpurand_init(n, seed)
    t0 = time.perf_counter()
    st = st0.copy()
    t = time.perf_counter()
    O.mcmc_gpu_run(off, idx, ncol, st, maxRip=1)
    one = time.perf_counter() - t
    k = max(1, min(30, int(max_seconds / max(one, 1e-3))))
    st = st0.copy()
    t = time.perf_counter()
    r = O.mcmc_gpu_run(off, idx, ncol, st, maxRip=k)
    loop = time.perf_counter() - t
    return {
        "value": n * r.res.sweeps / loop,
        "unit": "vertex-updates/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{r.res.sweeps} sweeps of the same graph/seed (oracle single-thread restatement of the "
                  f"reference GPU colorer: conflict count + balance-dynamic selection per sweep); "
                  f"{time.perf_counter() - t0:.1f} s wall",
    }


def refstruct_baseline(g, ncol: int, sweeps: int, seed: int, n: int, value: float) -> dict:
    """The reference CUDA path's per-sweep structure re-expressed in HIP (mcmc_refstruct_bench):
    the stand-in for 'the reference CUDA path's vertex-updates/sec', which cannot run on MI355X. Its analytic
    byte model (§8d): 3 uint32 arc passes (2 conflict counts + the selection) + 3 offset passes + the n*nCol
    checker reset + the per-vertex colour/state traffic, and 8n B over PCIe (4n B D2H of the colouring for
    the host histogram, plus the conflict partial sums)."""
    from mcmc_colorer_amd._lib import check, lib

    ms = ctypes.c_double()
    conf = ctypes.c_uint64()
    check(lib().mcmc_refstruct_bench(g.handle, ncol, sweeps, seed, ctypes.byref(ms), ctypes.byref(conf)))
    v = n / (ms.value * 1e-3)
    m = g.nEdges
    # uint32 ids of 3 arc passes; row offsets of 3 passes; checker reset + the selection's nCol scan of
    # it; own colour / count / taboo / Cs / qs words; 48 B XORWOW state read + written per vertex
    hbm = 3 * 4 * m + 3 * 8 * (n + 1) + 2 * n * ncol + 4 * n * 6 + 48 * 2 * n
    return {"value": v, "unit": "vertex-updates/s", "ms_per_sweep": ms.value, "sweeps": sweeps,
            "speedup": value / v,
            "model_bytes_hbm": hbm, "model_bytes_pcie": 8 * n,
            "achieved_GBs": hbm / (ms.value * 1e-3) / 1e9, "frac_of_hbm_peak": hbm / (ms.value * 1e-3) / 1e9 / HBM_PEAK_GBS,
            # the same structure if it streamed its model bytes at the HBM peak: an upper bound for any
            # implementation of the reference's per-sweep structure on this chip
            "bound_value_at_hbm_peak": n / (hbm / (HBM_PEAK_GBS * 1e9)),
            "speedup_vs_bound": value / (n / (hbm / (HBM_PEAK_GBS * 1e9))),
            "what": "HIP re-expression of ColoringMCMC::run's per-sweep structure (thread-per-vertex serial "
                    "row walks, 64-thread blocks, n*nCol checker memset, 2 conflict passes + host sums, 4n B "
                    "D2H + host histogram + H2D), host wall per sweep"}


def refstruct_full_occupancy(dev: int, ncol: int, seed: int, value: float, sweeps: int) -> dict:
    """refstruct on a graph with C3's mean degree (1e4) that fills the chip at thread-per-vertex: 2e6
    rows (31250 64-thread blocks, ~30 waves per SIMD), 2e10 arcs, the reference's uint32 CSR (80 GB)
    materialised on the device from the build's G(n, p). Per-vertex work is per-degree, so its rate
    compares directly with C3's (same degree, 1e7 rows)."""
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    t0 = time.perf_counter()
    g = M.Graph.er_fast(2_000_000, 0.005, 1, device=dev)
    check(lib().mcmc_graph_materialize_csr(g.handle))
    gen = time.perf_counter() - t0
    r = refstruct_baseline(g, ncol, sweeps, seed, g.nNodes, value)
    r["graph"] = (f"the build's G(n, p) with n = 2e6, p = 0.005 (mean degree {g.nEdges / g.nNodes:.0f} = C3's), "
                  f"{g.nEdges} arcs as a uint32 CSR on the device ({gen:.1f} s to build)")
    g.close()
    return r


def rank_share(a, dev: int = 0) -> dict:
    """One rank's share of configs[3] on one GPU: rows [0, n/K) of the C3 graph (every rank of the
    equal-rows plan holds as many rows and, G(n, p) being uniform, as many arcs), generated alone
    (Graph.er_fast(rows=...)), timed two ways:
      plain: a context over those rows, the one-GPU step (the sweep commits in its last workgroup),
             K steps as one hipGraph -- what the rank's sweep itself costs;
      rank:  a world-K partitioned context of rank 0 through the native driver (mcmc_part_bench_rank):
             sweep with the delta packing and footer, the part_commit launch, batches and polling,
             with the exchange left out -- everything of a world-K step but the RCCL transfers.
    The strong-scaling budget is the one-GPU C3 step / 6 (north_star: >= 6x at 8 GPUs)."""
    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import MCMCRunStats, check, lib, u32ptr
    from mcmc_colorer_amd.distributed import plan_rows

    n, p, K = 10_000_000, 0.001, a.rank_share
    bounds = plan_rows(n, K)
    b1 = int(bounds[1])
    t0 = time.perf_counter()
    g = M.Graph.er_fast(n, p, 1, device=dev, rows=(0, b1))
    gen = time.perf_counter() - t0
    params = M.ColoringMCMCParams(nCol=32, maxRip=0x7FFFFFF0)
    tot, ker = ctypes.c_double(), ctypes.c_double()
    col = M.ColoringMCMC(g, M.GPURand(n, a.seed, M.GlibcRand(1)), params, v_begin=0, v_end=b1)
    col.init(0)
    if a.warmup:
        check(lib().mcmc_bench_sweeps(col._ctx, a.warmup, ctypes.byref(tot), ctypes.byref(ker)))
    check(lib().mcmc_bench_prepare(col._ctx, a.steps))
    t1 = time.perf_counter()
    check(lib().mcmc_bench_sweeps(col._ctx, a.steps, ctypes.byref(tot), ctypes.byref(ker)))
    plain_wall = time.perf_counter() - t1
    info = col.info()
    col.close()
    prm = params.to_c(a.seed)
    ctx = ctypes.c_void_p()
    check(lib().mcmc_part_create(g.handle, ctypes.byref(prm), K, 0, u32ptr(bounds), None, ctypes.byref(ctx)))
    check(lib().mcmc_set_glibc_window(ctx, u32ptr(M.GlibcRand(1).window)))
    check(lib().mcmc_init_coloring(ctx, None))
    check(lib().mcmc_set_bench_mode(ctx, 1))
    st = MCMCRunStats()
    if a.warmup:
        check(lib().mcmc_part_bench_rank(ctx, a.warmup, ctypes.byref(st)))
    t1 = time.perf_counter()
    check(lib().mcmc_part_bench_rank(ctx, a.steps, ctypes.byref(st)))
    rank_wall = time.perf_counter() - t1
    rank_dev = st.loopMs / a.steps
    xs = [ctypes.c_uint64() for _ in range(4)]
    check(lib().mcmc_part_exchange_stats(ctx, *[ctypes.byref(x) for x in xs]))
    lib().mcmc_destroy(ctx)
    full_ms = 0.8955   # BENCH_r03.json (driver): the one-GPU C3 step
    return {
        "metric": "ms per step of one rank's share of configs[3]",
        "rank_share": K, "rows": b1, "arcs": g.nEdges, "graph_gen_s": round(gen, 2),
        "steps": a.steps, "warmup": a.warmup,
        "plain": {"ms_per_step": plain_wall * 1e3 / a.steps, "device_ms_per_step": ker.value,
                  "what": "context over rows [0, n/K), one-GPU fused step, hipGraph of the K steps"},
        "rank": {"ms_per_step": rank_wall * 1e3 / a.steps, "device_ms_per_step": rank_dev,
                 "delta_steps": xs[0].value, "full_steps": xs[1].value, "overflows": xs[2].value,
                 "what": "world-K rank 0 through mcmc_part_bench_rank: sweep + delta packing + part_commit "
                         "launch + driver batches/polls, exchange left out (RCCL over xGMI unmeasured)"},
        "budget_ms": full_ms / 6.0, "one_gpu_c3_ms": full_ms,
        "layout": info,
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=["c2", "c3", "c5"], default="c3",
                    help="c2: configs[1] (--simulate 0.01 -n 1e5, 16 colours; weak scaling at N > 1); "
                         "c3: configs[2]/[3] (n 1e7, p 0.001, 32 colours, the build's G(n,p) generator; "
                         "N > 1 partitions the same graph: strong scaling)")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--vertices", type=int, default=100000, help="n of --simulate (per GPU under weak scaling)")
    ap.add_argument("--prob", type=float, default=0.01)
    ap.add_argument("--ncol", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-refstruct", action="store_true", help="skip the refstruct (reference-structure) leg")
    ap.add_argument("--no-convergence", action="store_true", help="skip the reference-loop run (sweeps-to-zero-conflict)")
    ap.add_argument("--no-full-scan", action="store_true", help="skip the full-scan (MCMC_FULL_SCAN=1) comparison")
    ap.add_argument("--refstruct-sweeps", type=int, default=10)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--force-dist", action="store_true",
                    help="the native partitioned driver (RCCL inside the library) even at world size 1")
    ap.add_argument("--semantics", choices=["cpu", "ref"], default="cpu",
                    help="cpu: --mcmccpu semantics (the north-star path); ref: the reference GPU colorer's own "
                         "semantics (--mcmcgpu-ref), one GPU")
    ap.add_argument("--variant", default=None,
                    help="sweep kernel: lds | tiled | blocked | global[:block_log2[:lanes_log2[:group_rows"
                         "[:stream]]]] (empty field / default: the library's choice)")
    ap.add_argument("--rank-share", type=int, default=0,
                    help="K > 1: time one rank's share of configs[3] (rows [0, n/K) of the C3 graph) on this GPU, "
                         "as a plain sweep and as a world-K rank with the exchange left out (rank_share)")
    a = ap.parse_args()
    if a.rank_share > 1:
        print(json.dumps(rank_share(a)), flush=True)
        return 0
    if a.variant:
        for key, v in zip(("MCMC_GATHER", "MCMC_BLOCK_LOG2", "MCMC_SUB_LOG2", "MCMC_GROUP_ROWS",
                           "MCMC_TILE_STREAM"), a.variant.split(":")):
            if v:
                os.environ[key] = v

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or a.force_dist:
        import torch
        import torch.distributed as dist

        # The data path's RCCL communicator lives inside libmcmc_hip.so (mcmc_comm_init_rank,
        # mcmc_part_run); torch.distributed only carries rank 0's unique id, the barriers and the
        # max over ranks, on the CPU (gloo)
        torch.cuda.set_device(local)
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)   # --force-dist without a launcher: world 1
        dist.init_process_group("gloo")

    import mcmc_colorer_amd.colorer as M
    from mcmc_colorer_amd._lib import check, lib

    dev = local
    n_req, p_req = a.vertices, a.prob
    if a.config == "c3":
        n_req, p_req, a.ncol, a.scaling = 10_000_000, 0.001, 32, "strong"
    elif a.config == "c5":   # one fixed graph: N > 1 partitions it (strong scaling), like configs[3]
        n_req, p_req, a.scaling = 1 << 22, 0.0, "strong"
    elif world > 1 and a.scaling == "weak":
        n_req, p_req = a.vertices * world, a.prob / world
    t_gen = time.perf_counter()
    rng = M.GlibcRand(1)
    bounds = None
    if a.config == "c3":
        # setupRnd2 is infeasible at n = 1e7 (5e13 draws): the build's documented generator, fixed seed 1,
        # written straight into the tiled layout; under torchrun each rank generates only its rows of
        # the equal-rows plan (G(n, p) is uniform: equal rows are arc-balanced)
        if dist is not None:
            from mcmc_colorer_amd.distributed import plan_rows

            bounds = plan_rows(n_req, world)
            g = M.Graph.er_fast(n_req, p_req, 1, device=dev, rows=(int(bounds[rank]), int(bounds[rank + 1])))
        else:
            g = M.Graph.er_fast(n_req, p_req, 1, device=dev)
    elif a.config == "c5":
        g = M.Graph.rmat(22, 10, 0.5, 0.2, 0.2, 1, device=dev)
        a.ncol = g.getMaxNodeDeg()   # main.cu:162 default: maxDeg * numColRatio (1)
    else:
        g = M.Graph.simulate(n_req, p_req, rng, device=dev)
    if dist is not None and bounds is None:   # power-law C5: arc-balanced plan from the degree prefix
        from mcmc_colorer_amd.distributed import plan

        bounds = plan(g, world, balance=True)
    t_gen = time.perf_counter() - t_gen
    params = M.ColoringMCMCParams(nCol=a.ncol, maxRip=0x7FFFFFF0)   # throughput mode: no cap
    tot = ctypes.c_double()
    ker = ctypes.c_double()

    def barrier():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    ref = a.semantics == "ref"
    conv = None
    if dist is None and not ref and not a.no_convergence:
        # the reference loop itself (run(), coloringMCMC_CPU.cpp:115-270) from the initial colouring:
        # until Cviol <= z or the cap (maxRip 250: at most 251 sweeps, :264-269); the metric's second
        # half -- sweeps-to-zero-conflict, or "not converged at 251" with the final Cviol and the
        # per-sweep trajectory
        window = (M.GlibcRand(1, n_req * (n_req + 1) // 2) if a.config == "c2" else M.GlibcRand(1))
        cr = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, window), M.ColoringMCMCParams(nCol=a.ncol))
        t0 = time.perf_counter()
        st = cr.run(0)
        cw = time.perf_counter() - t0
        tr = [int(x) for x in cr.trajectory()]
        # the first sweep of a colouring alone (the dense sweep's count rebuild happens there), then
        # one more: their difference is the rebuild's cost, paid once per colouring
        cf = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, M.GlibcRand(1) if a.config != "c2" else
                                         M.GlibcRand(1, n_req * (n_req + 1) // 2)), M.ColoringMCMCParams(nCol=a.ncol))
        cf.init(0)
        s1 = cf.step(1)
        s2 = cf.step(1)
        cf.close()
        conv = {"sweeps_to_zero_conflict": int(st.iter) if st.finalViol == 0 else None,
                "converged": bool(st.finalViol == 0),
                "status": (f"converged after {int(st.iter)} sweeps" if st.finalViol == 0 else
                           f"not converged at {int(st.iter)} (maxRip 250 cap: {int(st.sweepsRun)} sweeps run)"),
                "iterations": int(st.iter), "max_iter_reached": bool(st.maxIterReached),
                "final_Cviol": int(st.finalViol), "sweeps_run": int(st.sweepsRun),
                "loop_ms": st.loopMs, "wall_s": round(cw, 4), "glibc_draws": int(st.glibcDraws),
                "amortized_ms_per_sweep": st.loopMs / max(1, int(st.sweepsRun)),
                "amortized_value": g.nNodes * int(st.sweepsRun) / (st.loopMs * 1e-3),
                "first_sweep_ms": s1.loopMs, "second_sweep_ms": s2.loopMs,
                "rebuild_ms": max(0.0, s1.loopMs - s2.loopMs),
                "note": "loop_ms = device time of the whole reference loop (run(), every sweep incl. the first "
                        "sweep's count rebuild); amortized_* = that loop per sweep; first/second_sweep_ms = one-sweep "
                        "launches of a fresh colouring, their difference the rebuild paid once per colouring",
                "trajectory": tr}
        cr.close()
    if ref and dist is not None:
        raise SystemExit("--semantics ref runs on one GPU")
    if dist is None:
        if ref:
            states = M.CurandStates(g.nNodes, a.seed, dev)
            col = M.ColoringMCMCGpuRef(g, states, params)
            col.init()
        else:
            col = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, rng), params)
            col.init(0)
        if a.warmup:
            # the last warm-up sweep on its own: its launch takes the path the timed sweeps will (the
            # persistent wide sweep once the colouring is nearly proper) and pays that path's entry
            # (violator list, counts) outside the timed region, as a long run amortises it
            if a.warmup > 1:
                check(lib().mcmc_bench_sweeps(col._ctx, a.warmup - 1, ctypes.byref(tot), ctypes.byref(ker)))
            check(lib().mcmc_bench_sweeps(col._ctx, 1, ctypes.byref(tot), ctypes.byref(ker)))
        check(lib().mcmc_bench_prepare(col._ctx, a.steps))   # graph instantiation outside the timed region
        dn0, inc0, ws0 = (None, None, None) if ref else ctx_stats(col._ctx)
        t0 = time.perf_counter()
        check(lib().mcmc_bench_sweeps(col._ctx, a.steps, ctypes.byref(tot), ctypes.byref(ker)))
        wall = time.perf_counter() - t0
        kernel_ms = ker.value
        info = col.info()
        dn1, inc1, ws1 = (None, None, None) if ref else ctx_stats(col._ctx)
    else:
        import torch

        from mcmc_colorer_amd._lib import MCMCRunStats
        from mcmc_colorer_amd.distributed import NativePartitionedColoringMCMC

        drv = NativePartitionedColoringMCMC(g, M.GPURand(g.nNodes, a.seed, rng), params, bounds, device=local)
        drv.init(0)
        check(lib().mcmc_set_bench_mode(drv._ctx, 1))   # throughput mode: no convergence stop
        arr = (ctypes.c_void_p * 1)(drv._ctx.value)
        st = MCMCRunStats()
        if a.warmup:
            check(lib().mcmc_part_run(arr, 1, a.warmup, ctypes.byref(st)))
        dn0, inc0, ws0 = ctx_stats(drv._ctx)
        barrier()
        t0 = time.perf_counter()
        check(lib().mcmc_part_run(arr, 1, a.steps, ctypes.byref(st)))   # sweeps + RCCL exchanges + commits
        barrier()
        dn1, inc1, ws1 = ctx_stats(drv._ctx)
        wall = time.perf_counter() - t0
        kernel_ms = st.loopMs / a.steps   # device time of one whole step on this rank's stream
        xs = [ctypes.c_uint64() for _ in range(4)]
        check(lib().mcmc_part_exchange_stats(drv._ctx, *[ctypes.byref(x) for x in xs]))
        exchange = {"delta_steps": xs[0].value, "full_steps": xs[1].value, "overflows": xs[2].value,
                    "bytes_sent": xs[3].value, "bytes_sent_per_step": xs[3].value / max(1, a.steps),
                    "what": "this rank's timed steps (mcmc_part_exchange_stats); world 1 sends nothing"}
        info = drv.info()
        info["bounds"] = [int(x) for x in bounds]
        w = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())

    n, m = g.nNodes, g.nEdges
    if dist is not None and a.config == "c3":   # per-rank graphs hold their rows' arcs only
        import torch

        mt = torch.tensor([m], dtype=torch.float64)
        dist.all_reduce(mt)
        m = int(mt.item())
    value = n * a.steps / wall          # all ranks together update n vertices per sweep
    # dominant kernel's bytes per launch on this rank: B_fmt of the layout it streams (SURVEY.md
    # §8d: with a compressed format the fraction is taken against the format's bytes), and the
    # same rows' B_alg in the reference's uint32 layout for comparison
    b_fmt, b_ref = info["sweep_bytes"], info["ref_bytes"]
    variant = info["variant"]
    scan = None
    b_alg = b_fmt
    dense_on = bool(dn1 and dn1["enabled"])
    if dense_on:
        variant = "dense"
    nrows = g.nNodes if dist is None else int(bounds[rank + 1] - bounds[rank])   # this context's rows
    dense = None
    if dense_on:
        # the dense-count sweep (csrc/dense_counts.h): per sweep every row's own colour and its open
        # bits (NW bits) read; per row that changed colour its new colour written, and the restore
        # (read + write) into the next sweep's buffer; per vertex of the dense range that changed
        # colour its local arcs (id + two count atomics); rows that scanned past the range (their
        # dense mask, ids + colour gathers, an upper bound: their whole rows outside it); a rebuild
        # reads every row's arcs into the range and copies the local colours
        d = {k: dn1[k] - dn0[k] for k in ("incremental_sweeps", "rebuilds", "moved_vertices", "open_rows",
                                          "changed_rows", "copy_sweeps", "solo_sweeps", "solo_evaluated")}
        S = max(1, d["incremental_sweeps"] + d["rebuilds"])
        nw = 1 if a.ncol <= 32 else 2 if a.ncol <= 64 else 4 if a.ncol <= 128 else 8
        deg = m / max(1, n)
        span = dn1["s1"] - dn1["s0"]
        # bytes from what the device counted (one definition for every dense line): a full sweep reads
        # every row's colour and open bits; a solo sweep (dense_sparse.h) reads the colour and open word
        # of each row it evaluates (candidates of the discrete-log window, open rows); a changed row
        # writes its colour (both buffers in solo sweeps, restore in full ones) and a list entry; a
        # moved vertex of S reads its local arcs (2 B ids) and moves two 4 B counts per arc; an open
        # row reads its mask and its arcs outside S with their colours (3 B per arc); a rebuild reads
        # the rows' arcs into S and writes counts, masks and a copy of the colours
        # (this context's rows: a partitioned rank prices its own rows the same way)
        full = S - d["solo_sweeps"]
        b_eval = full * nrows * (1.0 + nw / 8.0) + d["solo_evaluated"] * 9.0
        b_chg = d["changed_rows"] * 10.0 + d["copy_sweeps"] * 2.0 * nrows
        b_upd = d["moved_vertices"] * deg * (nrows / max(1, n)) * 10.0
        b_open = d["open_rows"] * (4.0 * nw + deg * (1.0 - span / max(1, n)) * 3.0)
        b_rebuild = d["rebuilds"] * (nrows * deg * span / max(1, n) * 2.0 + nrows * a.ncol * 4.0 + nrows * nw * 4.0
                                     + 2.0 * nrows)
        b_alg = (b_eval + b_chg + b_upd + b_open + b_rebuild) / S
        dense = dict(d, sweeps_counted=S, dense_range=[dn1["s0"], dn1["s1"]],
                     window_states=dn1["window_states"], persistent=dn1["persistent"],
                     solo_evaluated_per_sweep=d["solo_evaluated"] / S,
                     moved_vertices_per_sweep=d["moved_vertices"] / S, open_rows_per_sweep=d["open_rows"] / S,
                     rebuild_threshold=dn1["rebuild_threshold"], bytes_per_sweep=b_alg,
                     changed_rows_per_sweep=d["changed_rows"] / S,
                     bytes={"evaluation": b_eval, "changed_rows": b_chg / S, "updates": b_upd / S,
                            "open_rows": b_open / S, "rebuilds": b_rebuild / S},
                     note="dense-count sweep: every row keeps the counts of its neighbours' colours over a fixed "
                          "dense column range, moved each sweep by the vertices there that changed colour; a row "
                          "whose dense mask holds every colour (open bit clear) keeps its colour unless its minstd "
                          "state falls in the candidate window, whose rows are found by discrete logarithm "
                          "(csrc/dense_sparse.h): a solo sweep evaluates only those and the open rows, on one "
                          "workgroup of a persistent launch of all the timed sweeps; full sweeps (the count "
                          "rebuild) run on the whole grid inside it. Bit-identical to the scan sweeps "
                          "(tests/test_dense.py, tests/test_c3_full.py).")
        if conv is not None and conv.get("rebuild_ms"):
            # the count rebuild of a fresh colouring (dc_rebuild_kernel, once per colouring): every row's
            # ids inside S (2 B each), its nCol counts and mask words written, the colours copied
            rb_bytes = (nrows * deg * span / max(1, n) * 2.0 + nrows * a.ncol * 4.0 + nrows * nw * 4.0
                        + 2.0 * nrows)
            rb_gbs = rb_bytes / (conv["rebuild_ms"] * 1e-3) / 1e9
            dense["rebuild"] = {"ms": conv["rebuild_ms"], "bytes": rb_bytes, "achieved_GBs": rb_gbs,
                                "frac": rb_gbs / HBM_PEAK_GBS, "traffic": load_traffic("c3/rebuild") if a.config == "c3" else None,
                                "what": "first-sweep minus second-sweep device time of a fresh colouring (the count rebuild, "
                                        "csrc/dense_counts.h dc_rebuild_kernel); bytes: ids into S, counts, masks, copy"}
        if not a.no_full_scan and dist is None:
            # the same graph through the tiled scan sweep (MCMC_DENSE=0, the r03 early-exit kernel) and
            # the full scan (MCMC_FULL_SCAN=1): every sweep scans the layout
            for label, env in (("scan_sweep", "MCMC_DENSE"), ("full_scan", "MCMC_FULL_SCAN")):
                os.environ[env] = "0" if env == "MCMC_DENSE" else "1"
                cf = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, M.GlibcRand(1)), params)
                cf.init(0)
                tot2, ker2 = ctypes.c_double(), ctypes.c_double()
                check(lib().mcmc_bench_sweeps(cf._ctx, 3, ctypes.byref(tot2), ctypes.byref(ker2)))
                k = max(3, min(a.steps, 10))
                check(lib().mcmc_bench_sweeps(cf._ctx, k, ctypes.byref(tot2), ctypes.byref(ker2)))
                os.environ.pop(env)
                fi = cf.info()
                dense[label] = {"ms_per_sweep": ker2.value, "value": g.nNodes / (ker2.value * 1e-3), "sweeps": k,
                                "layout_bytes": fi["sweep_bytes"],
                                "layout_frac_if_full": fi["sweep_bytes"] / (ker2.value * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                "what": ("the tiled early-exit scan (MCMC_DENSE=0)" if env == "MCMC_DENSE" else
                                         "every arc scanned (MCMC_FULL_SCAN=1)")}
                cf.close()
    if not ref and variant == "tiled":
        # The tiled sweep stops scanning a row once its occupancy mask holds every colour (the
        # result cannot change; MCMC_FULL_SCAN=1 scans every arc): the bytes one launch moves are
        # counted on the device (mcmc_set_scan_stats, 3 sweeps outside the timed region) -- id quads,
        # the staged (group, block) pairs' table rows and colour slices, own colour read + write
        tot2, ker2 = ctypes.c_double(), ctypes.c_double()
        sctx = col._ctx if dist is None else drv._ctx
        check(lib().mcmc_set_scan_stats(sctx, 1))
        if dist is None:
            check(lib().mcmc_bench_sweeps(col._ctx, 3, ctypes.byref(tot2), ctypes.byref(ker2)))
        else:
            check(lib().mcmc_part_run(arr, 1, 3, ctypes.byref(st)))
        sv = (ctypes.c_uint64 * 6)()
        check(lib().mcmc_get_scan_stats_v2(sctx, sv))
        check(lib().mcmc_set_scan_stats(sctx, 0))
        # algorithmic: the quads whose ids the scan gathered (the exact early exit needs them);
        # issued: every quad loaded, incl. those fetched ahead for a row that filled up first; plus
        # the segment tables of the pairs, the colour slices staged (the tail queue keeps the two
        # dense blocks' slices resident: 2 per workgroup, then one per tail block), the tail queue's
        # entries (16 B written, 16 B read + 16 B of segment bounds / group base per read)
        quads_issued, pairs, quads, slices, qw, qr = [x / 3.0 for x in sv]
        R = info["grp_rows"]
        table = 4 * ((R + 4) & ~3)
        slice_b = 0 if info["resident"] else min(1 << info["block_log2"], ((g.nNodes + 15) // 16) * 16)
        nloc = g.nNodes if dist is None else int(bounds[rank + 1] - bounds[rank])
        rest = pairs * table + slices * slice_b + 16 * qw + 32 * qr + 2 * nloc
        b_alg = 16 * quads + rest
        scan = {"early_exit": info.get("early", True), "quads_per_sweep": quads, "pairs_per_sweep": pairs,
                "id_bytes": 16 * quads, "table_bytes": pairs * table, "slices_per_sweep": slices,
                "slice_bytes": slices * slice_b, "tail_queue_entries_written": qw, "tail_queue_entries_read": qr,
                "tail_queue_bytes": 16 * qw + 32 * qr,
                "quads_issued_per_sweep": quads_issued,
                "issued_bytes": 16 * quads_issued + rest,
                "layout_bytes_full_scan": b_fmt,
                "note": "exact early exit: a row's scan stops once its mask holds all nCol colours "
                        "(count_free_colors cannot change); rows still open after the two dense blocks wait "
                        "in the workgroup's tail queue and finish block by block after its last group. "
                        "Bit-identical results (tests/test_gpu_parity.py, tests/test_c3_full.py)."}
        if dist is None and not a.no_full_scan:
            # the same sweep scanning every arc (MCMC_FULL_SCAN=1): the layout-bound reference point
            os.environ["MCMC_FULL_SCAN"] = "1"
            cf = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, M.GlibcRand(1)), params)
            cf.init(0)
            check(lib().mcmc_bench_sweeps(cf._ctx, 2, ctypes.byref(tot2), ctypes.byref(ker2)))
            k = max(3, min(a.steps, 10))
            check(lib().mcmc_bench_sweeps(cf._ctx, k, ctypes.byref(tot2), ctypes.byref(ker2)))
            os.environ.pop("MCMC_FULL_SCAN")
            scan["full_scan"] = {"ms_per_sweep": ker2.value, "value": g.nNodes / (ker2.value * 1e-3),
                                 "sweeps": k, "bytes": b_fmt,
                                 "achieved_GBs": b_fmt / (ker2.value * 1e-3) / 1e9,
                                 "frac": b_fmt / (ker2.value * 1e-3) / 1e9 / HBM_PEAK_GBS}
            cf.close()
    wide_inc = None
    if not ref and variant == "wide" and inc1 and inc1["enabled"]:
        # incremental violation counts (sweep_wide.h wide_inc_*): a sweep moves the counts by the rows
        # that changed colour instead of scanning the slab layout, so it is priced by what it reads:
        # per vertex its flag and colour (3 B), per changed row its offsets, list entries and the
        # replica / fingerprint sync (30 B), per changed arc its id and both colour reads (8 B); a
        # full recount sweep (the first, or after many changes) by the layout's B_fmt
        d = {k: inc1[k] - inc0[k] for k in ("incremental_sweeps", "full_sweeps", "changed_rows", "changed_arcs")}
        S = max(1, d["incremental_sweeps"] + d["full_sweeps"])
        # persistent sweeps (csrc/wide_solo.h) read no per-vertex state: per candidate row of the
        # discrete-log window its table entry, colour and count (14 B), per violator its row's ids and
        # colours as the walks do (priced with the changed arcs: 8 B per arc)
        pw = {k: ws1[k] - ws0[k] for k in ("sweeps", "phases", "leader_walks", "walk_phases", "delta_phases",
                                            "collects", "candidates", "changed_rows")} if ws1 and ws1["enabled"] else None
        nws = pw["sweeps"] if pw else 0
        b_alg = (3.0 * nrows * max(0, d["incremental_sweeps"] - nws) + 14.0 * (pw["candidates"] if pw else 0)
                 + 30.0 * d["changed_rows"] + 8.0 * d["changed_arcs"] + b_fmt * d["full_sweeps"]) / S
        wide_inc = dict(d, sweeps_counted=S, changed_rows_per_sweep=d["changed_rows"] / S,
                        changed_arcs_per_sweep=d["changed_arcs"] / S, bytes_per_sweep=b_alg,
                        layout_bytes_full_sweep=b_fmt,
                        note="exact incremental violation counts: each sweep moves every row's same-colour "
                             "count by the rows that changed colour (a full recount over the slab layout when "
                             "many change); bit-identical to the full scan (tests/test_wide.py::"
                             "test_wide_incremental_counts). The roofline prices the sweep by these bytes: it "
                             "is bound by launch and dependent-latency chains, not by HBM.")
        if pw:
            wide_inc["persistent"] = dict(pw, window_states=ws1["window_states"],
                                          candidates_per_sweep=pw["candidates"] / max(1, nws),
                                          step_us_per_sweep={k: (ws1["step_us"][k] - ws0["step_us"][k]) / max(1, nws)
                                                             for k in ws1["step_us"]},
                                          probe_us_per_sweep=[(x - y) / max(1, nws)
                                                              for x, y in zip(ws1["probe_us"], ws0["probe_us"])],
                                          note="persistent wide sweep (csrc/wide_solo.h): one launch for the timed "
                                               "sweeps; a sweep evaluates the violators and the discrete-log "
                                               "window's candidate rows only, and moves the counts by the "
                                               "changed rows' arcs")
    achieved = b_alg / (kernel_ms * 1e-3) / 1e9
    key = f"{a.config}/{variant}" if (world == 1 and (a.config in ("c3", "c5") or n_req == 100000)) else None
    if key and ref:
        key += "-ref"
    data = {"c2": "synthetic (reference --simulate generator replayed exactly on the GPU)",
            "c3": "synthetic G(n,p) (the build's counter-based generator, er_gen.h, seed 1; setupRnd2 infeasible at n=1e7)",
            "c5": "synthetic R-MAT power-law stand-in for SNAP LiveJournal (er_gen.h rmat_edge, scale 22, edge factor "
                  "10, a/b/c 0.5/0.2/0.2, seed 1; the SNAP graphs are not available)"}[a.config]
    workload = (f"--mcmcgpu{'-ref' if ref else ''} --simulate {p_req:g} -n {n_req} --nCol {a.ncol} --seed {a.seed}"
                if a.config != "c5" else
                f"--mcmcgpu --graph <R-MAT scale 22 ef 10, LiveJournal stand-in> (nCol = maxDeg = {a.ncol}) --seed {a.seed}")
    out = {
        "metric": "vertex-updates/sec per MCMC sweep",
        "value": value,
        "unit": "vertex-updates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "strong" if a.config in ("c3", "c5") else ("weak" if (world == 1 or a.scaling == "weak") else "strong"),
        "vs_baseline": None,
        "dtype": "fp32",
        "data": data,
        "config": {"workload": workload,
                   "config": a.config,
                   "semantics": "reference GPU colorer (--mcmcgpu-ref)" if ref else "--mcmccpu (north star)",
                   "n": n, "arcs": m, "nCol": a.ncol,
                   "parallelism": (f"vertex-partitioned x{world} (native RCCL exchange per sweep, "
                                   f"{'arc-balanced' if a.config == 'c5' else 'equal-row'} plan)") if world > 1 else "single",
                   "graph_gen_s": round(t_gen, 3)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(key) if key else None,
                     "kernel": KERNELS.get(variant + ("-part" if (variant == "dense" and dist is not None) else "")
                                           + ("-persistent" if (wide_inc and "persistent" in wide_inc
                                                                and wide_inc["persistent"]["sweeps"]) else ""), variant)
                               + ("<REF>" if ref else "")
                               + ("" if world == 1 else " + exchange (per-rank step)"),
                     "kernel_ms": kernel_ms, "algorithmic_bytes": b_alg,
                     "ref_layout_bytes": b_ref, "ref_layout_equiv_GBs": b_ref / (kernel_ms * 1e-3) / 1e9,
                     "layout": info},
        "cpu_baseline": None,
    }
    if conv is not None:
        out["convergence"] = conv
    if wide_inc is not None:
        out["wide_inc"] = wide_inc
    if dense is not None:
        out["dense"] = dense
    if dist is not None:
        out["exchange"] = exchange
    if dist is None and a.config == "c5" and not a.no_convergence:
        # the wide sweep WITH violators in every timed sweep (nCol = maxDeg / 4 does not converge):
        # the reference loop capped at 20 sweeps, device time per sweep and the per-sweep Cviol
        nc4 = max(257, a.ncol // 4)
        cv = M.ColoringMCMC(g, M.GPURand(g.nNodes, a.seed, M.GlibcRand(1)), M.ColoringMCMCParams(nCol=nc4, maxRip=20))
        sv = cv.run(0)
        out["violators"] = {"nCol": nc4, "sweeps_run": int(sv.sweepsRun), "loop_ms": sv.loopMs,
                            "ms_per_sweep": sv.loopMs / max(1, sv.sweepsRun),
                            "value": g.nNodes * sv.sweepsRun / (sv.loopMs * 1e-3),
                            "trajectory": [int(x) for x in cv.trajectory()]}
        cv.close()
        # the three C5 rates side by side: `value` (sweeps of a converged colouring, throughput
        # mode), the violator-heavy loop above, and the reference loop itself at nCol = maxDeg from
        # C_0 (its sweeps: the violators of C_0, then the sweep that finds Cviol = 0 and stops)
        out["headline"] = {
            "converged_sweeps": {"value": value, "ms_per_sweep": wall * 1e3 / a.steps},
            "violator_sweeps": {"value": out["violators"]["value"], "ms_per_sweep": out["violators"]["ms_per_sweep"],
                                "nCol": nc4},
            "note": "value = converged-colouring sweeps; violator_sweeps = nCol maxDeg/4, every sweep with "
                    "violators and walks; reference_loop = run() from C_0 at nCol = maxDeg"}
        if conv is not None and conv["sweeps_run"]:
            out["headline"]["reference_loop"] = {
                "value": g.nNodes * conv["sweeps_run"] / (conv["loop_ms"] * 1e-3),
                "ms_per_sweep": conv["loop_ms"] / conv["sweeps_run"], "sweeps": conv["sweeps_run"],
                "trajectory": conv["trajectory"]}
    if scan is not None:
        out["scan"] = scan
    # CPU and refstruct legs: on the benchmarked graph for c2; for c3 (no CSR can exist: 400 GB) on
    # --simulate 0.1 -n 100000, which has C3's mean degree 1e4 (per-vertex work is per-degree)
    sample, sample_n, sample_window, sample_note = g, n, None, None
    cpu_ncol = a.ncol
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.config == "c5":
        # the oracle's fill_p / extract_new_color are O(nCol) per vertex (26K colours here): one sweep
        # of the full graph takes minutes, so the CPU leg runs on the same generator at scale 18
        cs = M.Graph.rmat(18, 10, 0.5, 0.2, 0.2, 1, device=dev)
        s = cs.getStruct()
        cpu_ncol = cs.getMaxNodeDeg()
        out["cpu_baseline"] = cpu_baseline(s.cumulDegs, s.neighs, cpu_ncol, a.seed, M.GlibcRand(1).window, cs.nNodes)
        out["cpu_baseline"]["sample"] += (f"; graph R-MAT scale 18 (same generator and seed, n = {cs.nNodes}, "
                                          f"nCol = maxDeg = {cpu_ncol}; the oracle is O(nCol) per vertex)")
        cs.close()
    if rank == 0 and world == 1 and a.config == "c3" and not a.no_refstruct:
        # refstruct at full occupancy (the C3 CSR itself would be 400 GB): a 2e6-row graph of C3's degree
        g.close()
        out["refstruct"] = refstruct_full_occupancy(dev, a.ncol, a.seed, value, max(2, min(a.refstruct_sweeps, 4)))
    if rank == 0 and world == 1 and not (a.no_refstruct and a.no_cpu_baseline):
        if a.config == "c3":
            g.close()
            r2 = M.GlibcRand(1)
            sample = M.Graph.simulate(100000, 0.1, r2, device=dev)
            sample_n, sample_window = 100000, r2.window.copy()
            sample_note = "--simulate 0.1 -n 100000 (mean degree 1e4 = C3's; C3's CSR cannot exist: 400 GB)"
        else:
            sample_window = M.GlibcRand(1, n_req * (n_req + 1) // 2).window
    if rank == 0 and world == 1 and not a.no_refstruct and a.config != "c3":
        out["refstruct"] = refstruct_baseline(sample, a.ncol, a.refstruct_sweeps, a.seed, sample_n, value)
        if sample_note:
            out["refstruct"]["graph"] = sample_note
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.config != "c5":
        s = sample.getStruct()
        if ref:
            out["cpu_baseline"] = cpu_baseline_ref(s.cumulDegs, s.neighs, a.ncol, a.seed, sample_n)
        else:
            out["cpu_baseline"] = cpu_baseline(s.cumulDegs, s.neighs, a.ncol, a.seed, sample_window, sample_n)
        if sample_note:
            out["cpu_baseline"]["sample"] += "; graph " + sample_note
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
