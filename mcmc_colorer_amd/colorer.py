"""Host-side mirror of the reference's colorer surface, over libmcmc_hip.so.

Reference classes (paths relative to /root/reference/src):
  ColoringMCMCParams        graph_coloring/coloring.h:65-74
  Graph<float,float>        graph/graph.h:84-133  (ctor (n, prob, seed) -> setupRnd2; (Graph*) device copy)
  GraphStruct               graph/graph.h:37-79
  GPURand                   GPUutils/GPURandomizer.h:42-55 (per-vertex RNG handle passed to the colorer)
  ColoringMCMC<float,float> graph_coloring/coloringMCMC.h:44-140 (ctor, run(int), setDirectoryPath)

Semantics are those of ColoringMCMC_CPU (graph_coloring/coloringMCMC_CPU.cpp): the north star
requires --mcmcgpu to be bit-identical to --mcmccpu. Where the reference shares process-global
state (glibc rand(), used by setupRnd2 and by the CDF-overflow fallback), it is an explicit
``GlibcRand`` object here.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

from ._lib import MCMCCtxInfo, MCMCParams, MCMCRunStats, check, lib, u32ptr, u64ptr

F32_EPS = float(np.float32(1e-8))


@dataclass
class ColoringMCMCParams:
    """ColoringMCMCParams (coloring.h:65-74) with main.cu:160-168 defaults."""

    nCol: int = 0
    numColorRatio: float = 1.0
    lambda_: float = 1.0
    epsilon: float = F32_EPS
    ratioFreezed: float = 1e-2
    maxRip: int = 250
    tabooIteration: int = 0
    tailcut: bool = False
    # extension: corrected tail cut after the loop (coloringMCMC_CPU.cpp:272-311 with k++), at
    # most this many passes; 0 = off (the reference's tail cut never returns, see tailcut.hip)
    tailcutRepair: int = 0

    def to_c(self, seed: int) -> MCMCParams:
        return MCMCParams(self.nCol, self.epsilon, self.lambda_, self.ratioFreezed, self.numColorRatio,
                          self.maxRip, self.tabooIteration, int(bool(self.tailcut)), seed & 0xFFFFFFFF)


class GlibcRand:
    """Position in glibc's rand() stream (TYPE_3 window of 31 words).

    The reference uses the process-global stream: unseeded (== srand(1)) when --seed is given
    (ArgHandle.cpp:272-276), advanced n(n+1)/2 draws by setupRnd2 (graphCPU.cpp:308) and one
    draw per CDF overflow (coloringMCMC_CPU.cpp:518)."""

    def __init__(self, seed: int = 1, draws: int = 0):
        self.window = np.zeros(31, dtype=np.uint32)
        check(lib().mcmc_glibc_window(seed & 0xFFFFFFFF, draws, u32ptr(self.window)))

    def rand(self, count: int = 1) -> np.ndarray:
        out = np.zeros(count, dtype=np.uint32)
        check(lib().mcmc_glibc_draw(u32ptr(self.window), count, u32ptr(out)))
        return out


@dataclass
class GraphStruct:
    """GraphStruct (graph.h:37-79): nNodes, nEdges, cumulDegs (uint64 here), neighs."""

    nNodes: int
    nEdges: int
    cumulDegs: np.ndarray
    neighs: np.ndarray

    def deg(self, i: int) -> int:
        return int(self.cumulDegs[i + 1] - self.cumulDegs[i])


class Graph:
    """Device-resident CSR graph (Graph<float,float> after its (Graph*) device copy)."""

    def __init__(self, handle: ctypes.c_void_p, prob: float = 0.0, device: int = 0):
        self._h = handle
        self.prob = float(prob)
        self.device = device
        n = ctypes.c_uint32()
        m = ctypes.c_uint64()
        mx = ctypes.c_uint32()
        mn = ctypes.c_uint32()
        check(lib().mcmc_graph_info(self._h, ctypes.byref(n), ctypes.byref(m), ctypes.byref(mx), ctypes.byref(mn)))
        self.nNodes, self.nEdges, self.maxDeg, self.minDeg = n.value, m.value, mx.value, mn.value
        self._struct: Optional[GraphStruct] = None

    @classmethod
    def simulate(cls, n: int, prob: float, rand: GlibcRand, device: int = 0) -> "Graph":
        """Graph(n, prob, seed) -> setupRnd2 (graphCPU.cpp:291-404), generated on the GPU.
        Advances ``rand`` by n(n+1)/2 draws, as the reference's global stream is."""
        h = ctypes.c_void_p()
        check(lib().mcmc_graph_simulate(n, ctypes.c_float(prob), u32ptr(rand.window), device, ctypes.byref(h)))
        return cls(h, prob=float(np.float32(prob)), device=device)

    @classmethod
    def er_fast(cls, n: int, prob: float, seed: int, device: int = 0, world: int = 1, rank: int = 0,
                rows: Optional[tuple[int, int]] = None) -> "Graph":
        """The build's counter-based G(n, p) (csrc/er_gen.h) for sizes where setupRnd2 is infeasible
        (SURVEY.md §8d C3/C4), generated on the GPU straight into the sweep's tiled layout.
        world > 1: only the rows rank ``rank`` owns under the equal-rows plan (a partitioned run);
        rows=(v_begin, v_end): only those rows. nEdges then counts those rows' arcs."""
        h = ctypes.c_void_p()
        if rows is not None:
            check(lib().mcmc_graph_er_fast_rows(n, float(prob), seed, rows[0], rows[1], device, ctypes.byref(h)))
        elif world == 1:
            check(lib().mcmc_graph_er_fast(n, float(prob), seed, device, ctypes.byref(h)))
        else:
            check(lib().mcmc_graph_er_fast_part(n, float(prob), seed, world, rank, device, ctypes.byref(h)))
        g = cls(h, prob=float(np.float32(prob)), device=device)
        g.generated = True
        return g

    @classmethod
    def rmat(cls, scale: int, edge_factor: int, a: float = 0.5, b: float = 0.2, c: float = 0.2, seed: int = 1,
             device: int = 0) -> "Graph":
        """R-MAT power-law stand-in for configs[4] (csrc/er_gen.h rmat_edge; SURVEY.md §8d C5: the SNAP
        graphs are not available), generated on the GPU as a CSR with ascending neighbour lists."""
        h = ctypes.c_void_p()
        check(lib().mcmc_graph_rmat(scale, edge_factor, a, b, c, seed, device, ctypes.byref(h)))
        n = 1 << scale
        g = cls(h, device=device)
        if n > 0:
            g.prob = g.nEdges / float(np.float32(n) * np.float32(n))
        return g

    @classmethod
    def from_csr(cls, row_off: np.ndarray, col_idx: np.ndarray, device: int = 0, prob: float = 0.0) -> "Graph":
        """Graph(Graph* host) device copy (graphGPU.cu:210-226) of a host CSR."""
        row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
        col_idx = np.ascontiguousarray(col_idx, dtype=np.uint32)
        n = len(row_off) - 1
        h = ctypes.c_void_p()
        check(lib().mcmc_graph_upload(u64ptr(row_off), u32ptr(col_idx) if len(col_idx) else None, n,
                                      len(col_idx), device, ctypes.byref(h)))
        if prob == 0.0 and n > 0:
            prob = len(col_idx) / float(np.float32(n) * np.float32(n))   # graphCPU.cpp:158 (without the overflow)
        return cls(h, prob=prob, device=device)

    def getStruct(self) -> GraphStruct:
        if self._struct is None:
            off = np.zeros(self.nNodes + 1, dtype=np.uint64)
            idx = np.zeros(max(self.nEdges, 1), dtype=np.uint32)
            check(lib().mcmc_graph_download(self._h, u64ptr(off), u32ptr(idx)))
            self._struct = GraphStruct(self.nNodes, self.nEdges, off, idx[: self.nEdges])
        return self._struct

    def rows(self, rows) -> tuple[list[np.ndarray], np.ndarray]:
        """Rows as stored on the device (mcmc_graph_rows: the tiled layout of a generated graph, else
        the CSR), each in layout order, and the layout index of each row's first stored id."""
        r = np.ascontiguousarray(rows, dtype=np.uint32)
        off = np.zeros(len(r) + 1, dtype=np.uint64)
        pos = np.zeros(max(len(r), 1), dtype=np.uint64)
        check(lib().mcmc_graph_rows(self._h, u32ptr(r), len(r), u64ptr(off), None, 0, u64ptr(pos)))
        ids = np.zeros(max(int(off[-1]), 1), dtype=np.uint32)
        check(lib().mcmc_graph_rows(self._h, u32ptr(r), len(r), u64ptr(off), u32ptr(ids), len(ids), None))
        return [ids[off[i]:off[i + 1]] for i in range(len(r))], pos[: len(r)]

    def getMaxNodeDeg(self) -> int:
        return self.maxDeg

    def getMinNodeDeg(self) -> int:
        return self.minDeg

    def getMeanNodeDeg(self) -> float:
        return float(np.float32(self.nEdges) / np.float32(self.nNodes)) if self.nNodes else 0.0

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def close(self) -> None:
        if self._h:
            lib().mcmc_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GPURand:
    """GPURand(n, seed) (GPURandomizer.h:42-55). The reference keeps 48-byte cuRAND states per
    vertex; this build needs none (counter-based minstd skip-ahead), only the seed and the glibc
    stream the CDF-overflow fallback draws from."""

    def __init__(self, n: int, seed: int, glibc: Optional[GlibcRand] = None):
        self.n = n
        self.seed = seed
        self.glibc = glibc if glibc is not None else GlibcRand(1)
        self.randStates = self   # the reference's public member name


def default_ncol(graph: Graph, params: ColoringMCMCParams, nColFromC: int = 0) -> int:
    """main.cu:162: nCol = --nCol, else (uint32)(maxDeg * numColorRatio) in float."""
    if nColFromC:
        return nColFromC
    return int(np.float32(graph.getMaxNodeDeg()) * np.float32(params.numColorRatio))


class ColoringMCMC:
    """ColoringMCMC<float,float> (coloringMCMC.h:44-140) on the MI355X sweep.

    ``run(iteration)`` colours with engine seed ``rand.seed + iteration`` (main.cu:171's seed+i)
    from the glibc stream position held by ``rand.glibc`` (advanced in place), and, when a
    directory path is set, writes ``<dir>.log`` and ``<dir>-colors.txt`` like the reference's
    colorers (coloringMCMC_prints.cu:37-38; report fields of coloringMCMC_CPUutils.cpp:70-109)."""

    def __init__(self, graph_d: Graph, randStates: GPURand, params: ColoringMCMCParams,
                 v_begin: int = 0, v_end: Optional[int] = None):
        if params.nCol == 0:
            params = ColoringMCMCParams(**{**params.__dict__, "nCol": default_ncol(graph_d, params)})
        self.graph = graph_d
        self.rand = randStates
        self.param = params
        self.v_begin = v_begin
        self.v_end = graph_d.nNodes if v_end is None else v_end
        self.directory: Optional[str] = None
        self._ctx = ctypes.c_void_p()
        self._cparams = params.to_c(randStates.seed)
        check(lib().mcmc_create(graph_d.handle, ctypes.byref(self._cparams), self.v_begin, self.v_end,
                                ctypes.byref(self._ctx)))
        self.stats: Optional[MCMCRunStats] = None
        self.duration = 0.0

    def setDirectoryPath(self, directory: str) -> None:
        self.directory = directory

    def init(self, iteration: int = 0, C0: Optional[np.ndarray] = None) -> None:
        self._cparams.seed = (self.rand.seed + iteration) & 0xFFFFFFFF
        lib().mcmc_destroy(self._ctx)
        self._ctx = ctypes.c_void_p()
        check(lib().mcmc_create(self.graph.handle, ctypes.byref(self._cparams), self.v_begin, self.v_end,
                                ctypes.byref(self._ctx)))
        check(lib().mcmc_set_glibc_window(self._ctx, u32ptr(self.rand.glibc.window)))
        if self.param.tailcutRepair:
            check(lib().mcmc_set_tailcut_repair(self._ctx, int(self.param.tailcutRepair)))
        c0 = None if C0 is None else u32ptr(np.ascontiguousarray(C0, dtype=np.uint32))
        check(lib().mcmc_init_coloring(self._ctx, c0))

    def run(self, iteration: int = 0, max_sweeps: int = 0) -> MCMCRunStats:
        self.init(iteration)
        st = MCMCRunStats()
        check(lib().mcmc_run(self._ctx, max_sweeps, ctypes.byref(st)))
        check(lib().mcmc_get_glibc_window(self._ctx, u32ptr(self.rand.glibc.window)))
        self.stats = st
        self.duration = st.loopMs / 1000.0
        if self.directory:
            self.save(iteration)
        return st

    def step(self, sweeps: int) -> MCMCRunStats:
        """Continues the loop of an initialised context by at most `sweeps` sweeps (no re-init)."""
        st = MCMCRunStats()
        check(lib().mcmc_run(self._ctx, sweeps, ctypes.byref(st)))
        return st

    def count_violations(self, flags: bool = False):
        """Cviol of the current colouring, recounted by the tail cut's kernel (mcmc_count_violations);
        flags=True also returns the per-vertex flags."""
        c = ctypes.c_uint64()
        f = np.zeros(self.graph.nNodes, dtype=np.uint8) if flags else None
        check(lib().mcmc_count_violations(self._ctx, ctypes.byref(c), f.ctypes.data_as(ctypes.c_void_p) if flags else None))
        return (c.value, f) if flags else c.value

    # -- results ------------------------------------------------------------------------------
    def coloring(self) -> np.ndarray:
        out = np.zeros(self.graph.nNodes, dtype=np.uint32)
        check(lib().mcmc_get_coloring(self._ctx, u32ptr(out)))
        return out

    def trajectory(self) -> np.ndarray:
        n = ctypes.c_uint64()
        check(lib().mcmc_get_trajectory(self._ctx, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        if n.value:
            check(lib().mcmc_get_trajectory(self._ctx, u64ptr(out), n.value, ctypes.byref(n)))
        return out

    def info(self) -> dict:
        """Sweep kernel / adjacency layout of the current context and its bytes per sweep
        (mcmc_get_info: B_fmt and the reference-layout B_alg of SURVEY.md §8d)."""
        if not self._ctx:
            self.init(0)
        i = MCMCCtxInfo()
        check(lib().mcmc_get_info(self._ctx, ctypes.byref(i)))
        return i.as_dict()

    def wide_inc_stats(self) -> dict:
        """The wide sweep's incremental violation counts since the colouring was initialised
        (mcmc_get_wide_inc_stats): whether the context keeps them, sweeps that moved them by the rows
        that changed, full recounts, changed rows and their arcs."""
        out = (ctypes.c_uint64 * 5)()
        check(lib().mcmc_get_wide_inc_stats(self._ctx, out))
        return {"enabled": bool(out[0]), "incremental_sweeps": int(out[1]), "full_sweeps": int(out[2]),
                "changed_rows": int(out[3]), "changed_arcs": int(out[4])}

    def wide_solo_stats(self) -> dict:
        """The persistent wide sweep (mcmc_get_wide_solo_stats; csrc/wide_solo.h): whether the
        context runs it, its candidate-window states, and cumulative sweeps, phases handed to the
        grid, violators walked by its leader, walk / count-move / collection phases, candidate rows
        evaluated and rows that changed colour."""
        out = (ctypes.c_uint64 * 30)()
        check(lib().mcmc_get_wide_solo_stats(self._ctx, out))
        keys = ("enabled", "window_states", "sweeps", "phases", "leader_walks", "walk_phases", "delta_phases",
                "collects", "candidates", "changed_rows", "watchdog", "dbg_sweep", "dbg_step", "dbg_gen")
        d = {k: int(v) for k, v in zip(keys, out)}
        steps = ("walks", "candidates", "walk_wait", "events", "changes", "count_moves", "violator_list", "sweep")
        d["step_us"] = {k: out[14 + i] / 100.0 for i, k in enumerate(steps)}   # summed over its sweeps
        d["probe_us"] = [out[22 + i] / 100.0 for i in range(8)]   # finer probes (csrc/wide_solo.h)
        return d

    def dense_stats(self) -> dict:
        """The dense-count sweep since the colouring was initialised (mcmc_get_dense_stats; csrc/
        dense_counts.h): whether the context runs it, its dense column range, sweeps whose update moved
        the counts by the changed vertices, count rebuilds, vertices moved, rows that scanned past the
        range, the update list's rebuild threshold, rows that changed colour and restore-list overflows."""
        out = (ctypes.c_uint64 * 16)()
        check(lib().mcmc_get_dense_stats_v2(self._ctx, out))
        return {"enabled": bool(out[0]), "s0": int(out[1]), "s1": int(out[2]), "incremental_sweeps": int(out[3]),
                "rebuilds": int(out[4]), "moved_vertices": int(out[5]), "open_rows": int(out[6]),
                "rebuild_threshold": int(out[7]), "changed_rows": int(out[8]), "copy_sweeps": int(out[9]),
                "solo_sweeps": int(out[10]), "window_states": int(out[11]), "persistent": bool(out[12]),
                "open_words": int(out[13]), "solo_evaluated": int(out[14]), "transposed_ids": bool(out[15])}

    def save(self, iteration: int) -> None:
        d = self.directory
        Path(d).parent.mkdir(parents=True, exist_ok=True)
        C = self.coloring()
        write_report(d + ".log", "GPU (MI355X)", self.graph, self.param, self.rand.seed + iteration, iteration,
                     self.duration, self.stats, C)
        with open(d + "-colors.txt", "w") as f:
            f.write("".join(f"{i} {c}\n" for i, c in enumerate(C.tolist())))

    def close(self) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CurandStates:
    """GPURand's per-vertex curandState array (GPURandomizer.cu:85-101: curand_init(seed, v, 0) for
    every vertex v) for the reference-GPU-semantics mode: cuRAND XORWOW states on the device, shared
    by every repetition (main.cu:80, 193) and advanced as the reference's are."""

    def __init__(self, n: int, seed: int, device: int = 0):
        self.n = n
        self.seed = seed & 0xFFFFFFFF
        self.device = device
        self._h = ctypes.c_void_p()
        check(lib().mcmc_gpurand_create(n, self.seed, device, ctypes.byref(self._h)))

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def states(self) -> np.ndarray:
        """[n][6] = {v0..v4, d} per vertex."""
        out = np.zeros((self.n, 6), dtype=np.uint32)
        check(lib().mcmc_gpurand_states(self._h, u32ptr(out)))
        return out

    def close(self) -> None:
        if self._h:
            lib().mcmc_gpurand_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ColoringMCMCGpuRef:
    """The reference's own --mcmcgpu colorer, semantics included: ColoringMCMC
    as built by default (coloringMCMC.h:22-41 -- balance-dynamic proposal, cuRAND XORWOW per vertex,
    conflicts counted as edges, the GPU tail cut), run on the MI355X tiled sweep. ``run()`` returns
    MCMCRunStats with iter = rip, finalViol = conflicting edges of the returned colouring; the
    trajectory holds the conflicting-edge count of every colouring the loop counted. Parity is
    unpinned against CUDA (none here): pinned pieces and the oracle are listed in DESIGN.md."""

    def __init__(self, graph_d: Graph, states: CurandStates, params: ColoringMCMCParams):
        if params.nCol == 0:
            params = ColoringMCMCParams(**{**params.__dict__, "nCol": default_ncol(graph_d, params)})
        self.graph = graph_d
        self.rand = states
        self.param = params
        self._cparams = params.to_c(states.seed)
        self._ctx = ctypes.c_void_p()
        check(lib().mcmc_ref_create(graph_d.handle, ctypes.byref(self._cparams), states.handle,
                                    ctypes.byref(self._ctx)))
        self.stats: Optional[MCMCRunStats] = None

    def init(self) -> None:
        """The run's initialisation alone (throughput benchmarks time mcmc_bench_sweeps after it)."""
        check(lib().mcmc_ref_init(self._ctx))

    def run(self, tail_max_passes: int = 1000) -> MCMCRunStats:
        st = MCMCRunStats()
        check(lib().mcmc_ref_run(self._ctx, tail_max_passes, ctypes.byref(st)))
        self.stats = st
        return st

    def coloring(self) -> np.ndarray:
        out = np.zeros(self.graph.nNodes, dtype=np.uint32)
        check(lib().mcmc_get_coloring(self._ctx, u32ptr(out)))
        return out

    def trajectory(self) -> np.ndarray:
        n = ctypes.c_uint64()
        check(lib().mcmc_get_trajectory(self._ctx, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        if n.value:
            check(lib().mcmc_get_trajectory(self._ctx, u64ptr(out), n.value, ctypes.byref(n)))
        return out

    def tail_trajectory(self) -> np.ndarray:
        n = ctypes.c_uint64()
        check(lib().mcmc_get_tail_trajectory(self._ctx, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint64)
        if n.value:
            check(lib().mcmc_get_tail_trajectory(self._ctx, u64ptr(out), n.value, ctypes.byref(n)))
        return out

    def info(self) -> dict:
        i = MCMCCtxInfo()
        check(lib().mcmc_get_info(self._ctx, ctypes.byref(i)))
        return i.as_dict()

    def close(self) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_report(path: str, flavour: str, graph: Graph, p: ColoringMCMCParams, seed: int, rep: int,
                 duration: float, st: MCMCRunStats, C: np.ndarray) -> None:
    """The .log block of saveStats (coloringMCMC_CPUutils.cpp:70-102), parseable by the
    reference's pyScripts/logParser.py lineParser."""
    nCol = p.nCol
    hist = np.bincount(C, minlength=nCol).astype(np.int64)
    used = int((hist > 0).sum())
    mean = np.float32(hist.sum()) / np.float32(nCol)
    var = np.float32(0)
    for h in hist:
        var = np.float32(var + np.float32((np.float32(h) - mean) * (np.float32(h) - mean)))
    var = np.float32(var / np.float32(nCol))
    lines = [
        f"MCMC Colorer - {flavour} version - Report",
        "-------------------------------------------",
        "GRAPH INFO",
        f"Nodes: {graph.nNodes} - Edges: {graph.nEdges}",
        f"Max deg: {graph.getMaxNodeDeg()} - Min deg: {graph.getMinNodeDeg()} - Avg deg: {graph.getMeanNodeDeg():g}",
        f"Edge probability (for randomly generated graphs): {graph.prob:g}",
        f"Seed: {seed}",
        "-------------------------------------------",
        "EXECUTION INFO",
        f"Repetition: {rep}",
        f"Execution time: {duration:g}",
        f"Iteration performed: {st.iter}",
        f"Max iteration reached: {'yes' if st.maxIterReached else 'no'}",
        "-------------------------------------------",
        "Color histogram:",
        *[f"{i}: {int(h)}" for i, h in enumerate(hist)],
        f"Number of colors: {nCol} - Used colors: {used}",
        f"Color ratio: {p.numColorRatio:g}",
        f"Average number of nodes for each color: {float(mean):g}",
        f"Variance: {float(var):g}",
        f"StD: {float(np.sqrt(var)):g}",
    ]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


class ColoringGreedyFF:
    """ColoringGreedyFF (graph_coloring/coloringGreedyFF.h/.cu, ``--grdffgpu``):
    the reference's deterministic parallel greedy first-fit colorer on the GPU (csrc/greedyff.hip).
    Colours are 1-based; ``numColors`` counts the distinct colours (coloringGreedyFF.cu:79-80)."""

    def __init__(self, graph: "Graph"):
        self.graph = graph
        self.colors = None
        self.numColors = 0
        self.rounds = 0

    def run(self) -> None:
        out = np.zeros(self.graph.nNodes, dtype=np.uint32)
        nc, r = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mcmc_greedyff_run(self.graph.handle, u32ptr(out), ctypes.byref(nc), ctypes.byref(r)))
        self.colors, self.numColors, self.rounds = out, nc.value, r.value

    def getColoring(self) -> tuple[int, np.ndarray]:
        return self.numColors, self.colors

    def saveColor(self, path: str) -> None:
        """saveColor (coloringGreedyFF.cu:305-310): one "<node> <colour>" line per node."""
        with open(path, "w") as f:
            f.writelines(f"{i} {int(c)}\n" for i, c in enumerate(self.colors))


class ColoringVFF:
    """ColoringVFF (graph_coloring/coloringVFF.h/.cu, ``--vffgpu``): the
    greedy first-fit colouring, then the reference's vertex-first-fit rebalancing, on the GPU
    (csrc/greedyff.hip). ``valid`` is the reference's not_looping: False when the rebalancing was
    found looping, and the colouring is then the greedy one."""

    def __init__(self, graph: "Graph"):
        self.graph = graph
        self.colors = None
        self.numColors = 0
        self.iterations = 0
        self.valid = True

    def run(self) -> None:
        out = np.zeros(self.graph.nNodes, dtype=np.uint32)
        nc, it, v = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
        check(lib().mcmc_vff_run(self.graph.handle, u32ptr(out), ctypes.byref(nc), ctypes.byref(it), ctypes.byref(v)))
        self.colors, self.numColors, self.iterations, self.valid = out, nc.value, it.value, bool(v.value)

    def getColoring(self) -> tuple[int, np.ndarray]:
        return self.numColors, self.colors

    def saveColor(self, path: str) -> None:
        """saveColor (coloringVFF.cu:484-490): one "<node> <colour>" line per node."""
        with open(path, "w") as f:
            f.writelines(f"{i} {int(c)}\n" for i, c in enumerate(self.colors))


class ColoringLuby:
    """ColoringLuby (graph_coloring/coloringLuby.h:17-68, ``run_fast`` coloringLubyFast.cu:21-174,
    ``--lubygpu``): Luby independent sets, one colour per outer round, on the
    GPU (csrc/luby.hip). ``randStates``: the per-vertex XORWOW states (CurandStates), advanced in
    place by every inner round's draw, as the reference's GPURand states are. Colours are 1..k."""

    def __init__(self, graph: "Graph", randStates: "CurandStates"):
        self.graph = graph
        self.randStates = randStates
        self.colors = None
        self.numOfColors = 0
        self.rounds = 0

    def run_fast(self) -> None:
        out = np.zeros(self.graph.nNodes, dtype=np.uint32)
        nc, r = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mcmc_luby_run(self.graph.handle, self.randStates.handle, u32ptr(out), ctypes.byref(nc),
                                  ctypes.byref(r)))
        self.colors, self.numOfColors, self.rounds = out, nc.value, r.value

    run = run_fast

    def getColoringGPU(self) -> tuple[int, np.ndarray]:
        return self.numOfColors, self.colors

    def saveColor(self, path: str) -> None:
        """saveColor (coloringLuby.cu:209-215): one "<node> <colour>" line per node."""
        with open(path, "w") as f:
            f.writelines(f"{i} {int(c)}\n" for i, c in enumerate(self.colors))
