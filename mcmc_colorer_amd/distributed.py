"""Vertex-partitioned multi-GPU MCMC colouring: one rank per GPU.

The sweep of vertex v depends only on the colours of N(v), on u_v (a function of the global id and
the sweep number) and on taboo[v], so rows shard exactly. Rank r owns rows [bounds[r], bounds[r+1])
of a partition plan (mcmc_part_plan: equal rows, or arc-balanced from the degree prefix for
power-law graphs), keeps global ids, a full colour replica in vertex order and a replicated glibc
window. Per sweep t:

  1. local sweep (HIP kernel): next colours of the owned rows + the rank's footer slot (local Cviol,
     event count, flags, sorted overflow events),
  2. exchange: every rank's row range and footer slot to every rank,
  3. commit (HIP kernel) on every rank: global Cviol, stop test, the rank-ordered (= ascending)
     glibc replay with the replicated glibc window -- replicas stay identical.

A rank whose overflow events outgrow its footer pauses the loop at that sweep on every rank; the
full sorted lists are then all-gathered and the paused sweep is committed from them (the spill
exchange). Results are bit-identical to the single-GPU run and to --mcmccpu.

Two drivers run that sequence:

  * ``NativePartitionedColoringMCMC`` -- the product path: the RCCL communicator lives inside
    libmcmc_hip.so (mcmc_comm_init_rank) and ``mcmc_part_run`` runs the whole loop natively
    (csrc/multi.hip: P2P sends of the row ranges over xGMI, one all-gather of the footers). Python
    only hands rank 0's ncclUniqueId to the others over torch.distributed.
  * ``PartitionedColoringMCMC`` -- the same exchange issued from Python over torch.distributed
    (a broadcast of every rank's row range, an all-gather of the footers), with a pluggable rank
    backend: ``HipRank`` here, or the numpy mirror of tests/partition_ref.py, which is how the
    protocol runs over gloo on CPU.

torch and libmcmc_hip.so each bring a HIP runtime: initialise torch's device (``torch.cuda`` calls,
as ``torch.distributed.run`` launches do) before the library is first loaded.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from ._lib import MCMCCtxInfo, MCMCRunStats, check, lib, u32ptr, u64ptr
from .colorer import ColoringMCMCParams, GlibcRand, GPURand, Graph, default_ncol

FOOTER_WORDS = 1024   # MCMC_FOOTER_WORDS
FOOTER_EVENTS = FOOTER_WORDS - 4
DELTA_WORDS = 4096    # MCMC_DELTA_WORDS: a rank's delta slot ([0] pairs appended, [1] 0, (v, colour) pairs)
DELTA_PAIRS = (DELTA_WORDS - 2) // 2
FULL_AFTER_OVERFLOW = 16   # full-mode steps after a delta slot overflowed (csrc/multi.hip kFullAfterOverflow)
COMM_ID_BYTES = 128   # MCMC_COMM_ID_BYTES


def plan_rows(n: int, world: int) -> np.ndarray:
    """Equal row ranges (mcmc_part_plan_rows): bounds[world + 1]."""
    b = np.zeros(world + 1, dtype=np.uint32)
    check(lib().mcmc_part_plan_rows(n, world, u32ptr(b)))
    return b


def plan_csr(row_off: np.ndarray, world: int) -> np.ndarray:
    """Arc-balanced ranges from a host CSR's offsets (mcmc_part_plan_csr)."""
    ro = np.ascontiguousarray(row_off, dtype=np.uint64)
    b = np.zeros(world + 1, dtype=np.uint32)
    check(lib().mcmc_part_plan_csr(u64ptr(ro), len(ro) - 1, world, u32ptr(b)))
    return b


def plan(graph: Graph, world: int, balance: bool = True) -> np.ndarray:
    """mcmc_part_plan: arc-balanced from the device CSR (balance and a CSR), else equal rows."""
    b = np.zeros(world + 1, dtype=np.uint32)
    check(lib().mcmc_part_plan(graph.handle, world, 1 if balance else 0, u32ptr(b)))
    return b


def group_default_ncol(graph, params: ColoringMCMCParams, group=None) -> int:
    """main.cu:162's default nCol (maxDeg * numColorRatio) over a partitioned group: a rank may hold
    only its own rows (Graph.er_fast(rows=...)), so the max degree is all-reduced (MAX) first and
    every rank samples the same colour range as the one-GPU run."""
    import torch
    import torch.distributed as dist

    mx = torch.tensor([int(graph.getMaxNodeDeg())], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        mx = mx.cuda()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)

    class _Whole:   # default_ncol reads only the max degree
        maxDeg = int(mx.item())

        def getMaxNodeDeg(self):
            return self.maxDeg

    return default_ncol(_Whole(), params)


class HipRank:
    """This rank's share of the sweep on its GPU, over the caller-exchanged C ABI (mcmc_part_*),
    with torch tensors as the exchange buffers."""

    def __init__(self, graph: Graph, params: ColoringMCMCParams, seed: int, world: int, rank: int, device,
                 bounds: Optional[np.ndarray] = None):
        import torch

        self.torch = torch
        self.world, self.rank = world, rank
        self.n = graph.nNodes
        self.bounds = plan_rows(self.n, world) if bounds is None else np.asarray(bounds, dtype=np.uint32)
        self.v_begin, self.v_end = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.graph = graph
        self.params = params
        self.cb = int(lib().mcmc_color_bytes(params.nCol))   # 2: the wide sweep's uint16 replicas
        size = (self.n + 256) * self.cb
        self.colors = [torch.zeros(size, dtype=torch.uint8, device=device) for _ in range(2)]
        self.foot = [torch.zeros(world * FOOTER_WORDS, dtype=torch.int32, device=device) for _ in range(2)]
        self.dlt = [torch.zeros(world * DELTA_WORDS, dtype=torch.int32, device=device) for _ in range(2)]
        self._ctx = ctypes.c_void_p()
        self._size = size
        self._make(seed)

    def _make(self, seed: int) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()
        self._cparams = self.params.to_c(seed)
        check(lib().mcmc_create(self.graph.handle, ctypes.byref(self._cparams), self.v_begin, self.v_end,
                                ctypes.byref(self._ctx)))
        stream = self.torch.cuda.current_stream().cuda_stream
        check(lib().mcmc_part_attach(self._ctx, self.world, self.rank, u32ptr(self.bounds), self.colors[0].data_ptr(),
                                     self.colors[1].data_ptr(), self._size, self.foot[0].data_ptr(),
                                     self.foot[1].data_ptr(), ctypes.c_void_p(stream)))
        check(lib().mcmc_part_attach_delta(self._ctx, ctypes.c_void_p(self.dlt[0].data_ptr()),
                                           ctypes.c_void_p(self.dlt[1].data_ptr())))

    def init(self, seed: int, glibc: GlibcRand) -> None:
        self._make(seed)
        check(lib().mcmc_set_glibc_window(self._ctx, u32ptr(glibc.window)))
        check(lib().mcmc_init_coloring(self._ctx, None))

    def delta_ok(self) -> bool:
        return bool(lib().mcmc_part_delta_ok(self._ctx))

    def sweep(self, delta: bool = False) -> None:
        check(lib().mcmc_part_sweep_mode_async(self._ctx, 1 if delta else 0))

    def commit(self, mode: int = 0, spill=None, stride: int = 0) -> None:
        """mode 1 delta, 0 full, -1 full-mode resumption of a paused sweep; spill: the gathered lists."""
        check(lib().mcmc_part_commit_mode_async(self._ctx, mode, ctypes.c_void_p(spill.data_ptr()) if spill is not None
                                                else None, stride))

    def sync_remote(self) -> None:
        check(lib().mcmc_part_sync_remote_async(self._ctx))

    def state(self) -> tuple[bool, int, int]:
        done, t, err = ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mcmc_part_state(self._ctx, ctypes.byref(done), ctypes.byref(t), ctypes.byref(err)))
        return bool(done.value), t.value, err.value

    def exchange_buffers(self, t: int):
        """(next-colour buffer, [(byte range of rank r's rows)], next footer buffer, next delta-slot
        buffer) of sweep t."""
        nb = (t + 1) & 1
        rngs = [(int(self.bounds[r]) * self.cb, int(self.bounds[r + 1]) * self.cb) for r in range(self.world)]
        return self.colors[nb], rngs, self.foot[nb], self.dlt[nb]

    def spill_counts(self) -> np.ndarray:
        c = np.zeros(self.world, dtype=np.uint32)
        check(lib().mcmc_part_spill_counts(self._ctx, u32ptr(c)))
        return c

    def spill_local(self, stride: int):
        """This rank's sorted event list of the paused sweep, padded to `stride` words."""
        out = self.torch.zeros(max(stride, 1), dtype=self.torch.int32, device=self.colors[0].device)
        cnt = ctypes.c_uint32()
        check(lib().mcmc_part_spill_local(self._ctx, ctypes.c_void_p(out.data_ptr()), ctypes.byref(cnt)))
        return out

    def spill_commit(self, gathered, stride: int) -> None:
        check(lib().mcmc_part_spill_commit_async(self._ctx, ctypes.c_void_p(gathered.data_ptr()), stride))

    def glibc_window(self, glibc: GlibcRand) -> None:
        check(lib().mcmc_get_glibc_window(self._ctx, u32ptr(glibc.window)))

    def coloring(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.uint32)
        check(lib().mcmc_get_coloring(self._ctx, u32ptr(out)))
        return out

    def trajectory(self) -> np.ndarray:
        self.state()   # refreshes the context's run summary (trajectory length) from the device
        k = ctypes.c_uint64()
        check(lib().mcmc_get_trajectory(self._ctx, None, 0, ctypes.byref(k)))
        out = np.zeros(k.value, dtype=np.uint64)
        if k.value:
            check(lib().mcmc_get_trajectory(self._ctx, u64ptr(out), k.value, ctypes.byref(k)))
        return out

    def info(self) -> dict:
        i = MCMCCtxInfo()
        check(lib().mcmc_get_info(self._ctx, ctypes.byref(i)))
        return i.as_dict()

    def close(self) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = None


class PartitionedColoringMCMC:
    """ColoringMCMC (graph_coloring/coloringMCMC.h:44-140) over a vertex-partitioned process group,
    the exchange issued from Python over torch.distributed.

    ``run(iteration)`` is bit-identical to ``ColoringMCMC.run(iteration)`` on one GPU."""

    def __init__(self, graph: Graph, randStates: GPURand, params: ColoringMCMCParams, group=None,
                 backend=None, check_every: int = 8, bounds: Optional[np.ndarray] = None, exchange: str = "delta"):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if params.nCol == 0:
            params = ColoringMCMCParams(**{**params.__dict__, "nCol": group_default_ncol(graph, params, group)})
        self.param = params
        self.rand = randStates
        self.check_every = max(1, check_every)
        if backend is None:
            backend = HipRank(graph, params, randStates.seed, self.world, self.rank,
                              torch.device("cuda", torch.cuda.current_device()), bounds=bounds)
        self.b = backend
        self.sweeps = 0
        self.spills = 0
        self.overflows = 0
        self.nccl = dist.get_backend(group) == "nccl"
        # exchange: "delta" (changed vertices only, as mcmc_part_run; ranks agree: the mode depends only
        # on the sweep kind every rank shares) or "full" (every rank's rows every step)
        self.delta = exchange == "delta" and self.world > 1 and backend_delta_ok(self.b)

    def _bcast(self, seg, src: int) -> None:
        if seg.numel() == 0:
            return
        if self.nccl or not seg.is_cuda:
            self.dist.broadcast(seg, src=self.dist.get_global_rank(self.group, src) if self.group else src,
                                group=self.group)
        else:   # gloo rehearsal of device ranks: through host memory
            h = seg.cpu()
            self.dist.broadcast(h, src=src, group=self.group)
            seg.copy_(h)

    def _allgather(self, out, mine) -> None:
        if self.nccl:
            self.dist.all_gather_into_tensor(out, mine, group=self.group)   # in place
        elif out.is_cuda:
            h = self.torch.empty(out.numel(), dtype=out.dtype)
            self.dist.all_gather_into_tensor(h, mine.cpu(), group=self.group)
            out.copy_(h)
        else:
            self.dist.all_gather_into_tensor(out, mine.clone(), group=self.group)

    def _exchange(self, t: int, delta: bool = False) -> None:
        C, rngs, F, D = self.b.exchange_buffers(t)
        if delta:   # every rank's delta slot to every rank
            self._allgather(D, D[self.rank * DELTA_WORDS:(self.rank + 1) * DELTA_WORDS])
        else:
            for r, (lo, hi) in enumerate(rngs):   # every rank's rows to every rank
                self._bcast(C[lo:hi], r)
        self._allgather(F, F[self.rank * FOOTER_WORDS:(self.rank + 1) * FOOTER_WORDS])

    def _step(self, t: int, delta: bool) -> None:
        if delta and not self._synced:   # replicas equal off the local rows before a delta step
            self.b.sync_remote()
        self._synced = delta
        self.b.sweep(delta)
        self._exchange(t, delta)
        self.b.commit(1 if delta else 0)

    def _resume(self, tdev: int, err: int, delta_step: bool) -> None:
        """A sweep paused at tdev: the full lists (err bit 1, the spill exchange) and/or its rows in full
        (err bit 2, a delta slot overflowed), then its commit."""
        gathered, stride = None, 0
        if err & 2:
            stride = int(max(1, self.b.spill_counts().max()))
            mine = self.b.spill_local(stride)
            gathered = self.torch.zeros(self.world * stride, dtype=mine.dtype, device=mine.device)
            self._allgather(gathered, mine)
            self.spills += 1
        full = bool(err & 4)
        if full:
            self._exchange(tdev, False)
            self.overflows += 1
        self.b.commit(-1 if full else (1 if delta_step else 0), gathered, stride)
        self._synced = delta_step and not full

    def run(self, iteration: int = 0, max_sweeps: int = 0):
        """max_sweeps > 0: stop after that many sweeps (bounded samples), as ColoringMCMC.run."""
        b = self.b
        b.init(self.rand.seed + iteration, self.rand.glibc)
        limit = max_sweeps if max_sweeps else self.param.maxRip + 2
        t = 0
        done = False
        self._synced = False
        full_left = 0
        modes = []
        while t < limit and not done:
            k = min(self.check_every, limit - t)
            for _ in range(k):
                d = self.delta and full_left == 0
                full_left = max(0, full_left - 1)
                modes.append(d)
                self._step(t, d)
                t += 1
            done, tdev, err = b.state()
            if err & 1:
                raise RuntimeError("partitioned sweep: device error flag")
            if err & 6:   # paused at sweep tdev (later steps were no-ops): exchange, resume from it
                self._resume(tdev, err, modes[tdev] if tdev < len(modes) else False)
                if err & 4:
                    full_left = FULL_AFTER_OVERFLOW
                done, tdev, err = b.state()
                t = tdev
                del modes[t:]
        _, tdev, _ = b.state()
        self.sweeps = tdev + 1 if done else tdev   # sweeps the device ran (incl. the final count pass)
        b.glibc_window(self.rand.glibc)
        return done

    def coloring(self) -> np.ndarray:
        return self.b.coloring()

    def trajectory(self) -> np.ndarray:
        return self.b.trajectory()


def backend_delta_ok(backend) -> bool:
    """Whether a rank backend runs delta-mode steps (HipRank: the tiled sweep; NumpyRank: always)."""
    f = getattr(backend, "delta_ok", None)
    return bool(f()) if f is not None else False


class NativePartitionedColoringMCMC:
    """ColoringMCMC over a vertex-partitioned process group, the loop run natively
    (mcmc_part_run over an RCCL communicator owned by libmcmc_hip.so). torch.distributed only
    carries rank 0's ncclUniqueId to the other ranks (any backend)."""

    def __init__(self, graph: Graph, randStates: GPURand, params: ColoringMCMCParams, bounds: np.ndarray,
                 group=None, device: int = 0):
        import torch.distributed as dist

        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if params.nCol == 0:
            params = ColoringMCMCParams(**{**params.__dict__, "nCol": group_default_ncol(graph, params, group)})
        self.param = params
        self.rand = randStates
        self.graph = graph
        self.bounds = np.ascontiguousarray(bounds, dtype=np.uint32)
        self.n = graph.nNodes
        uid = (ctypes.c_uint8 * COMM_ID_BYTES)()
        if self.rank == 0:
            check(lib().mcmc_comm_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=group)
        uid = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(obj[0])
        self._comm = ctypes.c_void_p()
        check(lib().mcmc_comm_init_rank(uid, self.world, self.rank, device, ctypes.byref(self._comm)))
        self._ctx = ctypes.c_void_p()
        self._cparams = params.to_c(randStates.seed)
        self._make(randStates.seed)
        self.stats: Optional[MCMCRunStats] = None

    def _make(self, seed: int) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()
        self._cparams.seed = seed & 0xFFFFFFFF
        check(lib().mcmc_part_create(self.graph.handle, ctypes.byref(self._cparams), self.world, self.rank,
                                     u32ptr(self.bounds), self._comm, ctypes.byref(self._ctx)))
        if self.param.tailcutRepair:
            check(lib().mcmc_set_tailcut_repair(self._ctx, int(self.param.tailcutRepair)))

    def init(self, iteration: int = 0) -> None:
        self._make(self.rand.seed + iteration)
        check(lib().mcmc_set_glibc_window(self._ctx, u32ptr(self.rand.glibc.window)))
        check(lib().mcmc_init_coloring(self._ctx, None))

    def run(self, iteration: int = 0, max_sweeps: int = 0) -> MCMCRunStats:
        self.init(iteration)
        st = MCMCRunStats()
        arr = (ctypes.c_void_p * 1)(self._ctx)
        check(lib().mcmc_part_run(arr, 1, max_sweeps, ctypes.byref(st)))
        check(lib().mcmc_get_glibc_window(self._ctx, u32ptr(self.rand.glibc.window)))
        self.stats = st
        return st

    def coloring(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.uint32)
        check(lib().mcmc_get_coloring(self._ctx, u32ptr(out)))
        return out

    def trajectory(self) -> np.ndarray:
        k = ctypes.c_uint64()
        check(lib().mcmc_get_trajectory(self._ctx, None, 0, ctypes.byref(k)))
        out = np.zeros(k.value, dtype=np.uint64)
        if k.value:
            check(lib().mcmc_get_trajectory(self._ctx, u64ptr(out), k.value, ctypes.byref(k)))
        return out

    def info(self) -> dict:
        i = MCMCCtxInfo()
        check(lib().mcmc_get_info(self._ctx, ctypes.byref(i)))
        return i.as_dict()

    def close(self) -> None:
        if self._ctx:
            lib().mcmc_destroy(self._ctx)
            self._ctx = None
        if self._comm:
            lib().mcmc_comm_destroy(self._comm)
            self._comm = None


class LoopbackPartition:
    """All `world` ranks of a partitioned run in this process (several may share a GPU), the native
    driver with its loopback transport (mcmc_part_create with no communicator + mcmc_part_run): the
    exact sequence of the RCCL path with device copies for the exchange. Tests; rehearsals."""

    def __init__(self, graphs, params: ColoringMCMCParams, seed: int, bounds: np.ndarray):
        self.world = len(bounds) - 1
        self.bounds = np.ascontiguousarray(bounds, dtype=np.uint32)
        self.graphs = graphs if isinstance(graphs, (list, tuple)) else [graphs] * self.world
        self.param = params
        self.n = self.graphs[0].nNodes
        self._cparams = params.to_c(seed)
        self._ctx = [ctypes.c_void_p() for _ in range(self.world)]
        for r in range(self.world):
            check(lib().mcmc_part_create(self.graphs[r].handle, ctypes.byref(self._cparams), self.world, r,
                                         u32ptr(self.bounds), None, ctypes.byref(self._ctx[r])))
            if params.tailcutRepair:   # the corrected tail cut after the loop, rank by rank (multi.hip)
                check(lib().mcmc_set_tailcut_repair(self._ctx[r], int(params.tailcutRepair)))

    def run(self, glibc: GlibcRand, max_sweeps: int = 0) -> list:
        for c in self._ctx:
            check(lib().mcmc_set_glibc_window(c, u32ptr(glibc.window)))
            check(lib().mcmc_init_coloring(c, None))
        stats = (MCMCRunStats * self.world)()
        arr = (ctypes.c_void_p * self.world)(*[c.value for c in self._ctx])
        check(lib().mcmc_part_run(arr, self.world, max_sweeps, stats))
        check(lib().mcmc_get_glibc_window(self._ctx[0], u32ptr(glibc.window)))
        return list(stats)

    def coloring(self, r: int = 0) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.uint32)
        check(lib().mcmc_get_coloring(self._ctx[r], u32ptr(out)))
        return out

    def trajectory(self, r: int = 0) -> np.ndarray:
        k = ctypes.c_uint64()
        check(lib().mcmc_get_trajectory(self._ctx[r], None, 0, ctypes.byref(k)))
        out = np.zeros(k.value, dtype=np.uint64)
        if k.value:
            check(lib().mcmc_get_trajectory(self._ctx[r], u64ptr(out), k.value, ctypes.byref(k)))
        return out

    def info(self, r: int = 0) -> dict:
        i = MCMCCtxInfo()
        check(lib().mcmc_get_info(self._ctx[r], ctypes.byref(i)))
        return i.as_dict()

    def close(self) -> None:
        for c in self._ctx:
            if c:
                lib().mcmc_destroy(c)
        self._ctx = []
