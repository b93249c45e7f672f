"""Vertex-partitioned multi-GPU MCMC colouring: one process per GPU, RCCL over xGMI.

SURVEY.md §8e. The sweep of vertex v depends only on the colours of N(v), on u_v (a function of the
global id and the sweep number) and on taboo[v], so rows shard exactly. Rank r of R owns rows
[r*S, min(n,(r+1)*S)), S = ceil(n/R) rounded up to 16, keeps global ids and a full colour replica.
A colour buffer is R regions of P = b*S + 4096 bytes (b = 1 colour byte, 2 for the wide sweep's
nCol > 256): region r holds the colours of rank r's rows followed by rank r's footer (local Cviol + sorted overflow events). Per sweep:

  1. local sweep (HIP kernel): next colours of the owned rows + the footer, into the rank's own
     region of the next-colour buffer,
  2. ONE in-place ``all_gather_into_tensor`` of the regions (colours and footers together),
  3. commit (HIP kernel) on every rank: global Cviol, stop test, the rank-ordered (= ascending)
     glibc replay with the replicated glibc window -- replicas stay identical.

Everything is enqueued on torch's current stream (the RCCL collective synchronises with it), and
the host only reads the device ``done`` flag every ``check_every`` sweeps. The result is
bit-identical to the single-GPU run and to --mcmccpu (tests/test_gpu_parity.py,
tests/test_distributed.py).

The exchange sequence lives in ``PartitionedColoringMCMC``; the per-rank work sits behind a small
backend interface (``HipRank`` here), which is what lets tests drive the same code over gloo.

torch and libmcmc_hip.so each bring a HIP runtime: initialise torch's device (``torch.cuda`` calls,
as ``torch.distributed.run`` launches do) before the library is first loaded, or one of the two
finds no GPU.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from ._lib import MCMCCtxInfo, check, lib, u32ptr, u64ptr
from .colorer import ColoringMCMCParams, GlibcRand, GPURand, Graph, default_ncol

FOOTER_WORDS = 1024   # MCMC_FOOTER_WORDS


def partition(n: int, world: int, rank: int) -> tuple[int, int, int]:
    """(S, v_begin, v_end) of rank ``rank``: S = ceil(n/world) rounded up to 16 (mcmc_part_layout),
    rows [rank*S, min(n,(rank+1)*S))."""
    S = ((n + world - 1) // world + 15) // 16 * 16
    return S, min(rank * S, n), min((rank + 1) * S, n)


def region_bytes(n: int, world: int, color_bytes: int = 1) -> int:
    """P: bytes of one rank's region of a partitioned colour buffer (slab of colours + footer);
    color_bytes = mcmc_color_bytes(nCol): 2 for the wide sweep (nCol > 256)."""
    return color_bytes * partition(n, world, 0)[0] + 4 * FOOTER_WORDS


class HipRank:
    """This rank's share of the sweep on its GPU, over the C ABI (mcmc_part_*)."""

    def __init__(self, graph: Graph, params: ColoringMCMCParams, seed: int, world: int, rank: int, device):
        import torch

        self.torch = torch
        self.world, self.rank = world, rank
        self.n = graph.nNodes
        self.S, self.v_begin, self.v_end = partition(self.n, world, rank)
        self.graph = graph
        self.params = params
        S, P = ctypes.c_uint64(), ctypes.c_uint64()
        self.color_bytes = int(lib().mcmc_color_bytes(params.nCol))   # 2: the wide sweep's uint16 replicas
        check(lib().mcmc_part_layout2(self.n, world, self.color_bytes, ctypes.byref(S), ctypes.byref(P)))
        assert S.value == self.S
        self.P = P.value
        size = world * self.P + 256
        self.colors = [torch.zeros(size, dtype=torch.uint8, device=device) for _ in range(2)]
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
        check(lib().mcmc_part_attach(self._ctx, self.world, self.rank, self.colors[0].data_ptr(),
                                     self.colors[1].data_ptr(), self._size, ctypes.c_void_p(stream)))

    def init(self, seed: int, glibc: GlibcRand) -> None:
        self._make(seed)
        check(lib().mcmc_set_glibc_window(self._ctx, u32ptr(glibc.window)))
        check(lib().mcmc_init_coloring(self._ctx, None))

    def sweep(self) -> None:
        check(lib().mcmc_part_sweep_async(self._ctx))

    def commit(self) -> None:
        check(lib().mcmc_part_commit_async(self._ctx))

    def state(self) -> tuple[bool, int, int]:
        done, t, err = ctypes.c_int32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mcmc_part_state(self._ctx, ctypes.byref(done), ctypes.byref(t), ctypes.byref(err)))
        return bool(done.value), t.value, err.value

    def region(self, t: int):
        """(all regions of sweep t's next-colour buffer, this rank's region of it)."""
        nxt = self.colors[(t + 1) & 1]
        return nxt[: self.world * self.P], nxt[self.rank * self.P:(self.rank + 1) * self.P]

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
    """ColoringMCMC (graph_coloring/coloringMCMC.h:44-140) over a vertex-partitioned process group.

    ``run(iteration)`` is bit-identical to ``ColoringMCMC.run(iteration)`` on one GPU."""

    def __init__(self, graph: Graph, randStates: GPURand, params: ColoringMCMCParams, group=None,
                 backend=None, check_every: int = 8):
        import torch.distributed as dist

        import torch

        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if params.nCol == 0:
            params = ColoringMCMCParams(**{**params.__dict__, "nCol": default_ncol(graph, params)})
        self.param = params
        self.rand = randStates
        self.check_every = max(1, check_every)
        if backend is None:
            import torch

            backend = HipRank(graph, params, randStates.seed, self.world, self.rank,
                              torch.device("cuda", torch.cuda.current_device()))
        self.b = backend
        self.sweeps = 0
        # RCCL gathers in place (send = this rank's slot of the receive buffer); other backends
        # get a copy of the region
        self.inplace = dist.get_backend(group) == "nccl"

    def _step(self, t: int) -> None:
        b = self.b
        b.sweep()
        regions, mine = b.region(t)
        if self.inplace:
            self.dist.all_gather_into_tensor(regions, mine, group=self.group)   # one collective per sweep
        elif regions.is_cuda:   # gloo rehearsal of device ranks: through host memory
            out = self.torch.empty(regions.numel(), dtype=regions.dtype)
            self.dist.all_gather_into_tensor(out, mine.cpu(), group=self.group)
            regions.copy_(out)
        else:
            self.dist.all_gather_into_tensor(regions, mine.clone(), group=self.group)
        b.commit()

    def run(self, iteration: int = 0, max_sweeps: int = 0):
        """max_sweeps > 0: stop after that many sweeps (bounded samples), as ColoringMCMC.run."""
        b = self.b
        b.init(self.rand.seed + iteration, self.rand.glibc)
        limit = max_sweeps if max_sweeps else self.param.maxRip + 2
        t = 0
        done = False
        while t < limit:
            k = min(self.check_every, limit - t)
            for _ in range(k):
                self._step(t)
                t += 1
            done, tdev, err = b.state()
            if err:
                raise RuntimeError("partitioned sweep: device error flag (footer event overflow)")
            if done:
                break
        self.sweeps = t
        b.glibc_window(self.rand.glibc)
        return done

    def coloring(self) -> np.ndarray:
        return self.b.coloring()

    def trajectory(self) -> np.ndarray:
        return self.b.trajectory()
