"""TEST INFRASTRUCTURE: a CPU rank backend for mcmc_colorer_amd.distributed.PartitionedColoringMCMC.

It restates, in numpy/float32, the partitioned protocol the HIP kernels implement (sweep of the
owned rows -> footer [Cviol_local, E, flags, sorted events] -> exchange -> commit with the
rank-ordered glibc replay; a list longer than the footer pauses the loop for the spill exchange),
with the same buffers (colour replicas in vertex order, rank r owning rows [bounds[r], bounds[r+1]);
footer buffers of world x FOOTER_WORDS words), using the oracle_np RNG restatements. Driving the
product's driver over gloo with this backend checks the exchange sequence and the protocol on CPU;
the HIP side of the same protocol is checked on the GPU (tests/test_gpu_parity.py,
tests/test_multi.py).
"""
from __future__ import annotations

import numpy as np
import torch

import oracle_np as NP

FOOTER_WORDS = 1024
FOOTER_EVENTS = FOOTER_WORDS - 4
DELTA_WORDS = 4096                      # MCMC_DELTA_WORDS
DELTA_PAIRS = (DELTA_WORDS - 2) // 2
M31 = 2147483647


class NumpyRank:
    def __init__(self, off, idx, nCol, world, rank, eps=1e-8, maxRip=250, taboo=0, z=0, bounds=None):
        self.off, self.idx = off.astype(np.int64), idx.astype(np.int64)
        self.n = len(off) - 1
        self.nCol, self.eps, self.maxRip, self.tabooIter, self.z = nCol, np.float32(eps), maxRip, taboo, z
        self.world, self.rank = world, rank
        if bounds is None:   # mcmc_part_plan_rows: ceil(n / world) rounded up to 64
            S = ((self.n + world - 1) // world + 63) // 64 * 64
            bounds = [min(r * S, self.n) for r in range(world)] + [self.n]
        self.bounds = [int(x) for x in bounds]
        self.cb = 2 if nCol > 256 else 1
        self.dt = np.uint16 if self.cb == 2 else np.uint8
        self.v_begin, self.v_end = self.bounds[rank], self.bounds[rank + 1]
        self.colors = [torch.zeros((self.n + 256) * self.cb, dtype=torch.uint8) for _ in range(2)]
        self.foot = [torch.zeros(world * FOOTER_WORDS, dtype=torch.int32) for _ in range(2)]
        self.dlt = [torch.zeros(world * DELTA_WORDS, dtype=torch.int32) for _ in range(2)]

    def delta_ok(self):
        return True

    def _view(self, buf):
        return buf.numpy()[: self.n * self.cb].view(self.dt)

    def _put(self, buf, v, c):
        self._view(buf)[v] = c

    # -- interface used by PartitionedColoringMCMC ------------------------------------------------
    def init(self, seed, glibc):
        gen = NP.Minstd(seed)
        C = np.zeros(self.n, dtype=np.int64)
        for v in range(self.n):
            C[v], _ = NP.uniform_int(gen, self.nCol)
        self._view(self.colors[0])[:] = C.astype(self.dt)
        self.x0 = gen.x                      # engine state after K0 draws
        self.t, self.done, self.err, self.paused = 0, False, 0, 0
        self.ring = [int(w) for w in glibc.window]   # oldest first
        self.taboo = np.zeros(self.v_end - self.v_begin, dtype=np.int64)
        self.traj = []
        self.events = []
        self.hi = np.float32(np.float32(1.0) - np.float32(self.nCol - 1) * self.eps)

    def _glibc(self):
        v = (self.ring[0] + self.ring[28]) & 0xFFFFFFFF
        self.ring = self.ring[1:] + [v]
        return v >> 1

    def sweep(self, delta=False):
        if self.done or self.paused:
            return
        t, n = self.t, self.n
        C = self._view(self.colors[t & 1]).astype(np.int64)
        nxt = self.colors[(t + 1) & 1]
        viol_local, events, changed = 0, [], []
        xt = (self.x0 * pow(NP.A_MINSTD, t * n, M31)) % M31
        for v in range(self.v_begin, self.v_end):
            nb = self.idx[self.off[v]:self.off[v + 1]]
            occ = np.zeros(self.nCol, dtype=bool)
            occ[C[nb]] = True
            pop = int(occ.sum())
            zvcomp = self.nCol - pop
            viol = bool(occ[C[v]])
            viol_local += viol
            l = v - self.v_begin
            if self.taboo[l] > 0:
                self.taboo[l] -= 1
                self._put(nxt, v, int(C[v]))
                continue
            u = NP.canonical((xt * pow(NP.A_MINSTD, v + 1, M31)) % M31)
            if viol and zvcomp > 0:
                pf = np.float32(np.float32(np.float32(1.0) - np.float32(self.eps * np.float32(pop))) / np.float32(zvcomp))
                p = [self.eps if occ[c] else pf for c in range(self.nCol)]
            else:
                p = [self.hi if c == C[v] else self.eps for c in range(self.nCol)]
            cdf, new = np.float32(0.0), self.nCol
            for c in range(self.nCol):
                cdf = np.float32(cdf + p[c])
                if cdf > u:
                    new = c
                    break
            if new == self.nCol:
                events.append(v)
                self._put(nxt, v, int(C[v]))
            else:
                self._put(nxt, v, new)
                self.taboo[l] = self.tabooIter if new == C[v] else 0
                if new != C[v]:
                    changed.append((v, new))
        self.events = sorted(events)
        if delta:   # this rank's slot: [pairs appended, 0, (v, colour) pairs up to the slot's capacity]
            d = np.zeros(DELTA_WORDS, dtype=np.uint32)
            d[0] = len(changed)
            for i, (v, c) in enumerate(changed[:DELTA_PAIRS]):
                d[2 + 2 * i], d[3 + 2 * i] = v, c
            self.dlt[(t + 1) & 1][self.rank * DELTA_WORDS:(self.rank + 1) * DELTA_WORDS] = torch.from_numpy(d.view(np.int32))
        f = np.zeros(FOOTER_WORDS, dtype=np.uint32)
        En = min(len(events), FOOTER_EVENTS)
        f[0], f[1], f[2] = viol_local & 0xFFFFFFFF, viol_local >> 32, len(events)
        f[3] = 2 if len(events) > FOOTER_EVENTS else 0      # spill: the list does not fit the footer
        f[4:4 + En] = self.events[:En]
        self.foot[(t + 1) & 1][self.rank * FOOTER_WORDS:(self.rank + 1) * FOOTER_WORDS] = torch.from_numpy(f.view(np.int32))

    def _footers(self):
        return self.foot[(self.t + 1) & 1].numpy().view(np.uint32).reshape(self.world, FOOTER_WORDS)

    def commit(self, mode=0, spill=None, stride=0):
        """mode 1: delta (every other rank's changed vertices into both replicas), 0: full, -1: the
        full-mode resumption of a paused sweep (its rows were exchanged in full)."""
        resume = spill is not None or mode == -1
        if self.done or (self.paused and not resume) or (resume and not self.paused):
            return
        F = self._footers()
        viol = int(sum(int(r[0]) | (int(r[1]) << 32) for r in F))
        t = self.t
        stop = t == self.maxRip + 1 or viol <= self.z
        D = self.dlt[(t + 1) & 1].numpy().view(np.uint32).reshape(self.world, DELTA_WORDS)
        dovf = mode == 1 and any(int(D[r][0]) > DELTA_PAIRS for r in range(self.world))
        spilled = spill is None and any(int(r[3]) & 2 for r in F)
        if not resume and not stop and (spilled or dovf):
            self.paused = (2 if spilled else 0) | (4 if dovf else 0)   # every rank sees the same data
            return
        self.paused = 0
        self.traj.append(viol)
        if stop:
            self.done, self.iter, self.final = True, t, viol
            return
        if spill is None:
            events = [int(e) for r in F for e in r[4:4 + int(r[2])]]
        else:
            sp = spill.numpy().view(np.uint32)
            events = [int(e) for r in range(self.world) for e in sp[r * stride: r * stride + int(F[r][2])]]
        C = self._view(self.colors[t & 1]).copy()
        nxt = self.colors[(t + 1) & 1]
        cur = self.colors[t & 1]
        if mode == 1:   # the other ranks' changes into both replicas
            for r in range(self.world):
                if r == self.rank:
                    continue
                for i in range(int(D[r][0])):
                    v, c = int(D[r][2 + 2 * i]), int(D[r][3 + 2 * i])
                    self._put(nxt, v, c)
                    self._put(cur, v, c)
        for v in events:                     # ascending: ranks own ascending ranges
            c = self._glibc() % (self.nCol - 1)
            self._put(nxt, v, c)
            if self.v_begin <= v < self.v_end:
                self.taboo[v - self.v_begin] = self.tabooIter if c == int(C[v]) else 0
            elif mode == 1:
                self._put(cur, v, c)
        self.t = t + 1

    def sync_remote(self):
        """Both replicas equal off this rank's rows: the next buffer takes the current colouring's."""
        if self.done or self.paused:
            return
        cur, nxt = self._view(self.colors[self.t & 1]), self._view(self.colors[(self.t + 1) & 1])
        nxt[: self.v_begin] = cur[: self.v_begin]
        nxt[self.v_end:] = cur[self.v_end:]

    def state(self):
        return self.done, self.t, self.paused

    def exchange_buffers(self, t):
        nb = (t + 1) & 1
        return (self.colors[nb], [(self.bounds[r] * self.cb, self.bounds[r + 1] * self.cb) for r in range(self.world)],
                self.foot[nb], self.dlt[nb])

    def spill_counts(self):
        return self._footers()[:, 2].astype(np.uint32)

    def spill_local(self, stride):
        out = np.zeros(max(stride, 1), dtype=np.uint32)
        out[: len(self.events)] = self.events
        return torch.from_numpy(out.view(np.int32))


    def glibc_window(self, glibc):
        glibc.window[:] = np.array(self.ring, dtype=np.uint32)

    def coloring(self):
        return self._view(self.colors[self.t & 1]).astype(np.uint32)

    def trajectory(self):
        return np.array(self.traj, dtype=np.uint64)
