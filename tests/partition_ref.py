"""TEST INFRASTRUCTURE: a CPU rank backend for mcmc_colorer_amd.distributed.PartitionedColoringMCMC.

It restates, in numpy/float32, the partitioned protocol the HIP kernels implement (sweep of the
owned rows -> footer [Cviol_local, E, flags, sorted events] -> all-gather -> commit with the
rank-ordered glibc replay), with the same partitioned buffer layout (per-rank regions of colours
followed by the footer, one all-gather per sweep), using the oracle_np RNG restatements. Driving the product's driver
over gloo with this backend checks the exchange sequence and the protocol on CPU; the HIP side of
the same protocol is checked on the GPU (tests/test_gpu_parity.py::test_partitioned_lockstep).
"""
from __future__ import annotations

import numpy as np
import torch

import oracle_np as NP

FOOTER_WORDS = 1024
M31 = 2147483647


class NumpyRank:
    def __init__(self, off, idx, nCol, world, rank, eps=1e-8, maxRip=250, taboo=0, z=0):
        self.off, self.idx = off.astype(np.int64), idx.astype(np.int64)
        self.n = len(off) - 1
        self.nCol, self.eps, self.maxRip, self.tabooIter, self.z = nCol, np.float32(eps), maxRip, taboo, z
        self.world, self.rank = world, rank
        # region layout of mcmc_part_layout2: S = ceil(n/world) rounded up to 16, region r =
        # [colours of rows r*S .. r*S+S-1 | footer of rank r], P = cb*S + 4*FOOTER_WORDS bytes with
        # cb = 2 colour bytes for nCol > 256 (the wide sweep), else 1
        self.S = ((self.n + world - 1) // world + 15) // 16 * 16
        self.cb = 2 if nCol > 256 else 1
        self.P = self.cb * self.S + 4 * FOOTER_WORDS
        self.v_begin, self.v_end = min(rank * self.S, self.n), min((rank + 1) * self.S, self.n)
        self.colors = [torch.zeros(world * self.P + 256, dtype=torch.uint8) for _ in range(2)]

    def _view(self, buf):
        """Colours of all n vertices (a copy) from a partitioned buffer."""
        dt = np.uint16 if self.cb == 2 else np.uint8
        return np.concatenate([buf[r * self.P: r * self.P + self.cb * self.S].numpy().view(dt)
                               for r in range(self.world)])[: self.n]

    def _put(self, buf, v, c):
        o = (v // self.S) * self.P + self.cb * (v % self.S)
        buf[o] = c & 0xFF
        if self.cb == 2:
            buf[o + 1] = c >> 8

    # -- interface used by PartitionedColoringMCMC ------------------------------------------------
    def init(self, seed, glibc):
        gen = NP.Minstd(seed)
        draws = 0
        C = np.zeros(self.n, dtype=np.int64)
        for v in range(self.n):
            C[v], d = NP.uniform_int(gen, self.nCol)
            draws += d
        for v in range(self.n):
            self._put(self.colors[0], v, int(C[v]))
        self.x0 = gen.x                      # engine state after K0 draws
        self.t, self.done, self.err = 0, False, 0
        self.ring = [int(w) for w in glibc.window]   # oldest first
        self.taboo = np.zeros(self.v_end - self.v_begin, dtype=np.int64)
        self.traj = []
        self.hi = np.float32(np.float32(1.0) - np.float32(self.nCol - 1) * self.eps)

    def _glibc(self):
        v = (self.ring[0] + self.ring[28]) & 0xFFFFFFFF
        self.ring = self.ring[1:] + [v]
        return v >> 1

    def sweep(self):
        if self.done:
            return
        t, n = self.t, self.n
        C = self._view(self.colors[t & 1]).astype(np.int64)
        nxt = self.colors[(t + 1) & 1]
        viol_local, events = 0, []
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
        f = np.zeros(FOOTER_WORDS, dtype=np.uint32)
        f[0], f[1], f[2] = viol_local & 0xFFFFFFFF, viol_local >> 32, len(events)
        f[4:4 + len(events)] = sorted(events)
        off = self.rank * self.P + self.cb * self.S
        nxt[off: off + 4 * FOOTER_WORDS] = torch.from_numpy(f.view(np.uint8))

    def commit(self):
        if self.done:
            return
        nb = self.colors[(self.t + 1) & 1].numpy()
        F = np.stack([nb[r * self.P + self.cb * self.S: (r + 1) * self.P].view(np.uint32) for r in range(self.world)])
        viol = int(sum(int(r[0]) | (int(r[1]) << 32) for r in F))
        events = [int(e) for r in F for e in r[4:4 + int(r[2])]]
        t = self.t
        self.traj.append(viol)
        if t == self.maxRip + 1 or viol <= self.z:
            self.done, self.iter, self.final = True, t, viol
            return
        C = self._view(self.colors[t & 1])
        nxt = self.colors[(t + 1) & 1]
        for v in events:                     # ascending: ranks own ascending ranges
            c = self._glibc() % (self.nCol - 1)
            self._put(nxt, v, c)
            if self.v_begin <= v < self.v_end:
                self.taboo[v - self.v_begin] = self.tabooIter if c == int(C[v]) else 0
        self.t = t + 1

    def state(self):
        return self.done, self.t, self.err

    def region(self, t):
        nxt = self.colors[(t + 1) & 1]
        return nxt[: self.world * self.P], nxt[self.rank * self.P:(self.rank + 1) * self.P]

    def glibc_window(self, glibc):
        glibc.window[:] = np.array(self.ring, dtype=np.uint32)

    def coloring(self):
        return self._view(self.colors[self.t & 1]).astype(np.uint32)

    def trajectory(self):
        return np.array(self.traj, dtype=np.uint64)
