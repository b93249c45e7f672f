"""Summarise MCMC_SOLO_TRACE stamps (dense_sparse.h dc_leader_solo, wall_clock64 at 100 MHz):
per solo sweep [0] start, [1] before the evaluation, [4] candidates evaluated and the open summary
read, [2] evaluation done, [5] loop control done, [6] events drawn, [3] accepted; sweeps with a move
phase also [7] the helpers' moves done. Medians in us."""
import sys

import numpy as np

ts = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
r = ts[(ts[:, 0] > 0) & (ts[:, 3] > 0)]
if len(r) < 2:
    print("no solo sweeps traced")
    sys.exit(0)
us = lambda x: float(np.median(x)) / 100.0
mv = r[:, 7] > 0
per = np.diff(r[:, 0])
print(f"solo sweeps traced: {len(r)}, with a move phase: {int(mv.sum())}")
print(f"  setup {us(r[~mv,1]-r[~mv,0]):.2f} us, evaluation {us(r[:,2]-r[:,1]):.2f} us, accept {us(r[:,3]-r[:,2]):.2f} us, "
      f"period median {us(per):.2f} us, mean {np.mean(per)/100:.2f} us")
if (r[:, 4] > 0).all() and (r[:, 5] > 0).all() and (r[:, 6] > 0).all():
    print(f"  evaluation: candidates + open summary {us(r[:,4]-r[:,1]):.2f}, open rows {us(r[:,2]-r[:,4]):.2f}; "
          f"accept: loop control {us(r[:,5]-r[:,2]):.2f}, events {us(r[:,6]-r[:,5]):.2f}, writes + state {us(r[:,3]-r[:,6]):.2f} us")
if mv.any():
    m = r[mv]
    print(f"  move phase (post -> helpers done) {us(m[:,7]-m[:,0]):.2f} us, to evaluation {us(m[:,1]-m[:,0]):.2f} us")
rb = ts.reshape(-1)[8 * 4096 - 64:]
if rb[63] == 1:
    t0 = rb[0]
    blocks = [(rb[1 + 2 * i] - t0, rb[2 + 2 * i] - t0) for i in range(28) if rb[2 + 2 * i] > 0]
    st = [blocks[0][0]] + [blocks[i][0] - blocks[i - 1][1] for i in range(1, len(blocks))]
    sm = [b[1] - b[0] for b in blocks]
    print(f"rebuild chunk (workgroup 0): {len(blocks)} blocks, stage+barrier median {np.median(st)/100:.2f} us, "
          f"stream median {np.median(sm)/100:.2f} us, write-out {(rb[62] - t0 - blocks[-1][1])/100:.2f} us, "
          f"total {(rb[62] - t0)/100:.2f} us")
