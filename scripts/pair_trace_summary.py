"""Summarise MCMC_PAIR_TRACE files (the tiled sweep's last benchmarked sweep, per workgroup and pair):
per column-block index b -- pairs, open rows at the pair's top, and the median wall time (us) of
  scan    pair top -> the last wave's scan end
  skew    first -> last wave's scan end (dynamic claims balance the waves)
  eval    last scan end -> last wave's evaluation end (the group's last pair only)
  bar     -> the pair's closing barrier (DMA of the next pair landed, LDS drained)
and the share of the sweep each kind takes, summed over the workgroups."""
import sys

import numpy as np

REC, PMAX = 8, 256
for path in sys.argv[1:]:
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, PMAX, REC).astype(np.int64)
    t = t[t[:, 0, 0] > 0]
    nwg = len(t)
    recs = t.reshape(-1, REC)
    recs = recs[recs[:, 0] > 0]
    tail = recs[(recs[:, 5] >> 39) & 1 == 1]     # tail-queue blocks (tile_tail): durations in slots 2-4
    recs = recs[(recs[:, 5] >> 39) & 1 == 0]
    info = recs[:, 5]
    b = info & 0xFFFF
    nopen = (info >> 16) & 0xFFFFFF
    drain, sparse, last, allfull = [(info >> k) & 1 for k in (40, 41, 42, 43)]
    us = lambda x: x / 100.0
    start, smin, smax, eend, bend = recs[:, 0], recs[:, 1], recs[:, 2], recs[:, 3], recs[:, 4]
    scan = us(smax - start)
    skew = us(smax - smin)
    ev = np.where(last == 1, us(np.maximum(eend, smax) - smax), 0.0)
    bar = us(bend - np.where(last == 1, np.maximum(eend, smax), smax))
    ebar = np.where((last == 1) & (recs[:, 6] > 0), us(recs[:, 6] - smax), 0.0)   # eval: its barrier passed
    span = us(t[:, :, 4].max(axis=1) - t[:, 0, 0])
    print(f"{path}: {nwg} workgroups, {len(recs)} pairs ({len(recs) / nwg:.1f} per workgroup), "
          f"workgroup span med {np.median(span):.1f} max {span.max():.1f} us")
    print("   b  pairs  open(med)  drain sparse allfull   scan   skew   eval (bar)    bar   (median us)")
    for k in range(int(b.max()) + 1):
        m = b == k
        if not m.any():
            continue
        print(f"{k:4d} {m.sum():6d} {np.median(nopen[m]):9.0f} {drain[m].sum():6d} {sparse[m].sum():6d} "
              f"{allfull[m].sum():7d} {np.median(scan[m]):6.2f} {np.median(skew[m]):6.2f} "
              f"{np.median(ev[m][last[m] == 1]) if (last[m] == 1).any() else 0:6.2f} "
              f"({np.median(ebar[m][last[m] == 1]) if (last[m] == 1).any() else 0:5.2f}) {np.median(bar[m]):6.2f}")
    tot = scan.sum() + ev.sum() + bar.sum()
    print(f"  share: scan {scan.sum() / tot:.2f}  eval {ev.sum() / tot:.2f}  barrier {bar.sum() / tot:.2f}")
    if len(tail):
        tb = tail[:, 5] & 0xFFFF
        tq = (tail[:, 5] >> 16) & 0xFFFFFF
        print("  tail queue: block  workgroups  entries(med)  stage  load  scan  classify   (median us)")
        for k in np.unique(tb):
            m = tb == k
            print(f"              {k:5d} {m.sum():11d} {np.median(tq[m]):13.0f} {np.median(us(tail[m, 1] - tail[m, 0])):6.2f} "
                  f"{np.median(us(tail[m, 2])):5.2f} {np.median(us(tail[m, 3])):5.2f} {np.median(us(tail[m, 4])):9.2f}")
        per_wg = (us(tail[:, 1] - tail[:, 0]) + us(tail[:, 2]) + us(tail[:, 3]) + us(tail[:, 4])).sum() / nwg
        print(f"  tail queue total {per_wg:.1f} us per workgroup")
    for k in range(int(b.max()) + 1):
        m = b == k
        if m.any():
            print(f"  b={k}: scan+bar total {(scan[m].sum() + bar[m].sum()) / nwg:.1f} us per workgroup, eval "
                  f"{ev[m].sum() / nwg:.1f}")
