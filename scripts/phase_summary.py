"""Summarise MCMC_PHASE_DUMP files: per-workgroup phase durations of the last benchmarked sweep."""
import sys

import numpy as np

for path in sys.argv[1:]:
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    if len(t) == 4096:   # row 4095: the stand-alone commit's stamps (MCMC_COMMIT_PHASE)
        c = t[4095]
        t = t[:4095]
        if c[0] > 0:
            d = (c[[1, 2, 3, 4, 5]] - c[0]) / 100.0
            print(path, f"commit (E = {c[6]}): control {d[0]:.2f}  sorted {d[1]:.2f}  drawn {d[2]:.2f}  "
                        f"applied {d[3]:.2f}  end {d[4]:.2f} us from its start")
    t = t[t[:, 0] > 0]
    if len(t) == 0:
        continue
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0   # wall_clock64 = 100 MHz -> us
    names = ["start", "scan0", "scans_done", "eval_done", "tail_done"]
    print(path, "workgroups", len(t))
    for k, nm in enumerate(names):
        c = rel[:, k]
        print(f"  {nm:11s} min {c.min():7.2f} med {np.median(c):7.2f} max {c.max():7.2f} us")
    d = np.diff(rel[:, :5], axis=1)
    for k, nm in enumerate(["stage", "scan", "evaluate", "tail"]):
        print(f"  d_{nm:9s} min {d[:, k].min():7.2f} med {np.median(d[:, k]):7.2f} max {d[:, k].max():7.2f} us")

# accumulated shader cycles per phase kind (slots 5-7, tiled kernel; wave 0 of each workgroup)
for path in sys.argv[1:]:
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 8).astype(np.float64)
    t = t[:4095][t[:4095, 0] > 0]
    if len(t) == 0 or t[:, 5:8].sum() == 0:
        continue
    tot = t[:, 5:8].sum(axis=1)
    for k, nm in zip(range(5, 8), ["land+barriers", "scan", "evaluate"]):
        print(f"  cycles {nm:14s} median share {np.median(t[:, k] / tot):.3f}  median {np.median(t[:, k]) / 2.4e3:9.1f} us @2.4GHz")
