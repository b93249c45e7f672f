"""Two small persistent dense cases (3000 rows, p 0.3 and 0.02, 16 colours, 60 sweeps) against the oracle at
the workgroup size MCMC_DCM_BS names; prints each step as it goes. Usage: python scripts/dcm_bs_probe.py"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
t0 = time.perf_counter()
print("bs", os.environ.get("MCMC_DCM_BS", "default"), flush=True)
from test_gpu_parity import gpu_run, oracle_case  # noqa: E402
import mcmc_colorer_amd.colorer as M  # noqa: E402

for p in (0.3, 0.02):
    off, idx, nc, r = oracle_case(3000, p, 16, 31, epsilon=1e-8, maxRip=60)
    print(f"p {p}: oracle {time.perf_counter() - t0:.1f} s", flush=True)
    col, st, _ = gpu_run(M, off, idx, nc, 31, 3000 * 3001 // 2, maxRip=60)
    print(f"gpu {time.perf_counter() - t0:.1f} s", flush=True)
    got, want = col.coloring(), r.colors
    print("colours equal", bool((got == want).all()), "trajectory equal", col.trajectory().tolist() == r.traj.tolist(),
          flush=True)
    print(col.dense_stats(), flush=True)
