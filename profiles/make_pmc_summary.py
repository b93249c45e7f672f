"""Folds rocprofv3 PMC passes (scripts/gpu_prof.sh: pass 1 FETCH_SIZE, pass 2 WRITE_SIZE) into
profiles/pmc_summary.json, which bench.py reads for roofline.traffic.

  python profiles/make_pmc_summary.py <prof_dir> <key> [kernel-substring[;...]] [last-K] [sweeps-per-launch]

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is doubled;
WRITE_SIZE is taken as is. Values are averaged over the kernel's profiled launches; a
semicolon-separated kernel list (one sweep made of several launches, e.g. the wide sweep) sums the
per-launch means of each. last-K: only each kernel's last K launches (the bench's timed sweeps,
not the convergence run's early exits before them). sweeps-per-launch: a persistent launch
(dc_multi_kernel, ws_kernel) runs all K timed sweeps; its bytes are divided by K into
hbm_bytes_per_sweep, which bench.py's roofline.traffic reports (per sweep, like `achieved`).
"""
import csv
import json
import sys
from pathlib import Path


def mean_counter(path: Path, counter: str, kernel: str, last: int = 0) -> tuple[float, int]:
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if last:
        vals = vals[-last:]
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel '{kernel}' in {path}")
    return sum(vals) / len(vals), len(vals)


def main() -> None:
    prof, key = Path(sys.argv[1]), sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "sweep_"
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    spl = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    fetch_kib = write_kib = 0.0
    nf = nw = 0
    for k in kernel.split(";"):
        f, n1 = mean_counter(prof / "pmc1" / "run_counter_collection.csv", "FETCH_SIZE", k, last)
        w, n2 = mean_counter(prof / "pmc2" / "run_counter_collection.csv", "WRITE_SIZE", k, last)
        fetch_kib, write_kib, nf, nw = fetch_kib + f, write_kib + w, max(nf, n1), max(nw, n2)
    out = Path(__file__).resolve().parent / "pmc_summary.json"
    d = json.loads(out.read_text()) if out.exists() else {}
    d[key] = {
        "kernel_substring": kernel,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib": write_kib,
        "launches": [nf, nw],
        "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
        "hbm_write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": 2 * fetch_kib * 1024 + write_kib * 1024,
        "sweeps_per_launch": spl,
        "hbm_bytes_per_sweep": (2 * fetch_kib * 1024 + write_kib * 1024) / spl,
        "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB -> bytes",
        "source": str(prof),
        "last_launches": last or None,
    }
    out.write_text(json.dumps(d, indent=1) + "\n")
    print(key, json.dumps(d[key]))


if __name__ == "__main__":
    main()
