"""Folds the FETCH_SIZE / WRITE_SIZE passes over scripts/fetch_probe into bytes-per-counted-byte
ratios per access pattern (profiles/r05/fetch_calib.json).

  python scripts/fetch_calib.py <dir with probe.log, pmc1/, pmc2/> <out.json>

probe.log is fetch_probe's stdout; pmc1 / pmc2 hold rocprofv3's counter_collection.csv of the two
passes. The probe's own dispatches (not flush_kernel, not the runtime's fills) are, in order: stream16, stream4, stream2, gather2,
gather4, gather16, scatter2.
"""
import csv
import json
import sys
from pathlib import Path

ORDER = ["stream16", "stream4", "stream2", "gather2", "gather4", "gather16", "scatter2"]
PROBES = ("stream_kernel", "gather_kernel", "scatter2_kernel")   # (not flush_kernel, not hipMemset's fills)


def per_dispatch(path: Path, counter: str) -> list[float]:
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not any(k in r["Kernel_Name"] for k in PROBES):
            continue
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
        rows[d] = rows.get(d, 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main() -> None:
    d, out = Path(sys.argv[1]), Path(sys.argv[2])
    known = {}
    for line in (d / "probe.log").read_text().splitlines():
        f = line.split()
        if f and f[0] in ORDER:
            kv = dict(zip(f[1::2], f[2::2]))
            known[f[0]] = {k: int(v) for k, v in kv.items()}
    fetch = per_dispatch(next((d / "pmc1").rglob("*counter_collection.csv")), "FETCH_SIZE")
    write = per_dispatch(next((d / "pmc2").rglob("*counter_collection.csv")), "WRITE_SIZE")
    res = {}
    for i, name in enumerate(ORDER):
        k = known.get(name, {})
        fk = fetch[i] if i < len(fetch) else None
        wk = write[i] if i < len(write) else None
        r = {"fetch_size_kib": fk, "write_size_kib": wk, **k}
        if "bytes" in k and fk is not None:
            r["fetch_bytes_over_known"] = fk * 1024 / k["bytes"]
        if "lines64" in k:
            for key, kib in (("fetch", fk), ("write", wk)):
                if kib is not None:
                    r[f"{key}_per_access_B"] = kib * 1024 / k["accesses"]
                    r[f"{key}_over_lines64"] = kib * 1024 / (64 * k["lines64"])
                    r[f"{key}_over_lines128"] = kib * 1024 / (128 * k["lines128"])
        res[name] = r
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(res, indent=1) + "\n")
    for name, r in res.items():
        print(name, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()})


if __name__ == "__main__":
    main()
