"""Summarise rocprofv3 counter passes into per-kernel HBM bytes per launch.

usage: python tools/pmc_summary.py --fetch DIR --write DIR --probe-bytes N --out profiles/X.json
                                   [--trace DIR] [--label TEXT]

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md "HBM":
  * FETCH_SIZE and WRITE_SIZE are in KiB (x 1024);
  * on gfx950 FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane)
    coalesced streaming read -> x 2;
  * cross-check: the read probe kernel streams a known byte count with the
    same load width, so probe_bytes / (2 * probe FETCH bytes) should be ~1.
Each counter comes from its own rocprofv3 pass (FETCH_SIZE alone, WRITE_SIZE
alone) with no tracing domains besides the kernel trace.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {
    "csum_flat_kernel": "csum_flat_kernel",
    "csum_batch_kernel": "csum_batch_kernel",
    "csum_kernel<": "csum_kernel",
    "read_probe_kernel": "read_probe_kernel",
}


def _short(name: str) -> str | None:
    for sub, short in KERNELS.items():
        if sub in name:
            return short
    return None


def read_counters(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = _short(row.get("Kernel_Name", ""))
            if k:
                vals[k].append(float(row["Counter_Value"]))
    return vals


def read_trace(d: str):
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            k = _short(row["Name"])
            if k:
                out.setdefault(k, {"calls": 0, "total_ns": 0.0})
                out[k]["calls"] += int(row["Calls"])
                out[k]["total_ns"] += float(row["TotalDurationNs"])
    for v in out.values():
        v["avg_us"] = v["total_ns"] / v["calls"] / 1e3
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--probe-bytes", type=float, required=True)
    ap.add_argument("--alg-bytes", type=float, default=None, help="algorithmic bytes per csum launch")
    ap.add_argument("--alg-kernel", default="csum_flat_kernel", help="kernel the --alg-bytes figure belongs to")
    ap.add_argument("--label", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = read_counters(a.fetch, "FETCH_SIZE")
    write = read_counters(a.write, "WRITE_SIZE")
    trace = read_trace(a.trace) if a.trace else {}
    probe_f = fetch.get("read_probe_kernel")
    calib = None
    if probe_f:
        probe_raw = sum(probe_f) / len(probe_f) * 1024
        calib = a.probe_bytes / (2 * probe_raw)
    res = {"label": a.label, "probe_bytes": a.probe_bytes, "probe_calibration": calib, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = (sum(f) / len(f)) * 1024 if f else None
        wb = (sum(w) / len(w)) * 1024 if w else None
        entry = {
            "dispatches_fetch": len(f),
            "dispatches_write": len(w),
            "fetch_size_raw_bytes": fb,
            "write_size_bytes": wb,
            "hbm_read_bytes_per_launch": 2 * fb if fb is not None else None,
            "hbm_bytes_per_launch": (2 * fb if fb else 0) + (wb or 0) if (fb or wb) else None,
        }
        if k in trace:
            entry["avg_us_kernel_trace"] = round(trace[k]["avg_us"], 2)
            entry["calls_kernel_trace"] = trace[k]["calls"]
        if a.alg_bytes and k == a.alg_kernel and entry["hbm_bytes_per_launch"]:
            entry["alg_bytes_per_launch"] = a.alg_bytes
            entry["traffic_over_alg"] = round(entry["hbm_bytes_per_launch"] / a.alg_bytes, 4)
        res["kernels"][k] = entry
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
