"""Cut the TIMED dispatches of a bench.py run out of rocprofv3 output and
summarise them: per-dispatch kernel trace (trimmed CSV, committed under
profiles/) and per-launch HBM bytes from separate FETCH_SIZE / WRITE_SIZE
counter passes of the same command.

bench.py prints, in its JSON line, roofline.trace_select = {kernel, skip,
count}: the timed launches are dispatches skip .. skip+count-1 (in dispatch
order) of the kernel whose name contains `kernel`.  The profiled runs are the
same command, so the same dispatches are selected from each pass.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md "HBM":
  * FETCH_SIZE and WRITE_SIZE are in KiB (x 1024);
  * on gfx950 FETCH_SIZE counts half the bytes of a wide (16 B/lane)
    coalesced streaming read -> x 2;
  * cross-check on the read probe kernel, which streams a known byte count
    (--probe-bytes) with the same load width: calibration ~= 1.

usage:
  python tools/prof_timed.py --bench-log LOG --trace DIR [--fetch DIR --write DIR --probe-bytes N]
                             --label TEXT --config NAME --out profiles/rNN_pmc_NAME.json
                             --trace-out profiles/rNN_trace_NAME.csv
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def bench_line(path: str) -> dict:
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def _rows(d: str, pattern: str):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        out.extend(csv.DictReader(open(f)))
    return out


def trace_dispatches(d: str, kernel: str):
    rows = [r for r in _rows(d, "*kernel_trace.csv") if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def counter_dispatches(d: str, kernel: str, counter: str):
    """[(dispatch_id, value)] in dispatch order; a counter with several
    instances per dispatch (per XCD / channel) is summed."""
    per = {}
    for r in _rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
            continue
        k = int(r["Dispatch_Id"])
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    return sorted(per.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench-log", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", default=None)
    ap.add_argument("--write", default=None)
    ap.add_argument("--probe-bytes", type=float, default=None)
    ap.add_argument("--probe-kernel", default="read_probe_kernel")
    ap.add_argument("--label", default="")
    ap.add_argument("--config", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--trace-out", required=True)
    a = ap.parse_args()

    line = bench_line(a.bench_log)
    roof = line["roofline"]
    sel = roof["trace_select"]
    kern, skip, count = sel["kernel"], int(sel["skip"]), int(sel["count"])

    tr = trace_dispatches(a.trace, kern)
    if len(tr) < skip + count:
        raise SystemExit(f"trace has {len(tr)} dispatches of {kern}, need {skip + count}")
    timed = tr[skip:skip + count]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in timed]
    gaps = [(int(b["Start_Timestamp"]) - int(a_["End_Timestamp"])) / 1e3 for a_, b in zip(timed, timed[1:])]
    cols = ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "SGPR_Count",
            "LDS_Block_Size", "Grid_Size_X", "Workgroup_Size_X"]
    os.makedirs(os.path.dirname(os.path.abspath(a.trace_out)), exist_ok=True)
    with open(a.trace_out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols + ["Duration_us"])
        for r, d in zip(timed, dur):
            w.writerow([r.get(c, "") for c in cols] + [f"{d:.3f}"])

    # further kernels of the same timed step (e.g. the fill's store pass): their
    # timed dispatches add to the step's kernel time
    extra = []
    step_rows = list(timed)
    for ex in roof.get("trace_select_extra", []):
        rows = trace_dispatches(a.trace, ex["kernel"])[int(ex["skip"]):int(ex["skip"]) + int(ex["count"])]
        step_rows += rows
        d_ex = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        if d_ex:
            extra.append({"kernel_match": ex["kernel"], "timed_dispatches": len(d_ex),
                          "avg_us_timed": round(statistics.mean(d_ex), 3)})
    alg = float(roof["alg_bytes_per_launch"])
    # with the step's launches alternated over two streams, consecutive launches
    # overlap (one's ramp under the other's drain): the per-launch time the
    # bench's events measure is then the span of the timed dispatches / count,
    # which the sum of durations exceeds by the overlap
    t_first = min(int(r["Start_Timestamp"]) for r in timed)
    t_last = max(int(r["End_Timestamp"]) for r in timed)
    span_us = (t_last - t_first) / 1e3 / count
    overlap = [max(0.0, (int(a_["End_Timestamp"]) - int(b["Start_Timestamp"])) / 1e3) for a_, b in zip(timed, timed[1:])]
    entry = {
        "kernel_match": kern,
        "timed_dispatches": count,
        "skipped_dispatches": skip,
        "all_dispatches_in_trace": len(tr),
        "avg_us_timed": round(statistics.mean(dur), 3),
        "median_us_timed": round(statistics.median(dur), 3),
        "min_us_timed": round(min(dur), 3),
        "max_us_timed": round(max(dur), 3),
        "mean_gap_us_between_timed": round(statistics.mean(gaps), 3) if gaps else None,
        "bench_avg_launch_us": roof["avg_launch_us"],
        "alg_bytes_per_launch": alg,
        "span_us_per_launch": round(span_us, 3),
        "mean_overlap_us_with_previous": round(statistics.mean(overlap), 3) if overlap else None,
        "achieved_GBps_from_trace": round(alg / span_us / 1e3, 1),
        "frac_from_trace": round(alg / span_us / 1e3 / roof["peak"], 4),
        "frac_from_mean_duration": round(alg / statistics.mean(dur) / 1e3 / roof["peak"], 4),
        "trace_csv": os.path.relpath(a.trace_out, os.path.dirname(os.path.abspath(a.out))),
    }
    if extra:
        step_us = statistics.mean(dur) + sum(e["avg_us_timed"] for e in extra)
        step_span = (max(int(r["End_Timestamp"]) for r in step_rows) -
                     min(int(r["Start_Timestamp"]) for r in step_rows)) / 1e3 / count
        entry["extra_kernels"] = extra
        entry["avg_us_step_kernels"] = round(step_us, 3)
        entry["span_us_per_step"] = round(step_span, 3)
        entry["frac_from_trace_step"] = round(alg / step_span / 1e3 / roof["peak"], 4)
    res = {"label": a.label, "config": a.config, "bench_line_value": line.get("value"), "kernels": {}}

    calib = None
    if a.fetch and a.write:
        fetch = counter_dispatches(a.fetch, kern, "FETCH_SIZE")
        write = counter_dispatches(a.write, kern, "WRITE_SIZE")
        if len(fetch) < skip + count or len(write) < skip + count:
            raise SystemExit(f"counter passes hold {len(fetch)} / {len(write)} dispatches of {kern}")
        f_t = [v for _, v in fetch[skip:skip + count]]
        w_t = [v for _, v in write[skip:skip + count]]
        fb = statistics.mean(f_t) * 1024
        wb = statistics.mean(w_t) * 1024
        entry.update({
            "fetch_size_raw_bytes": fb,
            "write_size_bytes": wb,
            "hbm_read_bytes_per_launch": 2 * fb,
            "hbm_bytes_per_launch": 2 * fb + wb,
            "traffic_over_alg": round((2 * fb + wb) / alg, 4),
            "write_bytes_per_packet": None,
        })
        for ex, e in zip(roof.get("trace_select_extra", []), extra):
            sk, ct = int(ex["skip"]), int(ex["count"])
            fx = [v for _, v in counter_dispatches(a.fetch, ex["kernel"], "FETCH_SIZE")[sk:sk + ct]]
            wx = [v for _, v in counter_dispatches(a.write, ex["kernel"], "WRITE_SIZE")[sk:sk + ct]]
            if fx and wx:
                # a pass of scattered small accesses: FETCH_SIZE x 2 is calibrated for wide
                # streaming reads only, so the raw value is reported beside it
                e["fetch_size_raw_bytes"] = statistics.mean(fx) * 1024
                e["write_size_bytes"] = statistics.mean(wx) * 1024
        if extra and all("write_size_bytes" in e for e in extra):
            step_bytes = 2 * fb + wb + sum(2 * e["fetch_size_raw_bytes"] + e["write_size_bytes"] for e in extra)
            entry["hbm_bytes_per_step"] = step_bytes
            entry["traffic_over_alg_step"] = round(step_bytes / alg, 4)
        if a.probe_bytes:
            pf = [v for _, v in counter_dispatches(a.fetch, a.probe_kernel, "FETCH_SIZE")]
            if pf:
                calib = a.probe_bytes / (2 * statistics.mean(pf) * 1024)
                res["kernels"][a.probe_kernel] = {"dispatches_fetch": len(pf),
                                                  "hbm_read_bytes_per_launch": 2 * statistics.mean(pf) * 1024}
    packets = line.get("config", {}).get("packets_per_gpu") or line.get("config", {}).get("segments_per_gpu")
    if packets and "write_size_bytes" in entry:
        entry["write_bytes_per_packet"] = round(entry["write_size_bytes"] / packets, 3)
    res["probe_bytes"] = a.probe_bytes
    res["probe_calibration"] = calib
    # bench.py reads kernels["csum_flat_kernel"]["hbm_bytes_per_launch"] for roofline.traffic
    # (per step when the step has further kernels)
    if "hbm_bytes_per_step" in entry:
        entry["hbm_bytes_per_launch_pass1"] = entry["hbm_bytes_per_launch"]
        entry["hbm_bytes_per_launch"] = entry["hbm_bytes_per_step"]
    res["kernels"]["csum_flat_kernel"] = entry
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
