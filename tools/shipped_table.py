"""One table for DESIGN.md §6: every config of one session (one box, one
tree) — bench value, bench µs per launch, fraction of 8 TB/s by bench events
and by the trace of the same command, traffic over algorithmic bytes — from
gpurun_out/TAG/bench_*.log and TAG_pmc_*.json (tools/gpu_session.sh).

usage: python tools/shipped_table.py gpurun_out/TAG [more session dirs: a box-spread column]
"""
from __future__ import annotations

import glob
import json
import os
import sys

ORDER = ["headline", "udp1500", "udp1500_launch_single", "mixed", "mixed_align_64", "tcp64k", "tcp64k_seglen_65535",
         "slots", "frags", "fill", "e2e", "sweep"]


def lines(d: str) -> dict[str, dict]:
    out = {}
    # a prof: step's trace pass prints the bench line of the profiled command (--steps 10)
    for f in sorted(glob.glob(os.path.join(d, "prof_*_trace.log"))):
        name = os.path.basename(f)[len("prof_"):-len("_trace.log")]
        for ln in open(f):
            if ln.startswith("{"):
                out[name] = json.loads(ln)
    for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
        name = os.path.basename(f)[len("bench_"):-len(".log")]
        for ln in open(f):
            if ln.startswith("{"):
                out[name] = json.loads(ln)  # the last line of the file (a step may append)
    return out


def pmcs(d: str) -> dict[str, dict]:
    out = {}
    for f in glob.glob(os.path.join(d, "*_pmc_*.json")):
        cfg = os.path.basename(f).split("_pmc_", 1)[1][:-len(".json")]
        k = next(iter(json.load(open(f))["kernels"].values()))
        out[cfg] = k
    return out


def row(name: str, d: dict, p: dict | None) -> str:
    r = d.get("roofline") or {}
    if "variants" in d:  # cfg 5: PCIe-bound, no roofline
        return f"| {name} | {d['value']:.1f} GiB/s | {d['best_variant']} {d['variants'][d['best_variant']]['ms_per_batch']} ms / batch | | PCIe-bound | | |"
    trace_us = p.get("avg_us_step_kernels") or p.get("avg_us_timed") if p else None
    ftrace = p.get("frac_from_trace_step") or p.get("frac_from_trace") if p else None
    traffic = p.get("traffic_over_alg_step") or p.get("traffic_over_alg") if p else None
    return (f"| {name} | {d['value']:.0f} GiB/s | {r.get('avg_launch_us', '')} | "
            f"{'' if trace_us is None else round(trace_us, 1)} | {r.get('frac', '')} | "
            f"{'' if ftrace is None else ftrace} | {'' if traffic is None else traffic} |")


def main():
    dirs = sys.argv[1:]
    first = lines(dirs[0])
    pm = pmcs(dirs[0])
    print("| config | value | bench µs / launch | trace µs | of 8 TB/s (bench) | (trace) | traffic / alg |"
          + ("" if len(dirs) == 1 else " other boxes (bench frac) |"))
    print("|---|---|---|---|---|---|---|" + ("" if len(dirs) == 1 else "---|"))
    names = sorted(first, key=lambda n: ORDER.index(n) if n in ORDER else 99)
    for n in names:
        # the headline's profile: the driver's form profiled as prof:udp1500+--steps+200+--warmup+5
        # where the session has it, else the 10-step udp1500 profile
        cfg = n if n != "headline" else ("udp1500_steps_200_warmup_5" if "udp1500_steps_200_warmup_5" in pm
                                         else "udp1500")
        line = row(n, first[n], pm.get(cfg))
        if len(dirs) > 1:
            others = [lines(x).get(n, {}).get("roofline", {}) or {} for x in dirs[1:]]
            line += " " + " / ".join(str(o.get("frac", "–")) for o in others) + " |"
        print(line)


if __name__ == "__main__":
    main()
