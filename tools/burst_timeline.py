"""Summarise a burst queue's kernel trace (rocprofv3 --kernel-trace of
build/burst_gpu): how much of the run the packet-reading kernel (the
fragment-list kernel, or the gather of the two-pass form) keeps PCIe busy,
per-batch time, kernel durations, overlap and gaps between batches.

usage: python tools/burst_timeline.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys


def main():
    for d in sys.argv[1:]:
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
        main_k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                        if "desc_kernel" in r["Kernel_Name"] or "gather_kernel" in r["Kernel_Name"])
        sub = main_k[10:-10]  # steady state
        busy, cs, ce = 0, None, None
        for s, e in sub:
            if cs is None:
                cs, ce = s, e
            elif s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        span = sub[-1][1] - sub[0][0]
        durs = sorted((e - s) / 1e3 for s, e in sub)
        gaps = sorted((b[0] - a[1]) / 1e3 for a, b in zip(sub, sub[1:]) if b[0] >= a[1])
        ov = sum(1 for a, b in zip(sub, sub[1:]) if b[0] < a[1])
        print(f"{d}: {len(main_k)} batches; steady state {len(sub)}: span {span / 1e3:.0f} us, reading kernel busy "
              f"{busy / span:.3f}, {span / 1e3 / len(sub):.1f} us per batch; kernel us p10/p50/p90 "
              f"{durs[len(durs) // 10]:.1f}/{durs[len(durs) // 2]:.1f}/{durs[9 * len(durs) // 10]:.1f}; "
              f"{ov} overlapping pairs; gap us p50/max "
              f"{(gaps[len(gaps) // 2] if gaps else 0):.1f}/{(gaps[-1] if gaps else 0):.1f}")


if __name__ == "__main__":
    main()
