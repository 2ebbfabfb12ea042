"""Read-probe ceiling by cache-policy mix: how many of the probe's 4 loads in
flight use the default policy (0, 1, 2, 4), interleaved, median of rounds.

usage: python tools/probe_policy.py [--rounds 6] [--gib 1.5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1_572_864_000)
    args = ap.parse_args()
    lib = native.load()
    native.check(lib.sccsum_init(0), "init")
    buf = torch.randint(0, 256, (args.bytes,), dtype=torch.uint8, device="cuda:0")
    sink = torch.zeros(lib.sccsum_read_probe_blocks(), dtype=torch.int64, device="cuda:0")
    modes = [0, 1, 2, 4]
    times = {m: [] for m in modes}
    for _ in range(args.rounds):
        for m in modes:
            native.check(lib.sccsum_set_probe_policy(m), "probe policy")
            batch.read_probe(buf, args.bytes, sink=sink)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                batch.read_probe(buf, args.bytes, sink=sink)
            e1.record()
            torch.cuda.synchronize()
            times[m].append(e0.elapsed_time(e1) / args.reps)
    native.check(lib.sccsum_set_probe_policy(0), "probe policy")
    for m in modes:
        t = np.median(times[m])
        print(json.dumps({"case": "read_probe", "default_loads_of_4": m, "median_us": round(t * 1e3, 1),
                          "GBps_median": round(args.bytes / (t / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
