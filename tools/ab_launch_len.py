"""Per-launch fixed cost of the flat kernel: launches over k = 1, 2, 4, 8
distinct 1 M x 1500 B batches (one sccsum_ipv4_frames_multi launch over k
queues), batches rotated so no launch rereads cached lines.  A line fit
T(k) = a + k * b gives the launch's fixed cost a (ramp, drain, dispatch) and
the steady-state per-batch time b.

usage: python tools/ab_launch_len.py [reps] [tile_packets,...]
(tile_packets: sccsum_diag.h's per-tile packet cap, one fit per value)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seastar_amd import batch, devsynth, native  # noqa: E402

FRAME = 1500


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    native.check(native.load().sccsum_init(0), "sccsum_init")
    dev = torch.device("cuda:0")
    n, NB = 1 << 20, 12
    bs = [devsynth.udp_frames(n, FRAME, seed=101 + r, device=dev) for r in range(NB)]
    outs = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(8)]
    s = torch.cuda.current_stream()
    tps = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64]
    for tp in tps:
        native.check(native.load().sccsum_set_tile_packets(tp), "tile_packets")
        print(f"tile_packets {tp}", flush=True)
        fit(bs, outs, s, n, NB, reps)


def fit(bs, outs, s, n, NB, reps):
    rows = []
    for k in (1, 2, 4, 8):
        def launch(j):
            items = [(bs[(j * k + q) % NB], outs[q], None) for q in range(k)]
            batch.ipv4_frames_multi(items, stream=s)

        for j in range(4):
            launch(j)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for j in range(reps):
            launch(j)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        alg = k * n * (FRAME + 12 + 4)
        rows.append((k, us))
        print(f"k={k}: {us:8.1f} us/launch  {alg / us / 1e3:7.1f} GB/s  {alg / us / 1e3 / 8000:.4f} of 8 TB/s",
              flush=True)
    ks = np.array([r[0] for r in rows], float)
    ts = np.array([r[1] for r in rows], float)
    b, a = np.polyfit(ks, ts, 1)
    print(f"fit: T(k) = {a:.1f} us + k * {b:.1f} us  (steady {n * (FRAME + 16) / b / 1e3:.1f} GB/s = "
          f"{n * (FRAME + 16) / b / 1e3 / 8000:.4f} of 8 TB/s)")


if __name__ == "__main__":
    main()
