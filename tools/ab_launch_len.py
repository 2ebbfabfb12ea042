"""Per-launch fixed cost of the flat kernel: launches over k = 1, 2, 4, 8
distinct batches (one sccsum_ipv4_frames_multi launch over k queues), batches
rotated so no launch rereads cached lines.  A line fit T(k) = a + k * b gives
the launch's fixed cost a (ramp, drain, dispatch) and the steady-state
per-batch time b.

Batches: cfg 2's 1 M x 1500 B frames (default), or with --mixed cfg 3's
Zipf(1.2) frames 64..9000 B packed at odd offsets (3.4 M frames, ~1.5 GB per
batch).  Outputs: both checksums per frame (out2, 4 B; the default), or with
--verify-only the status byte alone (the reference's verify keeps only
get() != 0: ip.cc:121-127).

usage: python tools/ab_launch_len.py [--reps R] [--tiles 64,32] [--mixed] [--verify-only] [--ks 1,2,4,8]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seastar_amd import batch, devsynth, native, synth  # noqa: E402

FRAME = 1500


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reps_pos", nargs="?", type=int, default=None)
    ap.add_argument("tiles_pos", nargs="?", default=None)
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--tiles", default="64")
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--verify-only", action="store_true")
    ap.add_argument("--ks", default="1,2,4,8")
    a = ap.parse_args()
    reps = a.reps_pos or a.reps
    tiles = a.tiles_pos or a.tiles
    native.check(native.load().sccsum_init(0), "sccsum_init")
    dev = torch.device("cuda:0")
    ks = [int(x) for x in a.ks.split(",")]
    NB = max(12, 2 * max(ks))
    if a.mixed:
        n = 3_400_000
        lens = synth.zipf_lengths(n, seed=0x5EA57A2C)
        bs = [devsynth.mixed_frames(lens, seed=0x5EA57A2C + 7 * r, device=dev) for r in range(NB)]
        nbytes = int(lens.sum())
    else:
        n = 1 << 20
        bs = [devsynth.udp_frames(n, FRAME, seed=101 + r, device=dev) for r in range(NB)]
        nbytes = n * FRAME
    outs = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(max(ks))]
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(max(ks))]
    s = torch.cuda.current_stream()
    print(f"{'cfg 3 Zipf frames' if a.mixed else 'cfg 2 1500 B frames'}: {n} frames, {nbytes} B per batch; "
          f"{'status only (verify-only)' if a.verify_only else 'out2 (both checksums)'}", flush=True)
    for tp in [int(x) for x in tiles.split(",")]:
        native.check(native.load().sccsum_set_tile_packets(tp), "tile_packets")
        print(f"tile_packets {tp}", flush=True)
        fit(bs, outs, sts, s, n, nbytes, NB, reps, ks, a.verify_only)


def fit(bs, outs, sts, s, n, nbytes, NB, reps, ks, verify_only):
    rows = []
    per_out = 1 if verify_only else 4
    for k in ks:
        def launch(j):
            items = [(bs[(j * k + q) % NB], None if verify_only else outs[q], sts[q] if verify_only else None)
                     for q in range(k)]
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
        alg = k * (nbytes + n * (12 + per_out))
        rows.append((k, us))
        print(f"k={k}: {us:8.1f} us/launch  {alg / us / 1e3:7.1f} GB/s  {alg / us / 1e3 / 8000:.4f} of 8 TB/s",
              flush=True)
    kk = np.array([r[0] for r in rows], float)
    ts = np.array([r[1] for r in rows], float)
    b, a = np.polyfit(kk, ts, 1)
    alg1 = nbytes + n * (12 + per_out)
    print(f"fit: T(k) = {a:.1f} us + k * {b:.1f} us  (steady {alg1 / b / 1e3:.1f} GB/s = "
          f"{alg1 / b / 1e3 / 8000:.4f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
