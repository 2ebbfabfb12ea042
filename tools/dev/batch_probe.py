"""Probe: do rotated batches of the same shape run at different speeds, and
does it follow their placement?  Builds R Zipf (cfg 3) or 1500 B (cfg 2)
batches as bench.py does, then times each batch alone (interleaved rounds,
median) and prints its data pointer's offset within a 2 MiB page."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native, synth  # noqa: E402


def main():
    native.check(native.load().sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    kind = sys.argv[1] if len(sys.argv) > 1 else "zipf"
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    if kind == "zipf":
        lens = synth.zipf_lengths(3_400_000, seed=0x5EA57A2C)
        bs = [devsynth.mixed_frames(lens, seed=0x5EA57A2C + 7 * r, device=dev) for r in range(R)]
    else:
        bs = [devsynth.udp_frames(1 << 20, 1500, seed=100 + r, device=dev) for r in range(R)]
    n = bs[0].n
    out = torch.empty(2 * n, dtype=torch.int16, device=dev)
    pre = [batch.prepare_call("sccsum_ipv4_frames", b.data, b.bytes_len, b.off, b.length, out, None, b.n, b.max_len)
           for b in bs]
    s = torch.cuda.current_stream()
    t = {r: [] for r in range(R)}
    for _ in range(3):
        for p in pre:
            p(s)
    torch.cuda.synchronize()
    for _ in range(12):
        for r in range(R):
            pre[(r + 1) % R](s)  # a different batch first, so the timed one is not cached
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pre[r](s)
            e1.record()
            torch.cuda.synchronize()
            t[r].append(e0.elapsed_time(e1) * 1e3)
    # chains: K launches back to back inside one event pair (K = 1, 2, 4, 8), over distinct batches
    for K in (1, 2, 4, 8):
        tk = []
        for _ in range(8):
            pre[R - 1](s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for j in range(K):
                pre[j % R](s)
            e1.record()
            torch.cuda.synchronize()
            tk.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"kind": kind, "chain": K, "median_us": round(float(np.median(tk)), 1),
                          "per_launch_us": round(float(np.median(tk)) / K, 1)}), flush=True)
    for r, b in enumerate(bs):
        print(json.dumps({"kind": kind, "batch": r, "median_us": round(float(np.median(t[r])), 1),
                          "min_us": round(float(np.min(t[r])), 1),
                          "data_ptr_mod_2MiB": b.data.data_ptr() % (2 << 20),
                          "off_ptr_mod_2MiB": b.off.data_ptr() % (2 << 20), "bytes": b.bytes_len}), flush=True)


if __name__ == "__main__":
    main()
