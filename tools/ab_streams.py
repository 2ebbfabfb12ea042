"""A/B: cfg 2 steps (one sccsum_ipv4_frames_multi launch over a tx and an rx
batch of 1 M x 1500 B frames, 4 rotated pairs) on one stream vs alternated
over two or more streams, so a launch's ramp can overlap the previous launch's
drain.  Every step still reads its whole batch pair; the timed region is
fork-joined (all streams wait on the start event; the end event waits on all).

usage: python tools/ab_streams.py [steps] [rounds]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seastar_amd import batch, devsynth, native  # noqa: E402

FRAME = 1500


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    native.check(native.load().sccsum_init(0), "sccsum_init")
    dev = torch.device("cuda:0")
    n, R = 1 << 20, 4
    txs, rxs = [], []
    for r in range(R):
        tx = devsynth.udp_frames(n, FRAME, seed=11 + r, device=dev)
        first = batch.ipv4_frames(tx)
        txs.append(tx)
        rxs.append(devsynth.store_checksums(tx, first))
    torch.cuda.synchronize()
    alg = 2 * n * (FRAME + 12 + 4) + n
    for rnd in range(rounds):
        for ns in (1, 2, 3):
            streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
            outs = [(torch.empty(2 * n, dtype=torch.int16, device=dev), torch.empty(2 * n, dtype=torch.int16, device=dev),
                     torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(ns)]

            def step(k):
                i = k % ns
                o = outs[i]
                batch.ipv4_frames_multi([(txs[k % R], o[0], None), (rxs[k % R], o[1], o[2])], stream=streams[i])

            for k in range(8):
                step(k)
            torch.cuda.synchronize()
            main_s = streams[0]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for s in streams[1:]:
                s.wait_event(e0)
            for k in range(steps):
                step(k)
            for s in streams[1:]:
                ev = torch.cuda.Event()
                ev.record(s)
                main_s.wait_event(ev)
            e1.record(main_s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / steps
            print(f"round {rnd} streams {ns}: {us:7.1f} us/step  {alg / us / 1e3:7.1f} GB/s  "
                  f"{alg / us / 1e3 / 8000:.4f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
