"""Probe: bench --config slots runs slower than tools/ab_kernels.py's
udp1500_slots_verify case.  Builds pools both ways (bench: each from its own
frames with stored checksums; ab: clones of one pool) and times each pool
alone and in 20-launch chains, verify-only."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native  # noqa: E402

N, FRAME, SLOT, OFF = 1 << 20, 1500, 2304, 256


def pool_from(fr, dev):
    slots = torch.zeros(N * SLOT + 16, dtype=torch.uint8, device=dev)
    slots[: N * SLOT].view(N, SLOT)[:, OFF:OFF + FRAME] = fr.data[: N * FRAME].view(N, FRAME)
    return batch.PacketBatch(data=slots, off=torch.arange(N, device=dev, dtype=torch.int64) * SLOT + OFF,
                             length=torch.full((N,), FRAME, dtype=torch.int32, device=dev), bytes_len=N * SLOT,
                             max_len=FRAME)


def main():
    native.check(native.load().sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    sets = {}
    bench_pools = []
    for r in range(4):
        fr = devsynth.udp_frames(N, FRAME, seed=0x5EA57A2C + 3 * r, device=dev)
        fr = devsynth.store_checksums(fr, batch.ipv4_frames(fr))
        bench_pools.append(pool_from(fr, dev))
        del fr
    sets["bench_style"] = bench_pools
    fr = devsynth.udp_frames(N, FRAME, seed=8, device=dev)
    p0 = pool_from(fr, dev)
    del fr
    sets["ab_style"] = [p0] + [batch.PacketBatch(data=p0.data.clone(), off=p0.off.clone(), length=p0.length.clone(),
                                                 bytes_len=p0.bytes_len, max_len=p0.max_len) for _ in range(3)]
    torch.cuda.empty_cache()
    for name, pools in sets.items():
        pre = [batch.prepare_call("sccsum_ipv4_frames", b.data, b.bytes_len, b.off, b.length, None, st, N, FRAME)
               for b in pools]
        for p in pre:
            p(s)
        torch.cuda.synchronize()
        alone = {i: [] for i in range(4)}
        for _ in range(8):
            for i in range(4):
                pre[(i + 1) % 4](s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                pre[i](s)
                e1.record()
                torch.cuda.synchronize()
                alone[i].append(e0.elapsed_time(e1) * 1e3)
        chain = []
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(20):
                pre[k % 4](s)
            e1.record()
            torch.cuda.synchronize()
            chain.append(e0.elapsed_time(e1) * 1e3 / 20)
        print(json.dumps({"set": name, "alone_us": [round(float(np.median(alone[i])), 1) for i in range(4)],
                          "chain20_us_per_launch": round(float(np.median(chain)), 1),
                          "data_mod_2MiB": [b.data.data_ptr() % (2 << 20) for b in pools]}), flush=True)


if __name__ == "__main__":
    main()
