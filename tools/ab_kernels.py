"""In-process interleaved A/B of kernel variants (sccsum_set_kernel_variant)
on the bench workload and on mixed / long packets.  Prints one JSON line per
(case, variant) with median and min launch time and GB/s (algorithmic bytes).

--rotate R (default 4) keeps R distinct copies of each batch and launches on
them in turn, so no launch finds the previous launch's lines in the 256 MB
MALL (a back-to-back replay of ONE 1.5 GB batch lets default-policy lines
survive between launches — a replay artefact, not streaming bandwidth).

usage: python tools/ab_kernels.py [--rounds 10] [--variants 1,2]
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

from seastar_amd import batch, devsynth, native, synth  # noqa: E402


CASES: set[str] = set()


def cases(dev):
    n = 1 << 20
    tx = devsynth.udp_frames(n, 1500, seed=1, device=dev)
    yield "udp1500_frames", tx, "frames", n * (1500 + 12 + 4)
    yield "udp1500_spans", tx, "spans", n * (1500 + 12 + 2)
    yield "udp1500_frames_rss", tx, "frames_rss", n * (1500 + 12 + 4 + 4)
    if "udp1500x2_frames" in CASES:  # one launch over 2 M frames: launch ramp/tail = 2 T(1 M) - T(2 M)
        del tx
        torch.cuda.empty_cache()
        tx2 = devsynth.udp_frames(2 * n, 1500, seed=2, device=dev)
        yield "udp1500x2_frames", tx2, "frames", 2 * n * (1500 + 12 + 4)
        del tx2
    lens = synth.zipf_lengths(200_000, seed=3)
    off, total = synth.pack(lens, seed=4, max_gap=3)
    buf = np.random.default_rng(5).integers(0, 256, size=total, dtype=np.uint8)
    mb = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    yield "zipf_spans", mb, "spans", int(lens.sum()) + lens.size * 14
    del mb
    big = synth.zipf_lengths(3_400_000, seed=6)
    fb = devsynth.mixed_frames(big, seed=7, device=dev)
    yield "cfg3_zipf_frames", fb, "frames", int(big.sum()) + big.size * 16
    n64 = 16384
    seg = torch.randint(0, 256, (n64 * 65536,), dtype=torch.uint8, device=dev)
    lb = batch.PacketBatch(data=seg, off=torch.arange(n64, device=dev, dtype=torch.int64) * 65536,
                           length=torch.full((n64,), 65536, dtype=torch.int32, device=dev),
                           bytes_len=n64 * 65536, max_len=65536)
    yield "tcp64k_spans", lb, "spans", n64 * (65536 + 14)
    if "tcp65535_spans" in CASES:  # 65 535 B segments back to back: every tile starts mid-line
        ob = batch.PacketBatch(data=seg, off=torch.arange(n64, device=dev, dtype=torch.int64) * 65535,
                               length=torch.full((n64,), 65535, dtype=torch.int32, device=dev),
                               bytes_len=n64 * 65535, max_len=65535)
        yield "tcp65535_spans", ob, "spans", n64 * (65535 + 14)
        del ob
    if "udp1500_slots" in CASES:  # frames where a NIC would DMA them: DPDK mbuf slots (2304 B, data at +256)
        del lb, seg
        torch.cuda.empty_cache()
        ns = 1 << 20
        fr = devsynth.udp_frames(ns, 1500, seed=8, device=dev)
        slots = torch.zeros(ns * 2304 + 16, dtype=torch.uint8, device=dev)
        slots[: ns * 2304].view(ns, 2304)[:, 256:1756] = fr.data[: ns * 1500].view(ns, 1500)
        sb = batch.PacketBatch(data=slots, off=torch.arange(ns, device=dev, dtype=torch.int64) * 2304 + 256,
                               length=torch.full((ns,), 1500, dtype=torch.int32, device=dev),
                               bytes_len=ns * 2304, max_len=1500)
        del fr
        yield "udp1500_slots", sb, "frames", ns * (1500 + 12 + 4)
        if "udp1500_slots_verify" in CASES:  # the same, verify only (status bytes, no out2)
            yield "udp1500_slots_verify", sb, "verify", ns * (1500 + 12 + 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="1,0", help="comma list of variant[:blocks_per_cu[:U[:tile[:dyn[:tile_bytes[:tail_split[:tail_quarters[:out_policy[:short_chunks[:run_align]]]]]]]]]]")
    ap.add_argument("--rotate", type=int, default=4, help="distinct copies of each batch, launched in turn")
    ap.add_argument("--cases", default="udp1500_frames,udp1500_spans,udp1500_frames_rss,zipf_spans,cfg3_zipf_frames,"
                                       "tcp64k_spans")
    args = ap.parse_args()
    CASES.update(args.cases.split(","))
    variants = args.variants.split(",")
    lib = native.load()
    native.check(lib.sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    wanted = set(args.cases.split(","))
    for name, b, mode, alg in cases(dev):
        if name not in wanted:
            continue
        outs = {}
        times = {v: [] for v in variants}
        copies = [b] + [batch.PacketBatch(data=b.data.clone(), off=b.off.clone(), length=b.length.clone(),
                                          bytes_len=b.bytes_len, max_len=b.max_len) for _ in range(args.rotate - 1)]
        turn = [0]

        def knobs(v):
            parts = (v.split(":") + [""] * 11)[:11]
            native.check(lib.sccsum_set_kernel_variant(int(parts[0])), "variant")
            native.check(lib.sccsum_set_blocks_per_cu(int(parts[1] or 8)), "blocks_per_cu")
            native.check(lib.sccsum_set_group_units(int(parts[2] or 0)), "group_units")
            native.check(lib.sccsum_set_tile_packets(int(parts[3] or 64)), "tile_packets")
            native.check(lib.sccsum_set_dynamic_tiles(int(parts[4] or 1)), "dynamic")
            native.check(lib.sccsum_set_tile_bytes(int(parts[5] or 49152)), "tile_bytes")
            native.check(lib.sccsum_set_tail_split(int(parts[6] or 1), int(parts[7] or 4)), "tail_split")
            native.check(lib.sccsum_set_out_policy(int(parts[8] or 1)), "out_policy")
            native.check(lib.sccsum_set_short_chunks(int(parts[9] or 1)), "short_chunks")
            native.check(lib.sccsum_set_run_align(int(parts[10] or 8)), "run_align")

        st_buf = torch.empty(max(b.n, 1), dtype=torch.uint8, device=dev)

        def run(bb):
            if mode == "frames":
                return batch.ipv4_frames(bb)
            if mode == "verify":
                return batch.verify_frames(bb, st_buf)
            if mode == "frames_rss":
                return batch.ipv4_frames_rss(bb)[1]
            return batch.spans(bb)

        def run_next():
            bb = copies[turn[0] % len(copies)]
            turn[0] += 1
            return run(bb)

        for v in variants:
            knobs(v)
            outs[v] = run(copies[0]).clone()
        torch.cuda.synchronize()
        ref = outs[variants[0]]
        for v in variants[1:]:
            assert torch.equal(outs[v], ref), f"{name}: variant {v} differs from {variants[0]}"
        for _ in range(args.rounds):
            for v in variants:
                knobs(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                run_next()
                e0.record()
                for _ in range(args.reps):
                    run_next()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps)
        for v in variants:
            t = np.array(times[v])
            print(json.dumps({"case": name, "variant": v, "rotate": len(copies),
                              "median_us": round(float(np.median(t)) * 1e3, 1),
                              "min_us": round(float(t.min()) * 1e3, 1),
                              "GBps_median": round(alg / (np.median(t) / 1e3) / 1e9, 1)}), flush=True)
        del b, copies
        torch.cuda.empty_cache()
    native.check(lib.sccsum_set_kernel_variant(0), "variant")
    native.check(lib.sccsum_set_blocks_per_cu(8), "blocks_per_cu")
    native.check(lib.sccsum_set_group_units(0), "group_units")
    native.check(lib.sccsum_set_tile_packets(64), "tile_packets")
    native.check(lib.sccsum_set_dynamic_tiles(1), "dynamic")
    native.check(lib.sccsum_set_tile_bytes(49152), "tile_bytes")
    native.check(lib.sccsum_set_tail_split(1, 4), "tail_split")
    native.check(lib.sccsum_set_out_policy(1), "out_policy")
    native.check(lib.sccsum_set_short_chunks(1), "short_chunks")
    native.check(lib.sccsum_set_run_align(8), "run_align")


if __name__ == "__main__":
    main()
