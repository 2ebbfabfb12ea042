"""bench.py — device-resident Internet-checksum throughput on MI355X.

Workload (BASELINE.json configs[1], the metric's config): per GPU, a batch of
1,048,576 IPv4/UDP frames of 1500 B packed back to back in HBM behind an
offset/length array.  One step = the checksum work the native stack does on
that traffic when offload is off, both directions:
  generate: sccsum_ipv4_frames over the tx batch (checksum fields zero) ->
            IPv4 header + UDP checksums       (src/net/ip.cc:271-277, udp.cc:184-195)
  verify:   sccsum_ipv4_frames over the rx batch (checksums stored, 1 % of
            frames corrupted) -> per-frame pass/fail status (ip.cc:121-127, tcp.hh:876-883)
value = bytes checksummed by all ranks / max-over-ranks wall time, GiB/s.
Multi-GPU: one process per GPU, each with its own independent shard (weak
scaling, no data-path collective; the only collectives are the timing
barrier and the max-over-ranks reduction).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native  # noqa: E402

METRIC = "GiB/s device-resident Internet checksum, 1500B-packet batches, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
FRAME = 1500
META_BYTES = 12  # u64 offset + u32 length per packet
SEED = 0x5EA57A2C


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 20, help="frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the pre-timing parity check (A/B builds only)")
    ap.add_argument("--pmc", default=None, help="PMC summary JSON for roofline.traffic (default: newest in profiles/)")
    ap.add_argument("--rotate", type=int, default=4,
                    help="distinct batches (pairs for udp1500) launched in turn, so no launch replays cached lines")
    ap.add_argument("--config", default="udp1500", choices=["udp1500", "mixed", "tcp64k", "e2e", "fill"],
                    help="udp1500 = the metric's config (cfg 2, default); mixed = cfg 3; tcp64k = cfg 4 "
                         "(per-GPU shard); e2e = cfg 5 (pinned host mbufs, PCIe-inclusive); fill = cfg 2 tx "
                         "generate with in-place write-back (sccsum_ipv4_fill)")
    return ap.parse_args()


# The path exchanges no data between GPUs (independent shards):
# the process group only carries the timing barrier and one max-over-ranks
# reduction, so it runs on gloo (host TCP) and RCCL is never initialised.
# SCCSUM_DIST_BACKEND=nccl puts that control traffic on RCCL instead.
BACKEND = os.environ.get("SCCSUM_DIST_BACKEND", "gloo")


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = local % max(ndev, 1)
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(BACKEND)
    native.check(native.load().sccsum_init(dev), "sccsum_init")
    return world, rank, dev


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device="cuda" if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(tx, budget_s: float):
    """Oracle (C restatement of src/net/ip_checksum.cc, -O2) on a bounded
    sample of the same frames, on this host's cores: threads = cores we may
    use (capped at 16, the box's CPU share), plus the 1-thread rate."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # cpu_baseline leg only

    n_sample = min(262144, tx.n)  # 393 MB: larger than the host L3, like the real stream
    host = tx.data[: n_sample * FRAME].cpu().numpy()
    off = np.arange(n_sample, dtype=np.uint64) * FRAME
    length = np.full(n_sample, FRAME, dtype=np.uint32)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def rate(nt, seconds):
        oracle.batch_ipv4(host, off, length, nthreads=nt)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.batch_ipv4(host, off, length, nthreads=nt)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
        # generate + verify = the same checksum work twice per frame on the GPU
        # side; the CPU rate is bytes checksummed per second either way.
        return reps * n_sample * FRAME / dt / 2**30, reps

    v1, r1 = rate(1, budget_s / 2)
    vn, rn = rate(threads, budget_s / 2)
    return {
        "value": round(vn, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_sample} x {FRAME} B IPv4/UDP frames ({n_sample * FRAME / 1e6:.0f} MB) from the same batch, "
                  f"IPv4 header + UDP checksum per frame, {rn} passes on {threads} threads "
                  f"(~{budget_s / 2:.0f} s) and {r1} passes on 1 thread",
        "value_1core": round(v1, 3),
        "cpu_model": cpu_model(),
    }


def pmc_traffic(path: str | None, kernel_substr: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (see
    tools/pmc_summary.py); None when no summary exists."""
    cands = [path] if path else sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")))
    for p in reversed(cands):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel_substr)
        if k and k.get("hbm_bytes_per_launch"):
            return float(k["hbm_bytes_per_launch"]), os.path.relpath(p, REPO)
    return None, None


def timed(step, steps, warmup, world, stream, launches_per_step=1):
    """Warm up, then time `steps` calls bracketed by barrier + sync; returns
    (max-over-ranks wall seconds, mean seconds per launch).  The launch mean
    comes from ONE pair of HIP events around the timed launches on their
    stream: an event between every two launches leaves the GPU idle ~5 us at
    each (a timestamp packet), which the old per-launch events added to the
    wall time (profiles/r01_kernel_stats_bench.csv gap analysis)."""
    for k in range(warmup):
        step(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for k in range(steps):
        step(k)
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()  # this rank's end, before the closing barrier's own latency
    barrier(world)
    wall = max_over_ranks(t1 - t0, world)
    return wall, e0.elapsed_time(e1) / 1e3 / (steps * launches_per_step)


def line(metric, value, unit, args, world, wall, dtype, config, roofline=None, cpu=None, extra=None):
    d = {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
         "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
         "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic", "config": config,
         "roofline": roofline, "cpu_baseline": cpu}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def run_tcp64k(args, world, rank, dev):
    """cfg 4: 64 KiB TCP segments with pseudo-header seeds (len 65536 wraps to
    0, tcp.hh:878), this rank's independent shard of the 16 M-segment job."""
    n = args.packets if args.packets != (1 << 20) else 2 * 1024 * 1024  # 16 M / 8 GPUs per rank
    seg = 65536
    b, seeds = devsynth.tcp_segments(n, seg, seed=SEED + 104729 * rank, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    batch.spans(b, seeds=seeds, out=out)  # generate
    devsynth.store_tcp_checksums(b, out)
    batch.spans(b, seeds=seeds, out=out, status=st)  # verify: every segment must pass
    torch.cuda.synchronize()
    assert int((st != 1).sum()) == 0, "tcp64k verify failed"
    stream = torch.cuda.current_stream()
    wall, launch_s = timed(lambda k: batch.spans(b, seeds=seeds, out=out, status=st, stream=stream),
                           args.steps, args.warmup, world, stream)
    alg = n * (seg + 12 + 4 + 2 + 1)
    if rank == 0:
        line("GiB/s device-resident Internet checksum, 64 KiB TCP segments (cfg 4)",
             world * n * seg * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": "cfg4: 65536 B TCP segments + pseudo-header seed per segment, verify pass",
              "segments_per_gpu": n, "segment_bytes": seg, "parallelism": f"{world} independent shards"},
             {"bound": "hbm", "achieved": round(alg / launch_s / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(alg / launch_s / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
              "avg_launch_us": round(launch_s * 1e6, 2)})


def run_mixed(args, world, rank, dev):
    """cfg 3: Zipf(1.2) frame lengths 64..9000 B, contiguous packing (odd
    offsets), ~1.5 GB per GPU, IPv4 + UDP checksums per frame."""
    from seastar_amd import synth

    n = args.packets if args.packets != (1 << 20) else 3_400_000
    lens = synth.zipf_lengths(n, seed=SEED + rank)
    R = max(1, args.rotate)  # distinct batches launched in turn (no cached-line replay)
    bs = [devsynth.mixed_frames(lens, seed=SEED + 31 * rank + 7 * r, device=dev) for r in range(R)]
    out = torch.empty(2 * n, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream()
    wall, launch_s = timed(lambda k: batch.ipv4_frames(bs[k % R], out2=out, stream=stream), args.steps,
                           max(args.warmup, R), world, stream)
    total = int(lens.sum())
    alg = total + n * (12 + 4)
    if rank == 0:
        line("GiB/s device-resident Internet checksum, mixed-MTU Zipf batches (cfg 3)",
             world * total * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": "cfg3: Zipf(s=1.2) IPv4/UDP frames 64..9000 B, packed back to back (odd offsets)",
              "packets_per_gpu": n, "bytes_per_gpu": total, "mean_len": round(total / n, 1),
              "rotation": f"{R} distinct batches launched in turn",
              "parallelism": f"{world} independent shards"},
             {"bound": "hbm", "achieved": round(alg / launch_s / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(alg / launch_s / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
              "avg_launch_us": round(launch_s * 1e6, 2)})


def run_fill(args, world, rank, dev):
    """cfg 2 tx side with in-place write-back: IPv4 header +
    UDP checksums generated and stored into the frames (wire-ready), every
    step over the same 1 M x 1500 B batch (generate ignores the fields' old
    contents, so repeated steps are identical work)."""
    n = args.packets
    R = max(1, args.rotate)  # distinct batches launched in turn (no cached-line replay)
    bs = [devsynth.udp_frames(n, FRAME, seed=SEED + 7 * rank + 13 * r, device=dev) for r in range(R)]
    mode = native.FILL_IP | native.FILL_L4
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for b in bs:
        batch.ipv4_fill(b, mode)
        batch.ipv4_frames(b, status=st)
        torch.cuda.synchronize()
        assert args.no_check or int((st != 3).sum()) == 0, "filled frames do not verify"
    stream = torch.cuda.current_stream()
    wall, launch_s = timed(lambda k: batch.ipv4_fill(bs[k % R], mode, stream=stream), args.steps,
                           max(args.warmup, R), world, stream)
    alg = n * (FRAME + META_BYTES + 4)  # read every byte + metadata, write the two 2-byte fields
    if rank == 0:
        line("GiB/s device-resident Internet checksum, 1500B-packet batches, in-place generate (cfg 2 tx)",
             world * n * FRAME * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": "cfg2 tx: 1500 B IPv4/UDP frames, IP + UDP checksums generated and stored in place",
              "packets_per_gpu": n, "rotation": f"{R} distinct batches launched in turn",
              "parallelism": f"{world} independent shards"},
             {"bound": "hbm", "achieved": round(alg / launch_s / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(alg / launch_s / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
              "avg_launch_us": round(launch_s * 1e6, 2)})


def run_e2e(args, world, rank, dev):
    """cfg 5: frames in a pinned, DPDK-mbuf-shaped host pool (2304-B slots,
    data at +256); chunks H2D on a copy stream, kernel on a compute stream,
    results D2H, 3 chunks in flight.  A = slots copied as they lie; B =
    packets gathered into pinned staging first; C = one 2D DMA per chunk of
    each slot's packet bytes (B and C: only packet bytes cross PCIe)."""
    from seastar_amd import pipeline

    n = args.packets
    tx = devsynth.udp_frames(n, FRAME, seed=SEED + rank, device=dev)
    want = batch.ipv4_frames(tx).cpu().numpy().view(np.uint16).reshape(n, 2)
    pool = pipeline.pinned_empty(n * pipeline.MBUF_SLOT)
    pv = pool.reshape(n, pipeline.MBUF_SLOT)
    pv[:, :pipeline.MBUF_DATA_OFF] = 0
    pv[:, pipeline.MBUF_DATA_OFF:pipeline.MBUF_DATA_OFF + FRAME] = tx.data[: n * FRAME].view(n, FRAME).cpu().numpy()
    off = np.arange(n, dtype=np.uint64) * pipeline.MBUF_SLOT + pipeline.MBUF_DATA_OFF
    length = np.full(n, FRAME, dtype=np.uint32)
    del tx
    torch.cuda.empty_cache()
    res = {}
    for name, gather, chunk_bytes in (("A_slots_as_is", native.GATHER_NONE, 65536 * pipeline.MBUF_SLOT),
                                      ("B_gathered", native.GATHER_HOST, 65536 * FRAME),
                                      ("C_strided_dma", native.GATHER_STRIDED, 65536 * ((FRAME + 15) & ~15))):
        pl = pipeline.HostPipeline(dev.index or 0, chunk_bytes=chunk_bytes, chunk_packets=65536, depth=3)
        got = pl.run(native.PIPE_IPV4, pool, off, length, gather=gather, max_len=FRAME)
        assert np.array_equal(got, want), f"e2e {name} mismatch vs device-resident results"
        times = []
        for _ in range(max(1, args.steps // 4)):
            t0 = time.perf_counter()
            pl.run(native.PIPE_IPV4, pool, off, length, gather=gather, max_len=FRAME)
            times.append(time.perf_counter() - t0)
        pl.close()
        t = float(np.median(times))
        pcie = n * (pipeline.MBUF_SLOT if gather == native.GATHER_NONE else FRAME) + n * (12 + 4)
        res[name] = {"GiBps_packet_bytes": round(n * FRAME / t / 2**30, 2), "ms_per_batch": round(t * 1e3, 2),
                     "pcie_GBps_h2d_plus_d2h": round(pcie / t / 1e9, 2)}
    if rank == 0:
        best = max(res.values(), key=lambda r: r["GiBps_packet_bytes"])
        line("GiB/s Internet checksum incl. PCIe: pinned mbuf-shaped host buffers -> HBM -> host (cfg 5)",
             world * best["GiBps_packet_bytes"], "GiB/s", args, world, best["ms_per_batch"] / 1e3 * args.steps, "u8",
             {"workload": "cfg5: 1,048,576 x 1500 B IPv4/UDP frames in 2304-B mbuf slots (pinned), "
                          "H2D + kernel + D2H of 4 B/frame, 3-deep pipeline, 64Ki-frame chunks",
              "parallelism": f"{world} independent shards"}, extra={"variants": res})


def main():
    args = parse()
    world, rank, local = dist_setup()
    dev = torch.device("cuda", local)
    if args.config != "udp1500":
        {"tcp64k": run_tcp64k, "mixed": run_mixed, "e2e": run_e2e, "fill": run_fill}[args.config](args, world, rank, dev)
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
        return
    n = args.packets

    # R distinct tx/rx batch pairs launched in turn: 2R x 1.5 GB per rank, so no
    # launch finds its batch's lines left in the 256 MB MALL by an earlier one
    # (a replay of one resident batch would measure cache reuse, not streaming)
    R = max(1, args.rotate)
    txs, rxs, sts = [], [], []
    out_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    out_rx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    bad = torch.randperm(n, device=dev, generator=g)[: n // 100]
    for r in range(R):
        tx = devsynth.udp_frames(n, FRAME, seed=SEED + 7919 * rank + 104723 * r, device=dev)
        first = batch.ipv4_frames(tx, out2=out_tx)
        rx = devsynth.store_checksums(tx, first)
        devsynth.corrupt(rx, bad, byte=700)
        txs.append(tx)
        rxs.append(rx)
        sts.append(torch.empty(n, dtype=torch.uint8, device=dev))
    tx = txs[0]
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()

    def step(k):
        r = k % R
        batch.ipv4_frames(txs[r], out2=out_tx, stream=stream)
        batch.ipv4_frames(rxs[r], out2=out_rx, status=sts[r], stream=stream)

    for k in range(max(args.warmup, R)):
        step(k)
    torch.cuda.synchronize()
    # sanity: every uncorrupted rx frame verifies, every corrupted one fails
    for st_rx in sts:
        n_fail = int(((st_rx & 2) == 0).sum())
        assert n_fail == bad.numel(), f"verify failures {n_fail} != corrupted {bad.numel()}"

    # timed region: barrier + sync on both sides, one HIP event pair around the
    # launches on their stream (see timed())
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e_start.record(stream)
    for k in range(args.steps):
        step(k)
    e_end.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0  # this rank's end, before the closing barrier's own latency
    barrier(world)
    wall_max = max_over_ranks(wall, world)
    avg_launch_s = e_start.elapsed_time(e_end) / 1e3 / (2 * args.steps)

    bytes_per_step = 2 * n * FRAME  # per rank
    value = world * bytes_per_step * args.steps / wall_max / 2**30
    alg_bytes_launch = n * (FRAME + META_BYTES + 4) + n // 2  # + status byte on the rx launch (avg)
    achieved = alg_bytes_launch / avg_launch_s / 1e9

    # measured HBM read ceiling with the same load shape over the tx bytes
    sink = torch.zeros(native.load().sccsum_read_probe_blocks(), dtype=torch.int64, device=dev)
    for _ in range(3):
        batch.read_probe(tx.data, tx.bytes_len, sink=sink, stream=stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    reps = 10
    for _ in range(reps):
        batch.read_probe(tx.data, tx.bytes_len, sink=sink, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ceiling = (tx.bytes_len & ~15) * reps / (e0.elapsed_time(e1) / 1e3) / 1e9

    traffic, traffic_src = pmc_traffic(args.pmc, "csum_flat_kernel")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(tx, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": "cfg2: 1,048,576 x 1500 B IPv4/UDP frames per GPU in HBM (offset/length array); "
                            "step = generate (IP+UDP csum) + verify (1% corrupted) pass",
                "packets_per_gpu": n,
                "frame_bytes": FRAME,
                "rotation": f"{R} distinct tx/rx batch pairs launched in turn ({2 * R * n * FRAME / 1e9:.1f} GB per GPU)",
                "global_batch": n * world,
                "parallelism": f"{world} independent shards, no collective",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "csum_flat_kernel<16,true,false,false,nt> (sccsum_ipv4_frames)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": alg_bytes_launch,
                "avg_launch_us": round(avg_launch_s * 1e6, 2),
                "measured_read_ceiling_GBps": round(ceiling, 1),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
