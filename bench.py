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
barrier and the max-over-ranks reduction, on gloo).  Under torchrun the ranks
come from the environment; `python bench.py --gpus N` without it starts the N
rank processes itself (launch_ranks).

Other configs (--config): mixed = cfg 3, tcp64k = cfg 4 (one GPU's shard),
fill = cfg 2 tx with in-place write-back, e2e = cfg 5 (PCIe-inclusive, pinned
mbuf-shaped host buffers), sweep = device-resident rate against batch size at
the reference's batch boundaries.

Every kernel-timed line carries "roofline" with "trace_select": which
dispatches of which kernel in this process were the timed ones, so
tools/prof_timed.py can cut exactly those out of a rocprofv3 kernel trace (or
a PMC pass) of the same command.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "GiB/s device-resident Internet checksum, 1500B-packet batches, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
FRAME = 1500
META_BYTES = 12  # u64 offset + u32 length per packet
SEED = 0x5EA57A2C


def flat_kernel(ipv4: bool, fill: bool, n: int, nbytes: int) -> str:
    """The flat-kernel instantiation the library's default picks (sccsum.hip
    launch(): U = 16 for >= 512 Ki packets and >= 256 MiB, else U = 8 with
    the next chunk in flight), as rocprofv3 names it."""
    big = n >= (512 << 10) and nbytes >= (256 << 20)
    u, pipe = (16, "false") if big else (8, "true")
    # the chunk-in-flight (U = 8) form reads its claims back late for packets of 1 KiB+ in 256 MiB+ (PLATE)
    plate = not big and nbytes // max(n, 1) >= 1024 and nbytes >= (256 << 20)
    return f"csum_flat_kernel<{u}, {str(ipv4).lower()}, {str(fill).lower()}, {pipe}, {str(plate).lower()}>"


def sparse_kernel(args, ipv4: bool, max_len: int) -> str:
    """The kernel a sparse layout gets (sccsum.hip pick_variant / launch_rows),
    as rocprofv3 names it: the row kernel, V units per lane from max_len."""
    units = (max_len + 30) // 16
    v = 2 if units <= 32 else 4 if units <= 64 else 6 if units <= 96 else 8
    return f"csum_row_kernel<{v}, {str(ipv4).lower()}, false, false>"  # (MQ, FILL: one batch, no fill)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps (~0.1 s of cfg 2): the timed region's fixed cost (first launch, closing
    # sync, ~100 us) is then 0.1 % of it instead of 1 % (profiles/r02_ab_steps.log)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 20, help="frames per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the pre-timing parity check (A/B builds only)")
    ap.add_argument("--pmc", default=None, help="PMC summary JSON for roofline.traffic (default: newest for the config)")
    ap.add_argument("--rotate", type=int, default=4,
                    help="distinct batches (pairs for udp1500) launched in turn, so no launch replays cached lines")
    ap.add_argument("--config", default="udp1500",
                    choices=["udp1500", "mixed", "tcp64k", "e2e", "fill", "sweep", "slots", "frags"],
                    help="udp1500 = the metric's config (cfg 2, default); mixed = cfg 3; tcp64k = cfg 4 "
                         "(per-GPU shard); e2e = cfg 5 (pinned host mbufs, PCIe-inclusive); fill = cfg 2 tx "
                         "generate with in-place write-back (sccsum_ipv4_fill); sweep = rate against batch size; "
                         "slots = cfg 2 frames in DPDK-mbuf-shaped slots in HBM (a sparse layout); frags = 9000 B "
                         "jumbo packets as 5-fragment mbuf chains in HBM (checksummer::sum(const packet&))")
    ap.add_argument("--tile-bytes", type=int, default=None, help="A/B: flat-kernel tile target (sccsum_diag.h)")
    ap.add_argument("--tile-packets", type=int, default=None,
                    help="A/B: flat-kernel packets-per-tile cap, <= 64 (sccsum_set_tile_packets)")
    ap.add_argument("--variant", type=int, default=None, help="A/B: kernel form (sccsum_set_kernel_variant)")
    ap.add_argument("--blocks-per-cu", type=int, default=None,
                    help="A/B: grid cap in workgroups per CU (sccsum_set_blocks_per_cu)")
    ap.add_argument("--out-policy", type=int, default=None,
                    help="A/B: cache policy of the flat kernel's result stores (sccsum_set_out_policy)")
    ap.add_argument("--engine-in-flight", type=int, default=8,
                    help="--launch engine: steps published ahead of the grid (max_in_flight)")
    ap.add_argument("--engine-sync", type=int, default=None,
                    help="A/B: --launch engine steps re-synchronise the grid every k steps (the step waits for "
                         "the one before it; sccsum_set_engine_sync_every)")
    ap.add_argument("--engine-wt", type=int, default=None,
                    help="A/B: engine result stores written through (1) or stored as a launch does (0) "
                         "(sccsum_set_engine_write_through)")
    ap.add_argument("--fill-single-max", type=int, default=None,
                    help="A/B: in-place fills of at most this many frames run in one pass (sccsum_set_fill_single_max)")
    ap.add_argument("--run-align", type=int, default=None, help="A/B: run-start alignment in units (sccsum_set_run_align)")
    ap.add_argument("--sync", default="auto", choices=["auto", "spin", "yield"],
                    help="how the host thread waits on the device (hipSetDeviceFlags schedule)")
    ap.add_argument("--seg-len", type=int, default=65536, help="tcp64k: segment bytes (65536, or 65535: odd offsets)")
    ap.add_argument("--align", type=int, default=1, help="mixed: frame start alignment (1 = packed, SURVEY §8(d) (i); "
                                                         "64 = layout (ii))")
    ap.add_argument("--streams", type=int, default=1,
                    help="udp1500 / mixed / fill: step k launches on stream k %% S (A/B: with 2, consecutive steps' "
                         "launches run concurrently)")
    ap.add_argument("--launch", default=None, choices=["multi", "single", "engine"],
                    help="udp1500 / mixed: engine (the default) = one resident grid per timed run, the steps "
                         "submitted into it as they go, at most --engine-in-flight in flight, the grid "
                         "re-synchronised every 10 steps (sccsum_engine_*, DESIGN.md §5.11; fill: "
                         "sccsum_engine_submit_fill, not its default); multi = one sccsum_ipv4_frames_multi "
                         "launch per step over the tx and rx batches (udp1500's launch form, and its default with "
                         "--share-devices); single = one sccsum_ipv4_frames launch per batch (mixed: the rx batch "
                         "only, mixed's launch form)")
    ap.add_argument("--rx-out2", action="store_true",
                    help="udp1500 / mixed: the verify (rx) half — mixed's single form: its one batch — also writes "
                         "both checksums per frame (default: status bits only, what the reference's verify keeps: "
                         "ip.cc:121-127, tcp.hh:876-883)")
    ap.add_argument("--dry-run", action="store_true",
                    help="multi-rank plumbing only: launch, rendezvous, barrier, max-over-ranks, one line; "
                         "no device call (the CPU test of the launcher)")
    ap.add_argument("--share-devices", action="store_true",
                    help="allow more ranks than visible GPUs (ranks then share devices: local %% ndev); "
                         "refused without it")
    ap.add_argument("--numa", default="bind", choices=["bind", "preferred", "none", "off"],
                    help="rank locality, as Seastar pins shards and binds their memory (reactor.cc:4163, "
                         "memory.cc:1898-1951): every thread onto the GPU's NUMA node's CPUs, and the host "
                         "memory policy MPOL_BIND (bind) / MPOL_PREFERRED (preferred) to that node, or CPUs only "
                         "(none); off = leave the rank where the OS put it")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without a torch.distributed launcher: start
    N rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, one GPU each), wait for all and return the worst exit code.
    This process never touches HIP (nothing has imported torch yet) and never
    execs: the ranks are children.  Rank 0 prints the JSON line on the shared
    stdout.  Reference analogue: one independent engine per shard,
    src/net/net.cc:309-341."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("GLOO_SOCKET_IFNAME", "lo")  # one node: the control plane stays on loopback
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    # wait for all; if a rank fails, the others would wait at the next barrier
    # until gloo's timeout: stop them (these exact children) and report it
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or (128 - code if code < 0 else code)  # a signal -s reads as 128 + s
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def _imports():
    """torch and the engine are imported only in a rank process (the
    multi-rank launcher must not touch HIP before it starts the ranks)."""
    global np, torch, batch, devsynth, native
    import numpy as np
    import torch

    from seastar_amd import batch, devsynth, native


# The path exchanges no data between GPUs (independent shards):
# the process group only carries the timing barrier and one max-over-ranks
# reduction, so it runs on gloo (host TCP) and RCCL is never initialised.
# SCCSUM_DIST_BACKEND=nccl puts that control traffic on RCCL instead.
BACKEND = os.environ.get("SCCSUM_DIST_BACKEND", "gloo")


SYNC_MODE = "auto"
_SCHEDULE = {"auto": 0, "spin": 1, "yield": 2}  # hipDeviceScheduleAuto / Spin / Yield (hip_runtime_api.h)


def set_sync_mode(dev: int, mode: str) -> None:
    """How this rank's host thread waits on its device.  "spin" polls, as
    Seastar's reactor polls its queues (include/seastar/core/internal/poll.hh:26-29);
    HIP's "auto" yields the core while the GPU works, unless contexts outnumber
    the logical CPUs.  Set before the device's context exists."""
    if mode == "auto":
        return
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    for rc, what in ((hip.hipSetDevice(ctypes.c_int(dev)), "hipSetDevice"),
                     (hip.hipSetDeviceFlags(ctypes.c_uint(_SCHEDULE[mode])), "hipSetDeviceFlags")):
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc})")


NUMA = {}  # this rank's locality (seastar_amd.numa.bind), reported in per_rank


def place_rank(bdf, mode: str) -> dict:
    """Bind this rank to its GPU's NUMA node (every thread onto the node's
    schedulable CPUs; host memory policy per --numa) before any host buffer
    of the run is allocated: the pinned mbuf pool, burst staging and the CPU
    baseline's sample then sit on the GPU's node, as Seastar binds a shard's
    memory to its core's node (src/core/memory.cc:1898-1951)."""
    from seastar_amd import numa

    sysfs = os.environ.get("SCCSUM_SYSFS", numa.SYSFS)  # a fake tree in the launcher test
    p = numa.plan(bdf, sysfs=sysfs)
    if mode == "off":
        return {"numa_node": p["numa_node"], "cpus": numa.format_cpulist(sorted(os.sched_getaffinity(0))),
                "ncpus": len(os.sched_getaffinity(0)), "affinity": "unchanged (--numa off)", "mempolicy": "default",
                "reason": "--numa off"}
    return numa.bind(p, mem="none" if mode == "none" else mode)


def check_devices(world_local: int, ndev: int, share: bool) -> None:
    """More ranks on this node than visible GPUs would silently stack ranks on
    one device (local % ndev): refuse unless --share-devices asks for it."""
    if world_local > ndev and not share:
        sys.exit(f"bench.py: {world_local} ranks on this node but {ndev} visible GPU(s); "
                 "pass --share-devices to let ranks share devices")


def dist_setup(dry_run=False, args=None):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    share = bool(args and args.share_devices)
    numa_mode = args.numa if args else "bind"
    if world > 1 and os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
        # one node (the driver's torchrun uses --master-addr 127.0.0.1): keep gloo's control traffic on
        # loopback rather than on whatever interface the box's hostname resolves to
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if dry_run:
        # the launcher test's stand-ins for the GPUs: PCI ids (one per local rank) and device count
        bdfs = [b for b in os.environ.get("SCCSUM_DRY_RUN_BDFS", "").split(",") if b]
        ndev_dry = int(os.environ.get("SCCSUM_DRY_RUN_NDEV", str(max(len(bdfs), local_world))))
        check_devices(local_world, ndev_dry, share)
        DRY_DEVICE.update(device=local % max(ndev_dry, 1), pci_bus_id=bdfs[local % len(bdfs)] if bdfs else None)
        NUMA.update(place_rank(bdfs[local % len(bdfs)] if bdfs else None, numa_mode))
        if world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo")
        return world, rank, local
    ndev = torch.cuda.device_count()
    check_devices(local_world, ndev, share)
    dev = local % max(ndev, 1)
    set_sync_mode(dev, SYNC_MODE)
    torch.cuda.set_device(dev)
    NUMA.update(place_rank(device_id(torch.device("cuda", dev))["pci_bus_id"], numa_mode))
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


def cpu_threads() -> tuple[int, str]:
    """Host threads for the CPU baseline: the cores this process may run on,
    capped by OMP_NUM_THREADS when the environment sets it (the GPU box sets
    16 = its CPU share per GPU; os.cpu_count() there shows the whole host)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), f"OMP_NUM_THREADS={omp} (of {aff} schedulable)"
    return aff, f"{aff} schedulable cores"


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
    sample of the same frames, shard-per-core as Seastar runs it (SURVEY
    §8(d)): one thread per PHYSICAL core, each pinned to its core (smp::pin,
    src/core/reactor.cc:4163), on the rank's CPUs — the GPU's NUMA node after
    place_rank — up to the box's CPU share (cpu_threads: OMP_NUM_THREADS).
    The cores are taken round robin over the node's L3 domains (CCDs): a CCD's
    link to memory caps what its cores stream together, so 16 threads packed
    on 2 CCDs measure the links, not the cores.  Also measured: 1 thread, a
    1/2/4/8 curve, and one CCD fully loaded (its link's ceiling), from which
    the all-cores figure is projected.  The sample is allocated after
    place_rank, so it sits on the GPU's node too."""
    from seastar_amd import numa

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # cpu_baseline leg only

    n_sample = min(262144, tx.n)  # 393 MB: larger than the host L3, like the real stream
    host = tx.data[: n_sample * FRAME].cpu().numpy()
    off = np.arange(n_sample, dtype=np.uint64) * FRAME
    length = np.full(n_sample, FRAME, dtype=np.uint32)
    share, why = cpu_threads()
    cores = numa.physical_cores(sorted(os.sched_getaffinity(0)))  # one hardware thread per physical core
    spread = numa.spread_over_l3(cores)
    pinned = spread[:share]
    threads = len(pinned)
    doms = numa.l3_domains(cores)
    one_ccd = max(doms.values(), key=len)[:share] if doms else pinned

    def rate(cpus, seconds):
        oracle.batch_ipv4(host, off, length, cpus=cpus)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.batch_ipv4(host, off, length, cpus=cpus)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
        # generate + verify = the same checksum work twice per frame on the GPU
        # side; the CPU rate is bytes checksummed per second either way.
        return reps * n_sample * FRAME / dt / 2**30, reps

    v1, r1 = rate(pinned[:1], budget_s * 0.25)
    curve = {}
    for k in (2, 4, 8):
        if k < threads:
            curve[str(k)] = round(rate(pinned[:k], budget_s * 0.07)[0], 3)
    vccd = rate(one_ccd, budget_s * 0.1)[0] if len(one_ccd) > 1 else None
    vn, rn = rate(pinned, budget_s * 0.4)
    host_cores, host_ccds = numa.host_physical_cores(), numa.host_l3_domains()
    node = NUMA.get("numa_node", -1)
    per_core = vn / max(threads, 1)
    per_ccd = vccd if vccd else per_core * max(len(one_ccd), 1)
    cands = [per_core * host_cores] + ([per_ccd * host_ccds] if host_ccds else [])
    # never below what the pinned threads measured (with every host core pinned, the projection is that run)
    all_cores = max(min(cands), vn) if host_cores else None
    return {
        "value": round(vn, 3),
        "unit": "GiB/s",
        "cores": threads,
        "cores_source": f"one thread per physical core, pinned, spread over the L3 domains of the rank's CPUs "
                        f"({NUMA.get('cpus')}, NUMA node {node}), up to the box's CPU share: {why}",
        "kind": "port",
        "sample": f"{n_sample} x {FRAME} B IPv4/UDP frames ({n_sample * FRAME / 1e6:.0f} MB, allocated on the rank's "
                  f"node) from the same batch, IPv4 header + UDP checksum per frame, {rn} passes on {threads} pinned "
                  f"threads and {r1} passes on 1",
        "value_1core": round(v1, 3),
        "scaling_GiBps": {"1": round(v1, 3), **curve, str(threads): round(vn, 3)},
        "pinned_cpus": numa.format_cpulist(pinned),
        "one_l3_domain": {"cpus": numa.format_cpulist(one_ccd), "GiBps": round(vccd, 3) if vccd else None},
        "physical_cores": {"host": host_cores, "schedulable": len(cores), "l3_domains_host": host_ccds,
                           "node": len(numa.physical_cores(numa.node_cpus(node))) if node >= 0 else None},
        # the whole host is not this run's to use (the box's CPU share is `share` threads): the
        # all-cores figure is projected from the measured rates — per physical core x the host's cores,
        # capped by one loaded L3 domain's rate x the host's domains; host DRAM bandwidth (not
        # measured) may cap it lower still
        "value_all_cores": round(all_cores, 3) if all_cores else None,
        "value_all_cores_kind": (f"projected: min({per_core:.2f} GiB/s per physical core x {host_cores} cores, "
                                 f"{per_ccd:.1f} GiB/s per loaded L3 domain x {host_ccds} domains); "
                                 "not run on all cores, DRAM bandwidth not applied"),
        "cpu_model": cpu_model(),
    }


def pmc_traffic(path: str | None, config: str, kernel: str):
    """(HBM bytes, algorithmic bytes) per launch of `kernel` from the newest
    committed rocprofv3 PMC summary for this config (tools/prof_timed.py:
    profiles/rNN_pmc_<config>.json), and its path; Nones when none exists."""
    cands = [path] if path else sorted(glob.glob(os.path.join(REPO, "profiles", f"*pmc_{config}.json")))
    for p in reversed(cands):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and k.get("hbm_bytes_per_launch"):
            return float(k["hbm_bytes_per_launch"]), k.get("alg_bytes_per_launch"), os.path.relpath(p, REPO)
    return None, None, None


def fill_floor(alg_bytes: float, fill_s: float):
    """The in-place fill's measured two-pass floor: the
    newest committed profiles/rNN_fill_floor.json, from tools/dev/store_probe.hip
    run on a GPU box — a plain nt read of 1 M x 1500 B frames followed by the
    cheapest field-writing pass measured (the aligned 64-byte line read and
    rewritten, `rd;st64rw`), and the register-stash form beside it.  A fill
    cannot beat a read of every byte plus a pass that writes the fields
    (DESIGN.md §5.6), so frac against this floor, not only against 8 TB/s, says
    how much of the fill's gap is the kernel's.  None when no file exists."""
    for p in reversed(sorted(glob.glob(os.path.join(REPO, "profiles", "*fill_floor.json")))):
        try:
            d = json.load(open(p))
            us = float(d["rd_st64rw_us"])
        except (OSError, ValueError, KeyError):
            continue
        return {"us_per_fill": us, "frac": round(alg_bytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                "fill_over_floor": round(fill_s * 1e6 / us, 4),
                "form": "plain nt read of the frames, then a pass rewriting each frame's aligned 64-byte head line "
                        "(tools/dev/store_probe.hip rd;st64rw: the cheapest two-pass form measured)",
                "register_stash_us": d.get("rdbar_lineR_us"), "read_only_us": d.get("rd_us"),
                "source": os.path.relpath(p, REPO), "box": d.get("box")}
    return None


class Launches:
    """Counts this process's launches per kernel, so a line can name which
    dispatches were timed (trace_select)."""

    def __init__(self):
        self.n = {}

    def add(self, kernel: str, k: int = 1):
        self.n[kernel] = self.n.get(kernel, 0) + k

    def select(self, kernel: str, count: int) -> dict:
        return {"kernel": kernel, "skip": self.n.get(kernel, 0), "count": count}


LAUNCHES = Launches()


def default_launch(args, launches: str) -> str:
    """cfg 2 and cfg 3 run through the resident engine by default (round 5):
    with the grid re-synchronised every 10 big steps (sccsum.hip engine_put)
    it beats one launch per step by 2.0-2.9 % on the same box
    (profiles/r05_engine_sync.log).  Ranks that share a device (--share-devices)
    use launches: one engine grid holds every CU of its device."""
    return launches if args.share_devices else "engine"


def launch_form(args) -> str:
    """The launch form a config's timed run uses (per_rank's "launch": an
    N-GPU line says what each rank ran)."""
    if args.config == "udp1500":
        return args.launch or default_launch(args, "multi")
    if args.config == "mixed":
        return args.launch or default_launch(args, "single")
    if args.config == "fill":
        return "engine" if args.launch == "engine" else "single"
    return {"tcp64k": "single", "slots": "single", "frags": "single", "e2e": "pipeline", "sweep": "sweep"}[args.config]


def make_streams(args, dev):
    """The step's launch streams: step k goes to streams[k % S].  Default 1 =
    the current stream, one launch at a time, so a launch's duration is the
    step's.  With 2 (A/B only), consecutive steps' launches run concurrently
    over their whole length — +2-3 % on the read-only passes, -8 % on the
    in-place fill (profiles/r02_ab_bench_streams.log) — and a kernel's trace
    duration is no longer its share of the step."""
    ns = args.streams
    if ns <= 1:
        return [torch.cuda.current_stream(dev)]
    return [torch.cuda.Stream(device=dev) for _ in range(ns)]


OWN = {}  # this rank's own timing of the last timed() region (per_rank diagnostics)


def timed(step, steps, warmup, world, streams, begin=None, end=None, between=None):
    """Warm up, then time `steps` calls bracketed by barrier + sync; returns
    (max-over-ranks wall seconds, seconds per step from ONE pair of HIP events
    around the timed launches: the start event on streams[0], which every other
    stream waits on, the end event on streams[0] after it has waited on every
    other stream).  An event between every two launches leaves the GPU idle
    ~5 us at each (a timestamp packet), which per-launch events would add to
    the wall time.  between(): called after the warm-up, before
    the timed region (outside it): e.g. poisoning outputs the timed steps must
    rewrite, so a check afterwards sees that they ran."""
    import gc

    streams = streams if isinstance(streams, (list, tuple)) else [streams]
    s0 = streams[0]
    torch.cuda.synchronize()  # inputs built on the default stream are complete before any step stream reads them
    # no collector pauses inside the step loops: a full collection (tens of ms with torch loaded) would
    # starve a resident engine, which holds only max_in_flight steps of work ahead of the host
    gc.collect()
    gc.disable()
    try:
        return _timed(step, steps, warmup, world, streams, s0, begin, end, between)
    finally:
        gc.enable()


def _timed(step, steps, warmup, world, streams, s0, begin, end, between):
    if warmup:
        if begin:  # (--launch engine: a run of its own)
            begin()
        for k in range(warmup):
            step(k)
        if end:
            end()
    torch.cuda.synchronize()
    if between:
        between()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(s0)
    for s in streams[1:]:
        s.wait_event(e0)
    if begin:  # --launch engine: the grid's launch (and its counters' reset) is inside the timed region
        begin()
    for k in range(warmup, warmup + steps):
        step(k)
    if end:
        end()
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        s0.wait_event(ev)
    e1.record(s0)
    torch.cuda.synchronize()
    t1 = time.perf_counter()  # this rank's end, before the closing barrier's own latency
    barrier(world)
    wall = max_over_ranks(t1 - t0, world)
    OWN.update(wall_s=t1 - t0, step_s=e0.elapsed_time(e1) / 1e3 / steps)
    return wall, e0.elapsed_time(e1) / 1e3 / steps


DRY_DEVICE = {}  # --dry-run: the stand-in device index and PCI address of this rank


def device_id(dev) -> dict:
    """Which GPU a rank ran on: its index and PCI address (so a slow device
    or box shows up by name in a multi-GPU line)."""
    if dev is None:
        return {"device": DRY_DEVICE.get("device"), "pci_bus_id": DRY_DEVICE.get("pci_bus_id")}
    p = torch.cuda.get_device_properties(dev)
    return {"device": dev.index, "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0",
            "device_name": p.name}


def per_rank(world, rank, dev, **fields):
    """Every rank's own figures — device, wall time, rate, average launch,
    read ceiling — gathered on rank 0 with one all_gather_object, so an N > 1
    line shows a slow rank or device beside the max-over-ranks `value`
    (reference analogue: independent per-shard engines, src/net/net.cc:309-341).
    Collective: every rank calls it."""
    me = {"rank": rank, "host": socket.gethostname(), **device_id(dev),
          "numa_node": NUMA.get("numa_node"), "cpus": NUMA.get("cpus"), "affinity": NUMA.get("affinity"),
          "mempolicy": NUMA.get("mempolicy"),
          **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in fields.items()}}
    if world == 1:
        return [me]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, me)
    check_distinct_devices(out, SHARE_DEVICES)
    return out


SHARE_DEVICES = False  # --share-devices


def check_distinct_devices(pr, share: bool) -> None:
    """Every rank on a device of its own: no two ranks of one host on the same
    device index or PCI address, unless --share-devices asked for sharing
    (a rank -> device mapping that stacked ranks on device 0
    would pass every other check).  Every rank holds the gathered list, so
    all of them stop together."""
    if share:
        return
    seen_dev, seen_bdf = {}, {}
    for r in pr:
        for key, seen in (((r["host"], r["device"]), seen_dev), ((r["host"], r["pci_bus_id"]), seen_bdf)):
            if key[1] is None:
                continue
            if key in seen:
                sys.exit(f"bench.py: ranks {seen[key]} and {r['rank']} share {key} without --share-devices")
            seen[key] = r["rank"]


def rank_rate(nbytes_per_step, steps):
    """This rank's own GiB/s and launch figures from its last timed() region."""
    return {"wall_s": OWN["wall_s"], "GiBps": nbytes_per_step * steps / OWN["wall_s"] / 2**30,
            "ms_per_step": OWN["wall_s"] / steps * 1e3}


def roofline(alg_bytes_launch: float, launch_s: float, config: str, kernel: str, sel: dict, args, extra=None):
    traffic, prof_alg, src = pmc_traffic(args.pmc, config, "csum_flat_kernel")
    scaled = None
    if traffic is not None and prof_alg and abs(prof_alg - alg_bytes_launch) > 0.001 * alg_bytes_launch:
        # the profile's launch had another size (a shorter batch, or the 65 535 B variant): its
        # traffic per algorithmic byte, applied to this launch's algorithmic bytes
        scaled = {"profile_alg_bytes_per_launch": int(prof_alg), "profile_hbm_bytes_per_launch": traffic}
        traffic = round(traffic / prof_alg * alg_bytes_launch, 1)
    achieved = alg_bytes_launch / launch_s / 1e9
    d = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": src,
         "alg_bytes_per_launch": int(alg_bytes_launch), "avg_launch_us": round(launch_s * 1e6, 2),
         "trace_select": sel}
    if scaled:
        d["traffic_scaled_from"] = scaled
    if extra:
        d.update(extra)
    return d


def layout_traffic(alg_bytes: float, gap_bytes: int, packet_bytes: int, frac: float) -> dict:
    """What a layout's gaps cost: frames placed at 64 B
    boundaries leave gap bytes between them that the stream reads with the
    frames (memory moves whole lines; a gap is never wider than the line
    holding its frame's end).  The bytes a launch streams are the algorithmic
    bytes plus the gaps, so the line's frac, divided by the traffic ratio,
    is not kernel loss: frac x ratio is the rate per byte actually streamed,
    the figure to compare with the packed layout's frac."""
    ratio = (alg_bytes + gap_bytes) / alg_bytes if alg_bytes else 1.0
    return {"gap_bytes": int(gap_bytes), "gap_per_packet_byte": round(gap_bytes / packet_bytes, 5) if packet_bytes else 0.0,
            "traffic_ratio": round(ratio, 5), "frac_of_streamed_bytes": round(frac * ratio, 4),
            "note": "layout (ii)'s ceiling is the packed layout's frac / traffic_ratio: the gaps are read, "
                    "not counted"}


def emit(metric, value, unit, args, world, wall, dtype, config, roof=None, cpu=None, extra=None):
    d = {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
         "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
         "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
         "config": dict(config, host_wait=SYNC_MODE), "roofline": roof, "cpu_baseline": cpu}
    # which library ran, and its ABI (an A/B line against an older build, SCCSUM_LIB + SCCSUM_ABI_ANY, may
    # have other semantics: ADVICE r03)
    lib = native.load()
    d["library"] = {"path": os.path.relpath(os.environ.get("SCCSUM_LIB", native.LIB_PATH), REPO),
                    "abi_version": int(lib.sccsum_abi_version())}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def read_ceiling(data, nbytes, stream, reps=10):
    """Measured HBM read ceiling: the plain nt stream over the same bytes."""
    sink = torch.zeros(native.load().sccsum_read_probe_blocks(), dtype=torch.int64, device=data.device)
    for _ in range(3):
        batch.read_probe(data, nbytes, sink=sink, stream=stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        batch.read_probe(data, nbytes, sink=sink, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    return (nbytes & ~15) * reps / (e0.elapsed_time(e1) / 1e3) / 1e9


def run_udp1500(args, world, rank, dev):
    n = args.packets
    args.launch = args.launch or default_launch(args, "multi")
    # R distinct tx/rx batch pairs launched in turn: 2R x 1.5 GB per rank, so no
    # launch finds its batch's lines left in the 256 MB MALL by an earlier one
    # (a replay of one resident batch would measure cache reuse, not streaming)
    R = max(1, args.rotate)
    kern = flat_kernel(True, False, n, n * FRAME)
    txs, rxs, sts = [], [], []
    streams = make_streams(args, dev)
    if R % len(streams):  # a batch (and its status buffer) must always come back to the same stream
        streams = streams[:1]
    ns = len(streams)
    # one result buffer pair per rotation (a rotation always comes back to the same stream), so the
    # timed run's outputs of every rotation can be checked against the warm-up's afterwards
    outs = [(torch.empty(2 * n, dtype=torch.int16, device=dev), torch.empty(2 * n, dtype=torch.int16, device=dev))
            for _ in range(R)]
    out_tx = outs[0][0]
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    bad = torch.randperm(n, device=dev, generator=g)[: n // 100]
    for r in range(R):
        tx = devsynth.udp_frames(n, FRAME, seed=SEED + 7919 * rank + 104723 * r, device=dev)
        first = batch.ipv4_frames(tx, out2=out_tx)
        LAUNCHES.add(flat_kernel(True, False, n, n * FRAME))
        rx = devsynth.store_checksums(tx, first)
        devsynth.corrupt(rx, bad, byte=700)
        txs.append(tx)
        rxs.append(rx)
        sts.append(torch.empty(n, dtype=torch.uint8, device=dev))
    multi = args.launch == "multi"
    engine = args.launch == "engine"
    per_step = 1 if (multi or engine) else 2  # launches per step
    if multi:  # the tx and rx batches of a step form ONE launch of 2 * n frames
        kern = flat_kernel(True, False, 2 * n, 2 * n * FRAME)
    if engine:  # one resident grid per run; each step (tx + rx batch) submitted into it
        kern = "csum_engine_kernel<16, true, false>"
        streams = streams[:1]
        ns = 1

    # multi: each (rotation, stream) pair's launch is prebuilt, so a step only
    # crosses the C-ABI (no per-step Python argument marshalling)
    pre = {}
    if multi:
        for r in range(R):
            o_tx, o_rx = outs[r]
            pre[r] = batch.prepare_ipv4_frames_multi([(txs[r], o_tx, None),
                                                      (rxs[r], o_rx if args.rx_out2 else None, sts[r])])

    warm = max(args.warmup, R)
    eng = begin = end = None
    if engine:
        eng = batch.Engine(dev.index or 0, frames=True, ring_slots=1024, max_in_flight=args.engine_in_flight)
        pre = {r: eng.prepare([(txs[r], outs[r][0], None), (rxs[r], outs[r][1] if args.rx_out2 else None, sts[r])])
               for r in range(R)}

        def begin():
            eng.start(streams[0])

        def end():
            eng.finish()  # stops the grid (it leaves once its steps are done), then waits on the run's last step (a give-up raises)

    def step(k):
        r = k % R
        s = streams[k % ns]
        if engine:
            eng.submit_prepared(pre[r])
        elif multi:
            pre[r](s)
        else:
            batch.ipv4_frames(txs[r], out2=outs[r][0], stream=s)
            batch.ipv4_frames(rxs[r], out2=outs[r][1], status=sts[r], stream=s)

    torch.cuda.synchronize()  # the batches were built on the default stream
    if begin:
        begin()
    for k in range(warm):
        step(k)
    if end:
        end()
    LAUNCHES.add(kern, 1 if engine else per_step * warm)
    torch.cuda.synchronize()
    # sanity: every uncorrupted rx frame verifies, every corrupted one fails; the tx outputs match the generate pass
    for st_rx in sts:
        n_fail = int(((st_rx & 2) == 0).sum())
        assert args.no_check or n_fail == bad.numel(), f"verify failures {n_fail} != corrupted {bad.numel()}"
    # the warm-up's results per rotation; the timed run's are checked against them afterwards (VERDICT r05:
    # the timed region itself was never checked), its outputs poisoned first so that a step that never ran
    # shows: 0xFFFF is no IPv4 or UDP checksum of these frames (~fold(sum) is 0xFFFF only for a zero sum)
    want_tx = [o[0].clone() for o in outs]
    want_st = [s.clone() for s in sts]
    ran = sorted({k % R for k in range(warm, warm + args.steps)})

    def poison():
        for r in ran:
            outs[r][0].fill_(-1)
            sts[r].fill_(0xEE)

    LAUNCHES.add(kern, 1 if engine else per_step * warm)  # the warm-up timed() runs again first
    sel = LAUNCHES.select(kern, 1 if engine else per_step * args.steps)
    # the warm-up again, right before the timed region: the checks above leave the GPU idle for
    # milliseconds, and a run that starts cold pays for it (+50 us after a 20 ms gap, +175 us after
    # 100 ms: profiles/r06_run_cost.log)
    wall, step_s = timed(step, args.steps, warm, world, streams, begin, end, between=None if args.no_check else poison)
    LAUNCHES.add(kern, 1 if engine else per_step * args.steps)
    avg_launch_s = step_s / per_step
    stream = streams[0]
    if engine:
        eng.close()  # raises if the run left a published step undone (sccsum_engine_destroy)
    if not args.no_check:  # outside the timed region
        torch.cuda.synchronize()
        for r in ran:
            n_fail = int(((sts[r] & 2) == 0).sum())
            assert n_fail == bad.numel(), f"timed run, rotation {r}: verify failures {n_fail} != {bad.numel()}"
            assert torch.equal(sts[r], want_st[r]), f"timed run, rotation {r}: rx status differs from the warm-up's"
            assert torch.equal(outs[r][0], want_tx[r]), f"timed run, rotation {r}: tx checksums differ from the warm-up's"

    value = world * 2 * n * FRAME * args.steps / wall / 2**30
    # per launch: every frame byte + 12 B metadata + the results written: tx 4 B (IP, UDP checksums), rx 1 B
    # of status bits (+ 4 B with --rx-out2; --launch single always writes both)
    rx_out = 4 if (args.rx_out2 or not (multi or engine)) else 0
    alg = (n * (FRAME + META_BYTES + 4) + n * (FRAME + META_BYTES + 1 + rx_out)) // per_step
    roof_alg, roof_s = alg, avg_launch_s
    if engine:  # the launch is the run: every step's bytes over the run's time (the same ratio)
        roof_alg, roof_s = alg * args.steps, avg_launch_s * args.steps
    ceiling = read_ceiling(txs[0].data, txs[0].bytes_len, stream)
    ranks = per_rank(world, rank, dev, **rank_rate(2 * n * FRAME, args.steps), avg_launch_us=avg_launch_s * 1e6,
                     read_ceiling_GBps=ceiling, frac=alg / avg_launch_s / 1e9 / HBM_PEAK_GBPS, launch=args.launch)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(txs[0], args.cpu_seconds)
    if rank == 0:
        emit(METRIC, value, "GiB/s", args, world, wall, "u8",
             {"workload": "cfg2: 1,048,576 x 1500 B IPv4/UDP frames per GPU in HBM (offset/length array); "
                          "step = generate (IP+UDP csum) + verify (1% corrupted) pass",
              "packets_per_gpu": n, "frame_bytes": FRAME,
              "launch": ("one sccsum_ipv4_frames_multi launch per step over the tx and rx batches" if multi
                         else ("one resident engine grid per timed run (sccsum_engine_*): each step's tx and rx "
                               f"batches submitted into it as one step, at most {args.engine_in_flight} steps in flight" if engine
                               else "one sccsum_ipv4_frames launch per batch (2 per step)")),
              "rotation": f"{R} distinct tx/rx batch pairs launched in turn ({2 * R * n * FRAME / 1e9:.1f} GB per GPU)",
              "timed_run_checked": (None if args.no_check else
                                    "after the timed region: every rotation's rx status and tx checksums equal the "
                                    "warm-up's (outputs poisoned before it), failures == corrupted frames"
                                    + ("; the run waited on its last step and its engine closed clean" if engine
                                       else "")),
              "streams": f"{ns} (step k on stream k % {ns})",
              "global_batch": n * world, "parallelism": f"{world} independent shards, no collective"},
             roofline(roof_alg, roof_s, "udp1500" if not engine else "udp1500_engine",
                      kern + (" (sccsum_ipv4_frames_multi, tx + rx)" if multi else
                              (" (sccsum_engine_*, tx + rx per step; one launch = the timed run)" if engine
                               else " (sccsum_ipv4_frames)")), sel, args,
                      {"measured_read_ceiling_GBps": round(ceiling, 1)}), cpu, extra={"per_rank": ranks})


def run_tcp64k(args, world, rank, dev):
    """cfg 4: 64 KiB TCP segments with pseudo-header seeds (len 65536 wraps to
    0, tcp.hh:878), this rank's independent shard of the 16 M-segment job."""
    n = args.packets if args.packets != (1 << 20) else 2 * 1024 * 1024  # 16 M / 8 GPUs per rank
    seg = args.seg_len  # 65536 (pseudo-header len wraps to 0), or the 65535 B variant of SURVEY §8(d)
    b, seeds = devsynth.tcp_segments(n, seg, seed=SEED + 104729 * rank, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    batch.spans(b, seeds=seeds, out=out)  # generate
    devsynth.store_tcp_checksums(b, out)
    batch.spans(b, seeds=seeds, out=out, status=st)  # verify: every segment must pass
    kern = flat_kernel(False, False, n, b.bytes_len)
    LAUNCHES.add(kern, 2)
    torch.cuda.synchronize()
    assert args.no_check or int((st != 1).sum()) == 0, "tcp64k verify failed"
    stream = torch.cuda.current_stream()
    LAUNCHES.add(kern, args.warmup)
    sel = LAUNCHES.select(kern, args.steps)
    pre = batch.prepare_call("sccsum_spans", b.data, b.bytes_len, b.off, b.length, seeds, out, st, b.n, b.max_len)
    wall, launch_s = timed(lambda k: pre(stream), args.steps, args.warmup, world, stream)
    alg = n * (seg + META_BYTES + 4 + 2 + 1)  # + seed in, result + status out
    cbytes = min(b.bytes_len, 16 << 30)
    ceiling = read_ceiling(b.data, cbytes, stream, reps=3)
    ranks = per_rank(world, rank, dev, **rank_rate(n * seg, args.steps), avg_launch_us=launch_s * 1e6,
                     read_ceiling_GBps=ceiling, frac=alg / launch_s / 1e9 / HBM_PEAK_GBPS)
    if rank == 0:
        emit("GiB/s device-resident Internet checksum, 64 KiB TCP segments (cfg 4)",
             world * n * seg * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": f"cfg4: {seg} B TCP segments + pseudo-header seed per segment, verify pass",
              "segments_per_gpu": n, "segment_bytes": seg, "parallelism": f"{world} independent shards"},
             roofline(alg, launch_s, "tcp64k" if seg == 65536 else f"tcp64k_seg{seg}", kern + " (sccsum_spans)",
                      sel, args, {"measured_read_ceiling_GBps": round(ceiling, 1), "read_ceiling_bytes": cbytes}),
             extra={"per_rank": ranks})


def run_mixed(args, world, rank, dev):
    """cfg 3: Zipf(1.2) frame lengths 64..9000 B, contiguous packing (odd
    offsets), ~1.5 GB per batch, IPv4 + UDP checksums per frame.  A step is
    one sccsum_ipv4_frames launch over an rx batch (checksums stored in place
    by sccsum_ipv4_fill; --launch single, the default), or, like cfg 2, both
    directions in one sccsum_ipv4_frames_multi launch: generate over a tx
    batch (checksum fields zero) plus verify-only over the rx batch (its own
    Zipf draw) (--launch multi; 1-2 % slower on three boxes), or the single
    form's steps submitted into one resident engine grid (--launch engine)."""
    from seastar_amd import synth

    n = args.packets if args.packets != (1 << 20) else 3_400_000
    args.launch = args.launch or default_launch(args, "single")
    multi = args.launch == "multi"
    engine = args.launch == "engine"
    # the verify step writes the status byte alone, what the reference's verify keeps (ip.cc:121-127:
    # drop when get() != 0); --rx-out2 adds both checksums (2-3.6 % slower: profiles/r05_cfg3_terms.log)
    vonly = not multi and not args.rx_out2
    lens = synth.zipf_lengths(n, seed=SEED + rank)
    lens_rx = synth.zipf_lengths(n, seed=SEED + 7717 + rank) if multi else lens
    R = max(1, args.rotate)  # distinct batches launched in turn (no cached-line replay)
    align = max(1, args.align)
    rxs = [devsynth.mixed_frames(lens_rx, seed=SEED + 31 * rank + 7 * r, device=dev, align=align) for r in range(R)]
    txs = ([devsynth.mixed_frames(lens, seed=SEED + 131 * rank + 17 * r + 5, device=dev, align=align)
            for r in range(R)] if multi else [])
    streams = make_streams(args, dev)
    if R % len(streams) or engine:  # a batch (and its status buffer) must always come back to the same stream
        streams = streams[:1]
    ns = len(streams)
    stream = streams[0]
    outs = [(torch.empty(2 * n, dtype=torch.int16, device=dev), torch.empty(2 * n, dtype=torch.int16, device=dev))
            for _ in range(ns)]
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    for rx, st in zip(rxs, sts):  # rx: checksums stored, so every frame verifies
        batch.ipv4_fill(rx, native.FILL_IP | native.FILL_L4, out2=outs[0][0])  # (out2: older A/B builds need it)
        if multi:
            batch.ipv4_frames(rx, out2=outs[0][1], status=st)
            LAUNCHES.add(flat_kernel(True, False, n, rx.bytes_len))
    LAUNCHES.add(flat_kernel(True, True, n, rxs[0].bytes_len), R)
    torch.cuda.synchronize()
    if multi:
        for st in sts:
            assert int((st != 3).sum()) == 0, "mixed rx frames do not verify"
    total = int(lens.sum()) + (int(lens_rx.sum()) if multi else 0)
    nbytes = total  # packet bytes checksummed per step
    if multi:
        kern = flat_kernel(True, False, 2 * n, rxs[0].bytes_len + txs[0].bytes_len)
        pre = {(r, i): batch.prepare_ipv4_frames_multi([(txs[r], outs[i][0], None),
                                                        (rxs[r], outs[i][1] if args.rx_out2 else None, sts[r])])
               for r in range(R) for i in range(ns)}
    else:
        kern = flat_kernel(True, False, n, rxs[0].bytes_len)
        # prebuilt launches: a step only crosses the C-ABI (--verify-only: status bits, no out2)
        pre = {(r, i): batch.prepare_call("sccsum_ipv4_frames", rxs[r].data, rxs[r].bytes_len, rxs[r].off,
                                          rxs[r].length, None if vonly else outs[i][1], sts[r] if vonly else None,
                                          rxs[r].n, rxs[r].max_len)
               for r in range(R) for i in range(ns)}
    warm = max(args.warmup, R)
    step, begin, end, eng = (lambda k: pre[(k % R, k % ns)](streams[k % ns])), None, None, None
    if engine:  # the single form's steps, submitted into one resident grid per run
        kern = "csum_engine_kernel<16, true, false>"
        eng = batch.Engine(dev.index or 0, frames=True, ring_slots=1024, max_in_flight=args.engine_in_flight)
        pre_e = {r: eng.prepare([(rxs[r], None, sts[r]) if vonly else (rxs[r], outs[0][1], None)]) for r in range(R)}

        def step(k):
            eng.submit_prepared(pre_e[k % R])

        def begin():
            eng.start(streams[0])

        end = eng.finish  # stops the grid (it leaves once its steps are done), then waits on the run's last step (a give-up raises)
    LAUNCHES.add(kern, 1 if engine else warm)
    sel = LAUNCHES.select(kern, 1 if engine else args.steps)
    # the timed run's statuses are checked afterwards (every frame verifies): poisoned before it, so
    # a step that never ran shows (the single form's status-only steps)
    ran = sorted({k % R for k in range(warm, warm + args.steps)})
    check_st = vonly and not args.no_check

    def poison():
        for r in ran:
            sts[r].fill_(0xEE)

    wall, launch_s = timed(step, args.steps, warm, world, streams, begin, end, between=poison if check_st else None)
    if engine:
        eng.close()  # raises if the run left a published step undone
    if check_st:
        torch.cuda.synchronize()
        for r in ran:
            assert int((sts[r] != 3).sum()) == 0, f"timed run, rotation {r}: frames that do not verify"
    # per launch: every frame byte + 12 B metadata + the results: 4 B per frame, except a multi step's rx
    # half, which writes 1 B of status bits (+ 4 B with --rx-out2)
    alg = (total + n * (META_BYTES + 4) + n * (META_BYTES + 1 + (4 if args.rx_out2 else 0)) if multi
           else total + n * (META_BYTES + (1 if vonly else 4)))
    roof_alg, roof_s = alg, launch_s
    if engine:  # the launch is the run: every step's bytes over the run's time (the same ratio)
        roof_alg, roof_s = alg * args.steps, launch_s * args.steps
    ceiling = read_ceiling(rxs[0].data, rxs[0].bytes_len, stream)
    ranks = per_rank(world, rank, dev, **rank_rate(nbytes, args.steps), avg_launch_us=launch_s * 1e6,
                     read_ceiling_GBps=ceiling, frac=alg / launch_s / 1e9 / HBM_PEAK_GBPS, launch=args.launch)
    # the gap bytes a step's batches hold between their frames (--align 64: layout (ii))
    gap = (rxs[0].bytes_len + (txs[0].bytes_len if multi else 0)) - total
    lay = layout_traffic(alg, gap, total, alg / launch_s / 1e9 / HBM_PEAK_GBPS)
    if rank == 0:
        emit("GiB/s device-resident Internet checksum, mixed-MTU Zipf batches (cfg 3)",
             world * nbytes * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": ("cfg3: Zipf(s=1.2) IPv4/UDP frames 64..9000 B, packed back to back (odd offsets)" if align == 1
                           else f"cfg3 (ii): Zipf(s=1.2) IPv4/UDP frames 64..9000 B, each at a {align} B boundary")
                          + ("; step = generate over a tx batch + verify over an rx batch" if multi
                             else ("; step = verify over one batch, status bits only" if vonly
                                   else "; step = verify over one batch (both checksums written)")),
              "packets_per_gpu": (2 * n if multi else n), "bytes_per_gpu": total,
              "mean_len": round(total / (2 * n if multi else n), 1),
              "launch": ("one sccsum_ipv4_frames_multi launch per step over the tx and rx batches" if multi
                         else (f"one resident engine grid per timed run (sccsum_engine_*): each step's batch "
                               f"submitted into it, at most {args.engine_in_flight} steps in flight" if engine
                               else "one sccsum_ipv4_frames launch per step")),
              "rotation": f"{R} distinct batch {'pairs' if multi else 'sets'} launched in turn",
              "streams": f"{ns} (step k on stream k % {ns})", "parallelism": f"{world} independent shards"},
             roofline(roof_alg, roof_s, ("mixed" if align == 1 else f"mixed_align{align}") + ("_engine" if engine else ""),
                      kern + (" (sccsum_ipv4_frames_multi, tx + rx)" if multi else
                              (" (sccsum_engine_*; one launch = the timed run)" if engine
                               else " (sccsum_ipv4_frames)")), sel, args,
                      {"measured_read_ceiling_GBps": round(ceiling, 1), "layout_traffic": lay}),
             extra={"per_rank": ranks})


def run_slots(args, world, rank, dev):
    """cfg 2's 1500 B frames where a NIC DMAs them: one per DPDK-mbuf-shaped
    slot in HBM (2304 B: 128 B rte_mbuf + 128 B headroom + 2048 B data room,
    frame at +256, src/net/dpdk.cc:139-156) — the device-resident form of
    cfg 5's pool.  A sparse layout (each frame its own run), which the library
    hands to the row kernel.  Step = verify over one batch of
    1 M slots, R rotated batches."""
    n = args.packets
    R = max(1, args.rotate)
    slot, data_off = 2304, 256
    bs = []
    for r in range(R):
        fr = devsynth.udp_frames(n, FRAME, seed=SEED + 17 * rank + 3 * r, device=dev)
        first = batch.ipv4_frames(fr)
        fr = devsynth.store_checksums(fr, first)
        slots = torch.zeros(n * slot + 16, dtype=torch.uint8, device=dev)
        slots[: n * slot].view(n, slot)[:, data_off:data_off + FRAME] = fr.data[: n * FRAME].view(n, FRAME)
        del fr, first
        bs.append(batch.PacketBatch(data=slots, off=torch.arange(n, device=dev, dtype=torch.int64) * slot + data_off,
                                    length=torch.full((n,), FRAME, dtype=torch.int32, device=dev),
                                    bytes_len=n * slot, max_len=FRAME))
    LAUNCHES.add(flat_kernel(True, False, n, n * FRAME), 2 * R)  # the frames were built packed
    torch.cuda.empty_cache()
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for b in bs:  # every frame verifies (checksums stored before the scatter into slots)
        batch.verify_frames(b, st)
        torch.cuda.synchronize()
        assert int((st != 3).sum()) == 0, "slot frames do not verify"
    kern = sparse_kernel(args, True, FRAME)
    LAUNCHES.add(kern, R)
    stream = torch.cuda.current_stream()
    warm = max(args.warmup, R)
    LAUNCHES.add(kern, warm)
    sel = LAUNCHES.select(kern, args.steps)
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    pre = {r: batch.prepare_call("sccsum_ipv4_frames", bs[r].data, bs[r].bytes_len, bs[r].off, bs[r].length, None,
                                 sts[r], n, FRAME) for r in range(R)}
    wall, launch_s = timed(lambda k: pre[k % R](stream), args.steps, warm, world, stream)
    alg = n * (FRAME + META_BYTES + 1)  # frame bytes + metadata + 1 status byte (verify only)
    ranks = per_rank(world, rank, dev, **rank_rate(n * FRAME, args.steps), avg_launch_us=launch_s * 1e6,
                     frac=alg / launch_s / 1e9 / HBM_PEAK_GBPS)
    if rank == 0:
        emit("GiB/s device-resident Internet checksum, 1500 B frames in mbuf-shaped slots (sparse layout)",
             world * n * FRAME * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": f"{n} x 1500 B IPv4/UDP frames, one per 2304 B mbuf-shaped slot in HBM (frame at +256), "
                          "verify only (status bits)",
              "packets_per_gpu": n, "rotation": f"{R} distinct batches launched in turn",
              "parallelism": f"{world} independent shards"},
             roofline(alg, launch_s, "slots", kern + " (sccsum_ipv4_frames, sparse layout -> row kernel)", sel, args),
             extra={"per_rank": ranks})


def run_frags(args, world, rank, dev):
    """SURVEY §8(f)1 at device-resident scale: checksummer::sum(const packet&)
    (src/net/ip_checksum.cc:64-68) over 9000 B jumbo packets held as DPDK
    multi-segment mbuf chains (src/net/dpdk.cc:2040-2057): fragments of 2048,
    2048, 2048, 2048 and 808 B, each in its own 2304 B mbuf slot (data room at
    +256) in HBM, with a pseudo-header seed per packet.  Step = one
    sccsum_fragments call (the fragments' raw sums, then their combination with
    the odd-offset byte swap); R rotated slot pools.  Also timed: the
    fragment-list kernel (sccsum_spans_desc) over the same fragments."""
    n = args.packets if args.packets != (1 << 20) else 174_763  # ~1.57 GB of packet bytes
    R = max(1, args.rotate)
    pkt, slot, data_off = 9000, 2304, 256
    fl = [2048, 2048, 2048, 2048, 808]
    nf = len(fl)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    frag_len = torch.tensor(fl * n, dtype=torch.int32, device=dev)
    frag_off = torch.arange(n * nf, device=dev, dtype=torch.int64) * slot + data_off
    first = torch.arange(n + 1, device=dev, dtype=torch.int32) * nf
    seeds = torch.randint(0, 65536, (n,), dtype=torch.int32, device=dev, generator=g)
    pools = [devsynth.random_bytes(n * nf * slot + 16, g, dev) for _ in range(R)]
    ws = torch.empty(int(native.load().sccsum_fragments_workspace(n * nf)), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    # parity: a sample of packets gathered contiguously on the device and summed as spans
    k = min(n, 4096)
    want = []
    for pool in pools:
        got = batch.fragments(pool, n * nf * slot, frag_off, frag_len, first, seeds=seeds, max_frag_len=2048)
        parts = [pool[i * slot + data_off:i * slot + data_off + fl[i % nf]] for i in range(k * nf)]
        contig = batch.PacketBatch(data=torch.cat(parts + [torch.zeros(16, dtype=torch.uint8, device=dev)]),
                                   off=torch.arange(k, device=dev, dtype=torch.int64) * pkt,
                                   length=torch.full((k,), pkt, dtype=torch.int32, device=dev),
                                   bytes_len=k * pkt, max_len=pkt)
        ref = batch.spans(contig, seeds=seeds[:k])  # (a small launch: the same row-kernel form, counted below)
        torch.cuda.synchronize()
        assert torch.equal(got[:k], ref), "fragment lists differ from the contiguous packets"
        want.append(got.clone())
    kern = sparse_kernel(args, False, 2048)  # the raw pass over the fragments (a sparse layout)
    LAUNCHES.add(kern, 2 * R)  # + the contiguous check launches (<= 65 536 packets: the row kernel, V 8 too)
    stream = torch.cuda.current_stream()
    pre = [batch.prepare_call("sccsum_fragments", pools[r], n * nf * slot, frag_off, frag_len, n * nf, first, seeds,
                              out, None, n, 2048, ws) for r in range(R)]
    warm = max(args.warmup, R)
    LAUNCHES.add(kern, warm)
    sel = LAUNCHES.select(kern, args.steps)
    wall, launch_s = timed(lambda k_: pre[k_ % R](stream), args.steps, warm, world, stream)
    own = rank_rate(n * pkt, args.steps)
    # the same fragments through the fragment-list kernel (one wave per packet, fragments where they lie)
    desc = []
    for pool in pools:
        src = (pool.data_ptr() + frag_off).cpu().numpy().astype(np.uint64)
        dst = (torch.arange(n, device=dev, dtype=torch.int64).repeat_interleave(nf) * pkt +
               torch.tensor([0, 2048, 4096, 6144, 8192] * n, device=dev)).cpu().numpy()
        desc.append(torch.from_numpy(batch.make_desc(src, dst, np.array(fl * n)).view(np.uint8)).to(dev))
    poff = torch.arange(n, device=dev, dtype=torch.int64) * pkt
    plen = torch.full((n,), pkt, dtype=torch.int32, device=dev)
    for r in range(R):
        d_out = batch.spans_desc(desc[r], first, poff, plen, pkt, seeds=seeds)
        torch.cuda.synchronize()
        assert torch.equal(d_out, want[r]), "fragment-list kernel differs from sccsum_fragments"
    pre_d = [batch.prepare_call("sccsum_spans_desc", desc[r], first, poff, plen, seeds, None, out, None, n, pkt)
             for r in range(R)]
    _, desc_s = timed(lambda k_: pre_d[k_ % R](stream), max(4, args.steps // 2), R, world, stream)
    alg = n * (pkt + nf * 12 + 4 + 4 + 2)  # packet bytes + fragment (offset, length) + first + seed + result
    ranks = per_rank(world, rank, dev, **own, avg_launch_us=launch_s * 1e6, frac=alg / launch_s / 1e9 / HBM_PEAK_GBPS)
    if rank == 0:
        emit("GiB/s device-resident Internet checksum, 9000 B jumbo packets as 5-fragment mbuf chains (f1)",
             world * n * pkt * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": f"{n} x 9000 B packets, each as mbuf fragments of 2048/2048/2048/2048/808 B in 2304 B slots "
                          "in HBM, pseudo-header seed per packet; step = one sccsum_fragments call",
              "packets_per_gpu": n, "rotation": f"{R} distinct slot pools launched in turn",
              "parallelism": f"{world} independent shards"},
             roofline(alg, launch_s, "frags", kern + " + frag_combine_kernel (sccsum_fragments)", sel, args,
                      {"trace_select_extra": [{"kernel": "frag_combine_kernel", "skip": sel["skip"],
                                               "count": sel["count"]}]}),
             extra={"per_rank": ranks, "fragment_list_kernel": {"us_per_call": round(desc_s * 1e6, 2),
                                             "GiBps_packet_bytes": round(n * pkt / desc_s / 2**30, 1),
                                             "note": "sccsum_spans_desc over the same HBM fragments"}})


def run_fill(args, world, rank, dev):
    """cfg 2 tx side with in-place write-back: IPv4 header +
    UDP checksums generated and stored into the frames (wire-ready), over R
    rotated 1 M x 1500 B batches (generate ignores the fields' old contents,
    so repeated steps are identical work).  A step is one sccsum_ipv4_fill
    call (generate launch + store launch; --launch single, the default) or one
    fill submitted into a resident engine grid per timed run (--launch engine:
    sccsum_engine_submit_fill, a generate step and the store step that waits
    for it)."""
    n = args.packets
    R = max(1, args.rotate)
    engine = args.launch == "engine"
    bs = [devsynth.udp_frames(n, FRAME, seed=SEED + 7 * rank + 13 * r, device=dev) for r in range(R)]
    mode = native.FILL_IP | native.FILL_L4
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for b in bs:
        batch.ipv4_fill(b, mode)
        batch.ipv4_frames(b, status=st)
        torch.cuda.synchronize()
        assert args.no_check or int((st != 3).sum()) == 0, "filled frames do not verify"
    kern = flat_kernel(True, True, n, n * FRAME)
    LAUNCHES.add(kern, R)
    streams = make_streams(args, dev)
    if R % len(streams) or engine:  # a batch filled in place must always come back to the same stream
        streams = streams[:1]
    ns = len(streams)
    warm = max(args.warmup, R)
    # prebuilt launches; the caller's out2 (the values stored) carries the generate pass's
    # words to the store pass, so no per-call scratch allocation is timed
    outs2 = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(ns)]
    begin = end = eng = None
    if engine:  # one resident grid per timed run; each step = one fill (generate step + store step)
        kern = "csum_engine_kernel<16, true, true>"
        eng = batch.Engine(dev.index or 0, frames=True, fill=True, ring_slots=1024,
                           max_in_flight=max(2, args.engine_in_flight))
        # one out2 per batch: a fill's store step reads its generate step's values from out2 while
        # the next fills run (sccsum.h: no other step may write a fill's d_out until it is done)
        outs2 = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(R)]
        pre_e = {r: eng.prepare([(bs[r], outs2[r], None)], fill_mode=mode) for r in range(R)}

        def step(k):
            eng.submit_prepared(pre_e[k % R])

        def begin():
            eng.start(streams[0])

        end = eng.finish  # stops the grid (it leaves once its steps are done), then waits on the run's last step (a give-up raises)
    else:
        pre = {(r, i): batch.prepare_call("sccsum_ipv4_fill", bs[r].data, bs[r].bytes_len, bs[r].off,
                                          bs[r].length, outs2[i], None, bs[r].n, bs[r].max_len, mode)
               for r in range(R) for i in range(ns)}

        def step(k):
            pre[(k % R, k % ns)](streams[k % ns])
    LAUNCHES.add(kern, 1 if engine else warm)
    sel = LAUNCHES.select(kern, 1 if engine else args.steps)
    # the fields the timed fills must write are cleared before the timed region (outside it), so the check
    # after it sees that every fill ran: a cleared frame does not verify
    ran = sorted({k % R for k in range(warm, warm + args.steps)})

    def clear_fields():
        for r in ran:
            fv = bs[r].data[: n * FRAME].view(n, FRAME)
            fv[:, 10:12] = 0  # IPv4 header checksum
            fv[:, 26:28] = 0  # UDP checksum (20-byte header + 6)

    wall, launch_s = timed(step, args.steps, warm, world, streams, begin, end,
                           between=None if args.no_check else clear_fields)
    if engine:
        eng.close()  # raises if the run left a published step undone
    if not args.no_check:  # outside the timed region: every timed fill stored its fields
        for r in ran:
            batch.ipv4_frames(bs[r], status=st)
            torch.cuda.synchronize()
            assert int((st != 3).sum()) == 0, f"timed run, rotation {r}: filled frames do not verify"
    alg = n * (FRAME + META_BYTES + 4)  # read every byte + metadata, write the two 2-byte fields
    roof_alg, roof_s = alg, launch_s
    if engine:  # the launch is the run: every step's bytes over the run's time (the same ratio)
        roof_alg, roof_s = alg * args.steps, launch_s * args.steps
    ranks = per_rank(world, rank, dev, **rank_rate(n * FRAME, args.steps), avg_launch_us=launch_s * 1e6,
                     frac=alg / launch_s / 1e9 / HBM_PEAK_GBPS, launch=launch_form(args))
    if rank == 0:
        emit("GiB/s device-resident Internet checksum, 1500B-packet batches, in-place generate (cfg 2 tx)",
             world * n * FRAME * args.steps / wall / 2**30, "GiB/s", args, world, wall, "u8",
             {"workload": "cfg2 tx: 1500 B IPv4/UDP frames, IP + UDP checksums generated and stored in place",
              "packets_per_gpu": n, "rotation": f"{R} distinct batches launched in turn",
              "launch": (f"one resident engine grid per timed run (sccsum_engine_submit_fill): each step's fill "
                         f"= a generate step + the store step that waits for it, at most "
                         f"{max(2, args.engine_in_flight)} steps in flight" if engine
                         else "one sccsum_ipv4_fill call per step (generate launch + store launch)"),
              "streams": f"{ns} (step k on stream k % {ns})", "parallelism": f"{world} independent shards"},
             roofline(roof_alg, roof_s, "fill_engine" if engine else "fill",
                      kern + (" (sccsum_engine_submit_fill: generate + store steps; one launch = the timed run)"
                              if engine else " + fill_store_kernel (sccsum_ipv4_fill: generate pass, "
                                             "then the field-store pass)"), sel, args,
                      dict({"floor": fill_floor(alg, launch_s)},
                           **({} if engine else {"trace_select_extra": [{"kernel": "fill_store_kernel",
                                                                         "skip": sel["skip"],
                                                                         "count": sel["count"]}]}))),
             extra={"per_rank": ranks})


def run_sweep(args, world, rank, dev):
    """Device-resident rate against batch size, at the reference's batch
    boundaries: 32-packet DPDK rx bursts (src/net/dpdk.cc:2190-2204), <= 128-
    packet tx refills (src/net/net.cc:81-105), the burst queue's 1 Ki / 16 Ki
    batches, up to 1 M.  Each size launches back to back over distinct slices
    of a 1.5 GB batch (no slice is reread while cached), eager and as one
    captured HIP graph of the same launches."""
    n_all = 1 << 20
    big = devsynth.udp_frames(n_all, FRAME, seed=SEED + rank, device=dev)
    sizes = [32, 128, 1024, 16384, 65536, 262144, 1048576]
    stream = torch.cuda.Stream(device=dev)
    res = []
    for B in sizes:
        nb = n_all // B
        k = min(nb, max(8, (64 << 20) // (B * FRAME)))  # launches per timed pass: >= 64 MB or all slices
        slices = [batch.PacketBatch(data=big.data[j * B * FRAME:], off=big.off[:B], length=big.length[:B],
                                    bytes_len=B * FRAME, max_len=FRAME) for j in range(nb)]
        out = torch.empty(2 * B, dtype=torch.int16, device=dev)
        st = torch.empty(B, dtype=torch.uint8, device=dev)
        for j in range(min(nb, 4)):
            batch.ipv4_frames(slices[j], out2=out, status=st, stream=stream)
        torch.cuda.synchronize()
        # eager: k launches, rotating over the slices (prebuilt: each launch only crosses the C-ABI)
        pre = [batch.prepare_call("sccsum_ipv4_frames", slices[j].data, B * FRAME, slices[j].off, slices[j].length,
                                  out, st, B, FRAME) for j in range(min(nb, k))]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for j in range(k):
            pre[j % len(pre)](stream)
        e1.record(stream)
        torch.cuda.synchronize()
        host_s = time.perf_counter() - t0
        eager_s = e0.elapsed_time(e1) / 1e3 / k
        # graph: the same k launches captured once, replayed
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for j in range(k):
                batch.ipv4_frames(slices[j % nb], out2=out, status=st, stream=stream)
        reps = 3
        with torch.cuda.stream(stream):  # replay() launches on the current stream
            g.replay()
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(reps):
                g.replay()
            e1.record(stream)
        torch.cuda.synchronize()
        graph_s = e0.elapsed_time(e1) / 1e3 / (reps * k)
        # 16 queues per launch (sccsum_ipv4_frames_multi): 16 slices of B packets each
        km = max(1, k // 16)
        outs16 = [torch.empty(2 * B, dtype=torch.int16, device=dev) for _ in range(16)]
        sts16 = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(16)]
        batch.ipv4_frames_multi([(slices[q % nb], outs16[q], sts16[q]) for q in range(16)], stream=stream)
        torch.cuda.synchronize()
        gm = torch.cuda.CUDAGraph()  # captured, so the host's Python cost per call is not on the clock
        with torch.cuda.graph(gm, stream=stream):
            for j in range(km):
                batch.ipv4_frames_multi([(slices[(16 * j + q) % nb], outs16[q], sts16[q]) for q in range(16)],
                                        stream=stream)
        with torch.cuda.stream(stream):
            gm.replay()
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(3):
                gm.replay()
            e1.record(stream)
        torch.cuda.synchronize()
        multi_s = e0.elapsed_time(e1) / 1e3 / (3 * km)
        del gm
        bytes_b = B * FRAME
        res.append({"packets": B, "bytes": bytes_b, "launches": k,
                    "multi16_us_per_launch": round(multi_s * 1e6, 2),
                    "multi16_GiBps": round(16 * bytes_b / multi_s / 2**30, 1),
                    "eager_us": round(eager_s * 1e6, 2), "eager_GiBps": round(bytes_b / eager_s / 2**30, 1),
                    "eager_host_us_per_launch": round(host_s / k * 1e6, 2),
                    "graph_us": round(graph_s * 1e6, 2), "graph_GiBps": round(bytes_b / graph_s / 2**30, 1),
                    "graph_frac_of_8TBps": round(B * (FRAME + META_BYTES + 5) / graph_s / 1e9 / HBM_PEAK_GBPS, 4)})
        del g, slices
    if rank == 0:
        best = res[-1]
        emit("GiB/s device-resident Internet checksum vs batch size (1500 B frames, verify pass)",
             best["graph_GiBps"] * world, "GiB/s", args, world, best["graph_us"] / 1e6 * args.steps, "u8",
             {"workload": "sweep: 1500 B IPv4/UDP frames, one sccsum_ipv4_frames per batch, batch = "
                          + "/".join(str(s) for s in sizes) + " packets",
              "parallelism": f"{world} independent shards"}, extra={"sweep": res})


def run_e2e(args, world, rank, dev):
    """cfg 5: frames in a pinned, DPDK-mbuf-shaped host pool (2304-B slots,
    data at +256); chunks H2D on a copy stream, kernel on a compute stream,
    results D2H, 3 chunks in flight.  A = slots copied as they lie; B =
    packets gathered into pinned staging first; C = one 2D DMA per chunk of
    each slot's packet bytes; D = no copies: the fragment-list kernel reads
    each packet in place over PCIe and writes results to pinned staging (B, C
    and D: only packet bytes cross PCIe)."""
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
    res, own_rates = {}, {}
    for name, gather, chunk_bytes in (("A_slots_as_is", native.GATHER_NONE, 65536 * pipeline.MBUF_SLOT),
                                      ("B_gathered", native.GATHER_HOST, 65536 * FRAME),
                                      ("C_strided_dma", native.GATHER_STRIDED, 65536 * ((FRAME + 15) & ~15)),
                                      ("D_zero_copy", native.GATHER_ZERO_COPY, 65536 * FRAME)):
        pl = pipeline.HostPipeline(dev.index or 0, chunk_bytes=chunk_bytes, chunk_packets=65536, depth=3)
        got = pl.run(native.PIPE_IPV4, pool, off, length, gather=gather, max_len=FRAME)
        assert np.array_equal(got, want), f"e2e {name} mismatch vs device-resident results"
        times, own = [], []
        for _ in range(max(1, args.steps // 4)):
            barrier(world)  # every rank's batch crosses its own PCIe link at the same time
            t0 = time.perf_counter()
            pl.run(native.PIPE_IPV4, pool, off, length, gather=gather, max_len=FRAME)
            own.append(time.perf_counter() - t0)
            times.append(max_over_ranks(own[-1], world))
        pl.close()
        t = float(np.median(times))  # median over runs of the slowest rank's time
        h2d, d2h = e2e_pcie_bytes(n, gather)
        res[name] = {"GiBps_packet_bytes": round(n * FRAME / t / 2**30, 2), "ms_per_batch": round(t * 1e3, 2),
                     "pcie_GBps_h2d_plus_d2h": round((h2d + d2h) / t / 1e9, 2)}
        to = float(np.median(own))
        own_rates[name] = {"GiBps_packet_bytes": round(n * FRAME / to / 2**30, 2), "ms_per_batch": round(to * 1e3, 2),
                           "h2d_GBps": round(h2d / to / 1e9, 2), "d2h_GBps": round(d2h / to / 1e9, 3)}
    from seastar_amd import numa

    # where this rank's pinned pool landed (move_pages query; place_rank bound the policy to the GPU's node)
    pages = {str(k): v for k, v in numa.page_nodes(pool.ctypes.data, pool.nbytes, 512).items()}
    ranks = per_rank(world, rank, dev, variants=own_rates, pool_pages_by_node=pages)
    if rank == 0:
        best_name = max(res, key=lambda k: res[k]["GiBps_packet_bytes"])
        best = res[best_name]
        emit("GiB/s Internet checksum incl. PCIe: pinned mbuf-shaped host buffers -> HBM -> host (cfg 5)",
             world * best["GiBps_packet_bytes"], "GiB/s", args, world, best["ms_per_batch"] / 1e3 * args.steps, "u8",
             {"workload": "cfg5: 1,048,576 x 1500 B IPv4/UDP frames in 2304-B mbuf slots (pinned), "
                          "H2D + kernel + D2H of 4 B/frame (or the kernel reading the slots in place), 3-deep "
                          "pipeline, 64Ki-frame chunks; value = the best variant, all ranks' bytes over the "
                          "slowest rank's median time",
              "parallelism": f"{world} independent shards"},
             extra={"variants": res, "per_rank": ranks, "best_variant": best_name,
                    "ranks_summary": e2e_ranks_summary(ranks, best_name)})


def e2e_pcie_bytes(n: int, gather: int) -> tuple[int, int]:
    """Bytes crossing PCIe per cfg 5 batch, (host -> device, device -> host):
    the slots as they lie (A) or only the packet bytes (B, C, D), plus 12 B of
    offset + length per frame; back, the 4 B of checksums per frame."""
    from seastar_amd import pipeline

    per = pipeline.MBUF_SLOT if gather == native.GATHER_NONE else FRAME
    return n * (per + META_BYTES), n * 4


def e2e_ranks_summary(ranks: list, variant: str) -> dict:
    """cfg 5 across ranks for one variant: the sum of the ranks' own rates,
    the slowest rank (by name: rank, device, PCI id, NUMA node) and the
    per-rank H2D / D2H rates — at 8 GPUs the ranks share host DRAM and PCIe
    root complexes, so one slow link or a pool on the far node shows here."""
    rows = [(r["rank"], r["variants"][variant]) for r in ranks]
    slow_rank, slow = min(rows, key=lambda x: x[1]["GiBps_packet_bytes"])
    sr = next(r for r in ranks if r["rank"] == slow_rank)
    return {"variant": variant,
            "sum_over_ranks_GiBps": round(sum(v["GiBps_packet_bytes"] for _, v in rows), 2),
            "sum_h2d_GBps": round(sum(v["h2d_GBps"] for _, v in rows), 2),
            "slowest_rank": {"rank": slow_rank, "device": sr.get("device"), "pci_bus_id": sr.get("pci_bus_id"),
                             "numa_node": sr.get("numa_node"), "GiBps_packet_bytes": slow["GiBps_packet_bytes"],
                             "h2d_GBps": slow["h2d_GBps"], "d2h_GBps": slow["d2h_GBps"]},
            "per_rank_h2d_GBps": [v["h2d_GBps"] for _, v in rows],
            "per_rank_d2h_GBps": [v["d2h_GBps"] for _, v in rows]}


def run_dry(args, world, rank):
    """--dry-run: the multi-rank control plane without a device."""
    import torch.distributed as dist

    if os.environ.get("SCCSUM_DRY_RUN_FAIL_RANK") == str(rank):  # test hook: a rank that dies
        sys.exit(3)
    t0 = time.perf_counter()
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid(), "local": os.environ.get("LOCAL_RANK")})
    # the per_rank block of a real line, with the figures a device-less rank has
    pr = per_rank(world, rank, None, wall_s=time.perf_counter() - t0, GiBps=None, avg_launch_us=None,
                  read_ceiling_GBps=None, launch=launch_form(args))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "ranks": ranks, "per_rank": pr,
                          "barrier_s": round(wall, 6)}), flush=True)


def main():
    args = parse()
    global SYNC_MODE, SHARE_DEVICES
    SYNC_MODE = args.sync
    SHARE_DEVICES = args.share_devices
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    _imports()
    world, rank, local = dist_setup(args.dry_run, args)
    if args.dry_run:
        run_dry(args, world, rank)
    else:
        dev = torch.device("cuda", local)
        if args.tile_bytes is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_tile_bytes(args.tile_bytes), "sccsum_set_tile_bytes")
        if args.tile_packets is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_tile_packets(args.tile_packets), "sccsum_set_tile_packets")
        if args.variant is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_kernel_variant(args.variant), "sccsum_set_kernel_variant")
        if args.blocks_per_cu is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_blocks_per_cu(args.blocks_per_cu), "sccsum_set_blocks_per_cu")
        if args.out_policy is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_out_policy(args.out_policy), "sccsum_set_out_policy")
        if args.engine_sync is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_engine_sync_every(args.engine_sync), "sccsum_set_engine_sync_every")
        if args.engine_wt is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_engine_write_through(args.engine_wt),
                         "sccsum_set_engine_write_through")
        if args.fill_single_max is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_fill_single_max(args.fill_single_max), "sccsum_set_fill_single_max")
        if args.run_align is not None:  # A/B only (sccsum_diag.h)
            native.check(native.load().sccsum_set_run_align(args.run_align), "sccsum_set_run_align")
        {"udp1500": run_udp1500, "tcp64k": run_tcp64k, "mixed": run_mixed, "e2e": run_e2e, "fill": run_fill,
         "sweep": run_sweep, "slots": run_slots, "frags": run_frags}[args.config](args, world, rank, dev)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
