"""Multi-rank sharding on CPU: world_size 2 over gloo.
Each rank takes its byte-balanced shard, checksums it, results are gathered
by index and must equal the unsharded batch; no data-path collective is
involved.  On CPU the oracle stands in for the per-rank engine; the gpu test
runs libsccsum's resident engine in every rank (two rank processes on the
box's one GPU, the same code path the driver's N-GPU run takes with
cuda:rank)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from seastar_amd import shard, synth


def test_partition_by_bytes_balanced():
    lens = synth.zipf_lengths(5000, seed=1)
    for world in (1, 2, 3, 4, 8):
        b = shard.partition_by_bytes(lens, world)
        assert b[0] == 0 and b[-1] == lens.size and np.all(np.diff(b) >= 0)
        per = [int(lens[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert max(per) - min(per) <= 2 * int(lens.max())


def test_partition_edge_cases():
    assert list(shard.partition_by_bytes(np.array([], np.uint32), 2)) == [0, 0, 0]
    assert list(shard.partition_by_bytes(np.array([5], np.uint32), 3))[-1] == 1
    with pytest.raises(ValueError):
        shard.partition_by_bytes(np.array([1]), 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine_gpu(sbuf, soff, slen, rank, world):
    """Rank r drives device r % ndev (bench.dist_setup's mapping), bound and
    initialised as a shard thread is (sccsum_init(d)), and runs its shard the
    way bench.py's ranks do by default: as steps of one resident engine run
     — slices of at most 4 096 frames of its one batch, 4 in
    flight on a 64-slot ring, waited on, the engine closed clean.  Where every
    rank has a device of its own the runs are concurrent; on the one-GPU box
    the ranks' runs take turns (a gloo barrier between turns: an engine grid
    holds every CU of its device while it runs)."""
    import torch
    from seastar_amd import batch, native

    ndev = torch.cuda.device_count()
    d = rank % ndev
    torch.cuda.set_device(d)
    native.check(native.load().sccsum_init(d), "sccsum_init")
    b = batch.PacketBatch.from_host(sbuf, soff, slen, device=f"cuda:{d}")
    status = torch.full((max(b.n, 1),), 0xEE, dtype=torch.uint8, device=b.device)
    out = torch.full((max(2 * b.n, 2),), -1, dtype=torch.int16, device=b.device)
    steps = []
    for lo in range(0, b.n, 4096):
        hi = min(lo + 4096, b.n)
        part = batch.PacketBatch(data=b.data, off=b.off[lo:hi], length=b.length[lo:hi], bytes_len=b.bytes_len,
                                 max_len=b.max_len)
        steps.append([(part, out[2 * lo:2 * hi], status[lo:hi])])
    torch.cuda.synchronize(d)
    turns = world if ndev < world else 1  # one GPU for several ranks: one engine run at a time

    def run():
        eng = batch.Engine(d, frames=True, ring_slots=64, max_in_flight=4)
        stream = torch.cuda.Stream(device=d)
        eng.start(stream)
        for items in steps:
            eng.submit(items)
        eng.finish()
        stream.synchronize()
        eng.close()

    for turn in range(turns):
        if turns == 1 or turn == rank:
            run()
        if turns > 1:
            dist.barrier()
    p = torch.cuda.get_device_properties(d)
    where = (d, f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0", ndev,
             "engine (runs take turns: one device)" if turns > 1 else "engine (concurrent runs)")
    return out[:2 * b.n].cpu().numpy().view(np.uint16), status[:b.n].cpu().numpy(), where


def _worker(rank, world, port, q, engine="oracle", n=3000):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, off, lens, _ = synth.mixed_udp_frames(n, seed=5, max_gap=3)
    sbuf, soff, slen, (lo, hi) = shard.shard(buf, off, lens, rank, world)
    where = None
    if engine == "gpu":
        out, st, where = _engine_gpu(sbuf, soff, slen, rank, world)
    else:
        out, st = oracle.batch_ipv4(sbuf, soff, slen)
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, out, st, where))
    if rank == 0:
        full = shard.assemble([(a, b, o.reshape(-1, 2)) for a, b, o, _, _ in parts], lens.size, width=2)
        full_st = shard.assemble([(a, b, s) for a, b, _, s, _ in parts], lens.size, dtype=np.uint8)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        ok = bool(np.array_equal(full, want) and np.array_equal(full_st, want_st))
        devs = [w for *_, w in parts]
        if engine == "gpu":
            ndev = devs[0][2]
            # one device per rank wherever there are enough: indices and PCI addresses differ
            if ndev >= world:
                ok = ok and len({w[0] for w in devs}) == world and len({w[1] for w in devs}) == world
            else:
                ok = ok and [w[0] for w in devs] == [r % ndev for r in range(world)]
        q.put((ok, devs))
    dist.destroy_process_group()


def _run(world, engine, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, engine, n)) for r in range(world)]
    for p in procs:
        p.start()
    ok, devs = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert ok, devs
    assert all(p.exitcode == 0 for p in procs)
    return devs


def test_two_rank_gloo_shards_match_unsharded():
    _run(2, "oracle", 3000)


@pytest.mark.gpu
def test_two_rank_gpu_engine_shards_match_oracle():
    """Two ranks, rank r on device r % ndev, each running its shard through a
    resident engine: devices 0 and 1 where two are visible (concurrent runs),
    both on device 0 on the one-GPU box (the runs take turns; stated in the
    output)."""
    devs = _run(2, "gpu", 20000)
    print("rank devices:", devs)
