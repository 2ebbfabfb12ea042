"""Multi-rank sharding on CPU: world_size 2 over gloo.
Each rank takes its byte-balanced shard, checksums it (the oracle stands in
for the per-rank GPU engine here), results are gathered by index and must
equal the unsharded batch; no data-path collective is involved."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, off, lens, _ = synth.mixed_udp_frames(3000, seed=5, max_gap=3)
    sbuf, soff, slen, (lo, hi) = shard.shard(buf, off, lens, rank, world)
    out, st = oracle.batch_ipv4(sbuf, soff, slen)
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, out, st))
    if rank == 0:
        full = shard.assemble([(a, b, o) for a, b, o, _ in parts], lens.size, width=2)
        full_st = shard.assemble([(a, b, s) for a, b, _, s in parts], lens.size, dtype=np.uint8)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        q.put(bool(np.array_equal(full, want) and np.array_equal(full_st, want_st)))
    dist.destroy_process_group()


def test_two_rank_gloo_shards_match_unsharded():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok
