"""Burst queue (sccsum_burst_*, the batching hook at the qp boundary, SURVEY.md
§8(f)3) against the oracle: packets handed over one at a time as fragment
lists, batched for the GPU, completed in submit order."""
import numpy as np
import pytest

import oracle
from seastar_amd import native, synth
from seastar_amd.burst import BurstQueue

pytestmark = pytest.mark.gpu


def _split(rng, pkt):
    """1-4 fragments at random cut points (odd lengths and empty fragments included)."""
    cuts = sorted(int(c) for c in rng.integers(0, pkt.size + 1, size=int(rng.integers(0, 4))))
    edges = [0, *cuts, pkt.size]
    return [pkt[a:b] for a, b in zip(edges[:-1], edges[1:])]


def _feed(q, rng, buf, off, lens, seeds=None, poll_every=7):
    """Submit every packet (polling while the queue pushes back), poll every
    few packets as the reactor would, drain at the end."""
    tickets = []
    for i in range(lens.size):
        pkt = buf[int(off[i]):int(off[i]) + int(lens[i])]
        frags = _split(rng, pkt)
        while (t := q.submit(frags, 0 if seeds is None else int(seeds[i]))) is None:
            q.poll()
        tickets.append(t)
        if i % poll_every == 0:
            q.poll()
    q.drain()
    return tickets


def test_burst_spans_fragments_seeds(dev):
    rng = np.random.default_rng(51)
    lens = np.concatenate([rng.integers(0, 2100, 3000), [0, 1, 9000, 65535, 70000]]).astype(np.uint32)
    off, total = synth.pack(lens, seed=52, max_gap=3)
    buf = rng.integers(0, 256, size=max(int(total), 1), dtype=np.uint8)
    seeds = rng.integers(0, 65536, lens.size).astype(np.uint32)
    q = BurstQueue(native.PIPE_SPANS, batch_bytes=256 << 10, batch_packets=200, max_delay_ns=0, depth=3)
    tickets = _feed(q, rng, buf, off, lens, seeds)
    assert tickets == list(range(lens.size))
    got = np.array([int(q.results[t]) for t in tickets], np.uint16)
    assert np.array_equal(got, oracle.batch_spans(buf, off, lens, seeds))
    assert q.batches >= lens.size // 200
    q.close()


def test_burst_frames_and_backpressure(dev):
    buf, off, lens, _ = synth.mixed_udp_frames(1500, seed=53, max_gap=3)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    rng = np.random.default_rng(54)
    q = BurstQueue(native.PIPE_IPV4, batch_bytes=1 << 20, batch_packets=128, max_delay_ns=10**12, depth=2)
    tickets = _feed(q, rng, buf, off, lens, poll_every=32)
    assert tickets == list(range(lens.size))
    got = np.stack([q.results[t] for t in tickets])
    st = np.array([q.status[t] for t in tickets], np.uint8)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)
    q.close()

    # depth 1, one packet per batch: the second submit finds the only slot in flight
    seen = []
    q1 = BurstQueue(native.PIPE_IPV4, batch_bytes=64 << 10, batch_packets=1, max_delay_ns=10**12, depth=1,
                    on_done=lambda first, r, s: seen.append((first, r, s)))
    f0 = buf[int(off[0]):int(off[0]) + int(lens[0])]
    f1 = buf[int(off[1]):int(off[1]) + int(lens[1])]
    assert q1.submit([f0]) == 0
    assert q1.submit([f1]) is None  # it launched the full slot; nothing is free until that one is delivered
    q1.drain()
    assert q1.submit([f1]) == 1
    assert q1.poll() in (True, False)
    q1.drain()
    assert [s[0] for s in seen] == [0, 1]
    assert np.array_equal(np.stack([s[1][0] for s in seen]), want[:2])
    assert [int(s[2][0]) for s in seen] == [int(x) for x in want_st[:2]]
    with pytest.raises(native.SccsumError):
        q1.submit([np.zeros((64 << 10) + 1, np.uint8)])  # longer than a batch
    q1.close()


@pytest.fixture(params=[2, 1, 0], ids=["zero_copy", "fused", "gather"])
def fused(request):
    """Zero-copy batches: one fragment-list launch on pinned metadata (default),
    the same kernel between metadata / result copies, or gathered first."""
    lib = native.load()
    assert lib.sccsum_set_burst_fused(request.param) == native.SCCSUM_OK
    yield request.param
    lib.sccsum_set_burst_fused(2)


def _pinned_copy(buf):
    from seastar_amd import pipeline

    pool = pipeline.pinned_empty(buf.size + 64)
    pool[: buf.size] = buf
    return pool


def test_burst_mapped_zero_copy(dev, fused):
    """sccsum_burst_submit_mapped: fragments in pinned host memory, read over
    PCIe by the device; odd fragment cuts, empty packets, seeds."""
    rng = np.random.default_rng(55)
    lens = np.concatenate([rng.integers(0, 2100, 2500), [0, 1, 9000, 65535]]).astype(np.uint32)
    off, total = synth.pack(lens, seed=56, max_gap=5)
    host = rng.integers(0, 256, size=max(int(total), 1), dtype=np.uint8)
    buf = _pinned_copy(host)
    seeds = rng.integers(0, 65536, lens.size).astype(np.uint32)
    q = BurstQueue(native.PIPE_SPANS, batch_bytes=256 << 10, batch_packets=150, max_delay_ns=0, depth=3)
    tickets = []
    for i in range(lens.size):
        pkt = buf[int(off[i]):int(off[i]) + int(lens[i])]
        while (t := q.submit(_split(rng, pkt), int(seeds[i]), mapped=True)) is None:
            q.poll()
        tickets.append(t)
        if i % 5 == 0:
            q.poll()
    q.drain()
    assert tickets == list(range(lens.size))
    got = np.array([int(q.results[t]) for t in tickets], np.uint16)
    assert np.array_equal(got, oracle.batch_spans(host, off, lens, seeds))
    q.close()


def test_burst_mixed_copy_and_mapped(dev, fused):
    """Copied and zero-copy packets alternate inside the same batches (the
    H2D then carries the staged bytes; the fragment-list kernel reads those
    from the batch and the rest where they lie)."""
    host, off, lens, _ = synth.mixed_udp_frames(1200, seed=57, max_gap=3)
    want, want_st = oracle.batch_ipv4(host, off, lens)
    buf = _pinned_copy(host)
    rng = np.random.default_rng(58)
    q = BurstQueue(native.PIPE_IPV4, batch_bytes=1 << 20, batch_packets=100, max_delay_ns=10**12, depth=2)
    for i in range(lens.size):
        src = buf if i % 3 else host
        pkt = src[int(off[i]):int(off[i]) + int(lens[i])]
        while q.submit(_split(rng, pkt), mapped=bool(i % 3)) is None:
            q.poll()
    q.drain()
    got = np.stack([q.results[t] for t in range(lens.size)])
    st = np.array([q.status[t] for t in range(lens.size)], np.uint8)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)
    q.close()


def test_gather_kernel_any_alignment(dev):
    """sccsum_gather from pinned host memory and from device memory into odd
    destination offsets; bytes between the fragments stay untouched."""
    import ctypes

    import torch

    lib = native.load()
    rng = np.random.default_rng(59)
    n = 3000
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    lens[:5] = [0, 1, 15, 16, 17]
    src_off, stotal = synth.pack(lens, seed=60, max_gap=7)
    host = rng.integers(0, 256, size=int(stotal) + 64, dtype=np.uint8)
    pinned = _pinned_copy(host)
    gaps = rng.integers(0, 9, n)
    dst_off = np.zeros(n, np.uint64)
    pos = 3
    for i in range(n):
        dst_off[i] = pos
        pos += int(lens[i]) + int(gaps[i])
    d_src = torch.from_numpy(host).to(dev)
    for base in (pinned.ctypes.data, d_src.data_ptr()):
        desc = np.zeros(n, dtype=[("src", "<u8"), ("dst_off", "<u4"), ("len", "<u4")])
        desc["src"] = base + src_off
        desc["dst_off"] = dst_off
        desc["len"] = lens
        d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
        dst = torch.full((pos + 16,), 0xA5, dtype=torch.uint8, device=dev)
        assert lib.sccsum_gather(ctypes.c_void_p(d_desc.data_ptr()), n, ctypes.c_void_p(dst.data_ptr()),
                                 None) == native.SCCSUM_OK
        torch.cuda.synchronize()
        want = np.full(pos + 16, 0xA5, np.uint8)
        for i in range(n):
            want[int(dst_off[i]):int(dst_off[i]) + int(lens[i])] = host[int(src_off[i]):int(src_off[i]) + int(lens[i])]
        assert np.array_equal(dst.cpu().numpy(), want)


def test_pinned_view_outlives_pool(dev):
    """A view of a pinned_empty pool keeps the pinned block alive after the
    pool array itself is dropped (the block is freed with its last view)."""
    import gc

    from seastar_amd import pipeline

    pool = pipeline.pinned_empty(1 << 20)
    pool[:] = 7
    view = pool[4096:8192]
    addr = view.ctypes.data
    del pool
    gc.collect()
    assert pipeline.is_pinned(view)
    view[:] = np.arange(view.size, dtype=np.uint8)
    assert view.ctypes.data == addr and int(view[255]) == 255
    # the view is still good for a zero-copy submit
    q = BurstQueue(native.PIPE_SPANS, batch_bytes=64 << 10, batch_packets=8, max_delay_ns=0, depth=2)
    q.submit([view[:1500]], 0, mapped=True)
    q.drain()
    assert int(q.results[0]) == int(oracle.batch_spans(view.copy(), np.zeros(1, np.uint64),
                                                       np.full(1, 1500, np.uint32))[0])
    q.close()
    del view
    gc.collect()


def test_mapped_submit_rejects_pageable_memory(dev):
    q = BurstQueue(native.PIPE_SPANS, batch_bytes=64 << 10, batch_packets=8, max_delay_ns=0, depth=2)
    with pytest.raises(ValueError):
        q.submit([np.zeros(100, np.uint8)], mapped=True)  # ordinary pageable numpy memory
    with pytest.raises(ValueError):
        q.submit([b"\x00" * 100], mapped=True)
    q.close()


def test_callback_reentrancy(dev):
    """A completion callback that polls / drains is refused (SCCSUM_EINVAL),
    one that submits works; every batch is delivered exactly once, in order."""
    import ctypes

    lib = native.load()
    seen, inner = [], []
    holder = {}

    def on_done(first, r, s):
        seen.append((first, r.copy()))
        inner.append(lib.sccsum_burst_poll(holder["q"]._h, None))
        inner.append(lib.sccsum_burst_drain(holder["q"]._h))
        if first < 40:  # resubmit from inside the callback
            holder["q"].submit([np.full(64, first, np.uint8)])

    q = BurstQueue(native.PIPE_SPANS, batch_bytes=64 << 10, batch_packets=4, max_delay_ns=0, depth=3, on_done=on_done)
    holder["q"] = q
    for i in range(20):
        while q.submit([np.full(64, i, np.uint8)]) is None:
            q.poll()
        q.poll()
    for _ in range(20):
        q.drain()
    firsts = [f for f, _ in seen]
    assert firsts == sorted(firsts) and len(set(firsts)) == len(firsts)
    total = sum(r.size for _, r in seen)
    assert firsts[0] == 0 and total == firsts[-1] + seen[-1][1].size  # consecutive tickets, none lost or repeated
    assert all(code == native.SCCSUM_EINVAL for code in inner)
    q.close()
    assert ctypes.sizeof(ctypes.c_void_p) == 8


def test_burst_mapped_recycled_buffers(dev, fused):
    """Zero-copy submits from a small pinned pool whose slots the host rewrites
    after every drain (recycled mbufs): no batch may see an earlier batch's
    bytes."""
    from seastar_amd import pipeline

    rng = np.random.default_rng(81)
    nslot, slot = 64, 2304
    pool = pipeline.pinned_empty(nslot * slot)
    q = BurstQueue(native.PIPE_SPANS, batch_bytes=256 << 10, batch_packets=32, max_delay_ns=0, depth=2)
    for rnd in range(10):
        lens = rng.integers(0, 2049, nslot).astype(np.uint32)
        pool[:] = rng.integers(0, 256, pool.size, dtype=np.uint8)
        tickets = []
        for i in range(nslot):
            pkt = pool[i * slot + 128:i * slot + 128 + int(lens[i])]
            while (t := q.submit(_split(rng, pkt), 0, mapped=True)) is None:
                q.poll()
            tickets.append(t)
        q.drain()
        off = (np.arange(nslot, dtype=np.uint64) * slot + 128)
        want = oracle.batch_spans(np.array(pool), off, lens, np.zeros(nslot, np.uint32))
        got = np.array([int(q.results[t]) for t in tickets], np.uint16)
        assert np.array_equal(got, want), rnd
    q.close()
