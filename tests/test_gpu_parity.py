"""Parity of the HIP kernels (through the C-ABI) with the oracle — bit-exact.

Small cases compare every output with the oracle; the full-size cases
(BASELINE.json configs at full scale) use size-independent properties:
generate -> store -> verify round trips, exact failure sets after corruption,
and oracle comparison on a random sample.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

import oracle
from seastar_amd import batch, native, synth

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(params=[1, 2, 14, 15, 16], ids=["simple", "rows", "flat8", "flat8_pipe", "flat16"],
                autouse=True)
def kernel_variant(request, dev):
    """Every parity test runs against both kernel families."""
    lib = native.load()
    native.check(lib.sccsum_set_kernel_variant(request.param), "set variant")
    yield request.param
    native.check(lib.sccsum_set_kernel_variant(0), "reset variant")


def _spans(dev, buf, off, length, seeds=None, with_status=False):
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    sd = None if seeds is None else torch.from_numpy(np.asarray(seeds, np.uint32).view(np.int32)).to(dev)
    st = torch.empty(max(b.n, 1), dtype=torch.uint8, device=dev) if with_status else None
    out = batch.spans(b, seeds=sd, status=st)
    torch.cuda.synchronize()
    got = batch.as_u16(out)
    return (got, st[: b.n].cpu().numpy()) if with_status else got


def _frames(dev, buf, off, length):
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    st = torch.empty(max(b.n, 1), dtype=torch.uint8, device=dev)
    out = batch.ipv4_frames(b, status=st)
    torch.cuda.synchronize()
    return batch.as_u16(out), st[: b.n].cpu().numpy()


def test_known_answers(dev):
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    cases = [c for c in kat["ip_checksum"]]
    datas = [bytes.fromhex(c["hex"]) for c in cases]
    buf = np.frombuffer(b"".join(datas), np.uint8) if any(datas) else np.zeros(0, np.uint8)
    length = np.array([len(d) for d in datas], np.uint32)
    off = np.concatenate([[0], np.cumsum(length)[:-1]]).astype(np.uint64)
    got = _spans(dev, buf, off, length)
    want = np.array([int.from_bytes(bytes.fromhex(c["result_bytes"]), "little") for c in cases], np.uint16)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("fill", ["random", "zeros", "ones"])
def test_every_length_every_alignment(dev, fill):
    """Lengths 0..2100 at all 16 start alignments (head/tail masking, odd starts)."""
    rng = np.random.default_rng(11)
    lens = np.tile(np.arange(0, 2101, dtype=np.uint32), 16)
    heads = np.repeat(np.arange(16, dtype=np.uint64), 2101)
    off = np.empty(lens.size, np.uint64)
    pos = 0
    for i, (L, h) in enumerate(zip(lens.tolist(), heads.tolist())):
        pos = ((pos + 15) // 16) * 16 + h
        off[i] = pos
        pos += L
    if fill == "random":
        buf = rng.integers(0, 256, size=pos, dtype=np.uint8)
    elif fill == "zeros":
        buf = np.zeros(pos, np.uint8)
    else:
        buf = np.full(pos, 0xFF, np.uint8)
    got = _spans(dev, buf, off, lens)
    want = oracle.batch_spans(buf, off, lens)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatches (len, head): {[(int(lens[i]), int(heads[i])) for i in bad[:8]]}"


def test_seeds_and_status(dev):
    rng = np.random.default_rng(5)
    n = 4000
    lens = rng.integers(0, 9001, size=n).astype(np.uint32)
    off, total = synth.pack(lens, seed=9, max_gap=15)
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    seeds = rng.integers(0, 65536, size=n).astype(np.uint32)
    seeds[:50] = 0
    seeds[50:100] = 0xFFFF
    got, st = _spans(dev, buf, off, lens, seeds, with_status=True)
    want = oracle.batch_spans(buf, off, lens, seeds)
    assert np.array_equal(got, want)
    assert np.array_equal(st, (want == 0).astype(np.uint8))


def test_zero_sum_edge(dev):
    """fold(0)=0 vs 0xFFFF: all-zero data with zero seed -> 0xFFFF; zero data
    with seed 0xFFFF -> 0x0000; ff ff -> 0."""
    buf = np.zeros(4096, np.uint8)
    buf[2048:2050] = 0xFF
    off = np.array([0, 0, 100, 2048, 2048, 3000], np.uint64)
    lens = np.array([0, 2000, 1, 2, 0, 96], np.uint32)
    seeds = np.array([0, 0, 0xFFFF, 0, 0xFFFF, 0xFFFF], np.uint32)
    got = _spans(dev, buf, off, lens, seeds)
    want = oracle.batch_spans(buf, off, lens, seeds)
    assert np.array_equal(got, want)
    assert got[0] == 0xFFFF and got[1] == 0xFFFF and got[3] == 0


def test_large_spans_tcp64k_pseudo_wrap(dev):
    """64 KiB TCP segments: pseudo-header length 65536 truncates to 0
    (ip.hh:70-75, tcp.hh:878); also 65535 and jumbo lengths."""
    n = 64
    buf, off, lens, meta = synth.tcp_segments(n, 65536, seed=21)
    seeds = np.array([oracle.pseudo_seed(int(s), int(d), 6, 65536) for s, d in zip(meta["src"], meta["dst"])],
                     np.uint32)
    seeds_cabi = np.array([batch.pseudo_seed(int(s), int(d), 6, 65536) for s, d in zip(meta["src"], meta["dst"])],
                          np.uint32)
    assert np.array_equal(seeds, seeds_cabi)
    got = _spans(dev, buf, off, lens, seeds)
    want = oracle.batch_spans(buf, off, lens, seeds)
    assert np.array_equal(got, want)
    # 65535-byte variant at odd offsets
    lens2 = np.full(16, 65535, np.uint32)
    off2, total = synth.pack(lens2, seed=3, max_gap=5)
    rb = np.random.default_rng(8).integers(0, 256, size=total, dtype=np.uint8)
    got2 = _spans(dev, rb, off2, lens2)
    assert np.array_equal(got2, oracle.batch_spans(rb, off2, lens2))


def test_udp1500_generate_verify_roundtrip(dev):
    n = 20000
    buf, off, lens, _ = synth.udp_ipv4_frames(n, 1500, seed=42)
    got, st = _frames(dev, buf, off, lens)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    assert np.array_equal(got, want)
    assert np.array_equal(st, want_st)
    rx = buf.copy()
    synth.store_ipv4_checksums(rx, off, got)
    got2, st2 = _frames(dev, rx, off, lens)
    assert np.all(got2 == 0) and np.all(st2 == 3)
    # corrupt 1 %: one payload byte each -> exactly those fail L4, IP still ok
    rng = np.random.default_rng(4)
    bad = rng.choice(n, size=n // 100, replace=False)
    for i in bad:
        rx[int(off[i]) + 100 + int(i % 1000)] ^= 0x5A
    got3, st3 = _frames(dev, rx, off, lens)
    fail = np.nonzero((st3 & 2) == 0)[0]
    assert np.array_equal(np.sort(fail), np.sort(bad))
    assert np.all(st3 & 1)
    want3, want_st3 = oracle.batch_ipv4(rx, off, lens)
    assert np.array_equal(got3, want3) and np.array_equal(st3, want_st3)


@pytest.mark.parametrize("align,gap", [(1, 0), (1, 9), (64, 0)])
def test_mixed_mtu_frames(dev, align, gap):
    buf, off, lens, _ = synth.mixed_udp_frames(3000, seed=77, align=align, max_gap=gap)
    got, st = _frames(dev, buf, off, lens)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    assert np.array_equal(got, want)
    assert np.array_equal(st, want_st)


def test_malformed_and_range(dev):
    rng = np.random.default_rng(3)
    buf, off, lens, _ = synth.udp_ipv4_frames(8, 200, seed=1)
    buf = buf.copy()
    # 0: short frame; 1: ip_len > len; 2: ihl 15 (options beyond ip_len 200? no: 60 < 200);
    # 3: ihl 0 (L4 starts at 0 as in the reference); 4: ip_len < len (trim);
    # 5: ihl*4 > ip_len; 6: out of range; 7: normal
    lens = lens.copy()
    off = off.copy()
    lens[0] = 19
    buf[int(off[1]) + 2:int(off[1]) + 4] = [0x01, 0x00]  # 256 > 200
    buf[int(off[2])] = 0x4F
    buf[int(off[3])] = 0x40
    buf[int(off[4]) + 2:int(off[4]) + 4] = [0x00, 0x80]  # 128 < 200
    buf[int(off[5])] = 0x4F
    buf[int(off[5]) + 2:int(off[5]) + 4] = [0x00, 0x28]  # 40 < 60
    off[6] = buf.size - 10
    got, st = _frames(dev, buf, off, lens)
    want, want_st = oracle.batch_ipv4(buf, off[:6].copy(), lens[:6].copy())
    assert np.array_equal(got[:6], want)
    assert np.array_equal(st[:6], want_st)
    assert st[6] == native.ST_RANGE and np.all(got[6] == 0)
    want7, want_st7 = oracle.batch_ipv4(buf, off[7:].copy(), lens[7:].copy())
    assert np.array_equal(got[7:], want7) and np.array_equal(st[7:], want_st7)
    assert st[0] == native.ST_MALFORMED and (st[1] & native.ST_MALFORMED) and (st[5] & native.ST_MALFORMED)
    # spans: range errors never read
    sg, ss = _spans(dev, rng.integers(0, 256, 100, dtype=np.uint8), np.array([0, 90, 200], np.uint64),
                    np.array([100, 20, 0], np.uint32), with_status=True)
    assert ss[1] == native.ST_RANGE and ss[2] == native.ST_RANGE and sg[1] == 0


def test_cabi_errors(dev):
    lib = native.load()
    assert lib.sccsum_spans(None, 0, None, None, None, None, None, 0, 0, None) == 0  # n == 0 is a no-op
    assert lib.sccsum_spans(None, 16, None, None, None, None, None, 5, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_init(10_000) == native.SCCSUM_ENODEV


def test_full_scale_udp1500(dev):
    """BASELINE cfg 2 at full size: 1,048,576 x 1500 B, generate -> store ->
    verify (all pass), 1 % corrupted fail exactly, oracle on a 8192 sample."""
    n, L = 1 << 20, 1500
    from seastar_amd import devsynth

    tx = devsynth.udp_frames(n, L, seed=0x5EA57A2C, device=dev)
    out = batch.ipv4_frames(tx)
    rx = devsynth.store_checksums(tx, out)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    out_rx = batch.ipv4_frames(rx, status=st)
    assert int((out_rx != 0).sum()) == 0 and int((st != 3).sum()) == 0
    idx = torch.randperm(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1))[: n // 100]
    devsynth.corrupt(rx, idx, byte=777)
    out_bad = batch.ipv4_frames(rx, status=st)
    failed = torch.nonzero((st & 2) == 0).flatten()
    assert torch.equal(torch.sort(failed).values, torch.sort(idx).values)
    sample = np.sort(np.random.default_rng(0).choice(n, 8192, replace=False))
    frames = rx.data[: n * L].view(n, L)[torch.from_numpy(sample).to(dev)].cpu().numpy().reshape(-1)
    soff = np.arange(sample.size, dtype=np.uint64) * L
    want, _ = oracle.batch_ipv4(frames, soff, np.full(sample.size, L, np.uint32))
    assert np.array_equal(batch.as_u16(out_bad)[sample], want)


def test_read_probe(dev):
    buf = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8, device=dev)
    sink = batch.read_probe(buf, buf.numel())
    torch.cuda.synchronize()
    assert int(sink.sum()) > 0


def test_zipf_large_spans_odd_offsets(dev):
    """cfg 3 shape at scale: 200k Zipf(1.2) lengths 64..9000 packed with odd
    gaps (the A/B tool's batch), with seeds, every packet vs the oracle."""
    lens = synth.zipf_lengths(200_000, seed=3)
    off, total = synth.pack(lens, seed=4, max_gap=3)
    buf = np.random.default_rng(5).integers(0, 256, size=total, dtype=np.uint8)
    seeds = np.random.default_rng(6).integers(0, 65536, size=lens.size).astype(np.uint32)
    got = _spans(dev, buf, off, lens)
    want = oracle.batch_spans(buf, off, lens, nthreads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first (idx, len, off): " + str(
        [(int(i), int(lens[i]), int(off[i])) for i in bad[:5]])
    got = _spans(dev, buf, off, lens, seeds)
    assert np.array_equal(got, oracle.batch_spans(buf, off, lens, seeds, nthreads=8))


def test_zipf_large_frames(dev):
    buf, off, lens, _ = synth.mixed_udp_frames(20_000, seed=12, max_gap=3)
    got, st = _frames(dev, buf, off, lens)
    want, want_st = oracle.batch_ipv4(buf, off, lens, nthreads=8)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)


@pytest.mark.parametrize("gather", [0, 1, 2, 3], ids=["as_is", "host_gather", "strided_dma", "zero_copy"])
def test_host_pipeline_mbuf_pool(dev, gather, kernel_variant):
    """cfg 5 path: frames in an mbuf-shaped pinned pool, chunked through the
    GPU with async copies; small chunks force many stage recycles."""
    if kernel_variant not in (1, 15):
        pytest.skip("pipeline exercised with two kernel families")
    from seastar_amd import pipeline

    # one mbuf data room holds 2048 B (dpdk.cc:147-156): clip the Zipf lengths
    lens = np.minimum(synth.zipf_lengths(2500, seed=30), 2048).astype(np.uint32)
    buf, off, lens, _ = synth.mixed_udp_frames(2500, seed=31, max_gap=5, lengths=lens)
    pool, poff, plen = pipeline.mbuf_pool(buf, lens, off)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    pl = pipeline.HostPipeline(0, chunk_bytes=1 << 20, chunk_packets=300, depth=3)
    got, st = pl.run(native.PIPE_IPV4, pool, poff, plen, status=True, gather=gather, max_len=9000)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)
    seeds = np.random.default_rng(2).integers(0, 65536, lens.size).astype(np.uint32)
    got2 = pl.run(native.PIPE_SPANS, pool, poff, plen, seeds=seeds, gather=gather)
    assert np.array_equal(got2, oracle.batch_spans(pool, poff, plen, seeds))
    pl.close()


def test_host_pipeline_zero_copy_refuses_pageable_memory(dev):
    """gather = 3 reads the caller's buffer in place: pageable memory is
    refused (ValueError in Python, SCCSUM_EINVAL from the C-ABI) instead of
    faulting the GPU."""
    import ctypes

    from seastar_amd import pipeline

    buf, off, lens, _ = synth.mixed_udp_frames(50, seed=41)
    pl = pipeline.HostPipeline(0, chunk_bytes=1 << 20, chunk_packets=64, depth=2)
    with pytest.raises(ValueError):
        pl.run(native.PIPE_IPV4, buf, off, lens, gather=native.GATHER_ZERO_COPY)
    off64 = np.ascontiguousarray(off, np.uint64)
    l32 = np.ascontiguousarray(lens, np.uint32)
    out = np.empty(2 * lens.size, np.uint16)
    rc = native.load().sccsum_pipeline_run(pl._h, native.PIPE_IPV4, native.GATHER_ZERO_COPY, buf.ctypes.data, buf.size,
                                           off64.ctypes.data, l32.ctypes.data, None, lens.size, 1500,
                                           out.ctypes.data, None)
    assert rc == native.SCCSUM_EINVAL
    pinned = pipeline.pinned_empty(buf.size + 64)
    pinned[64:] = buf
    got = pl.run(native.PIPE_IPV4, pinned[64:], off, lens, gather=native.GATHER_ZERO_COPY, max_len=1500)
    assert np.array_equal(got, oracle.batch_ipv4(buf, off, lens)[0])
    # the whole range must lie in ONE pinned allocation: a host_len that runs past the block is refused
    # (an ends-only check would pass two pinned blocks with pageable memory between them: ADVICE r02)
    rc = native.load().sccsum_pipeline_run(pl._h, native.PIPE_IPV4, native.GATHER_ZERO_COPY, pinned.ctypes.data,
                                           pinned.size + (1 << 20), off64.ctypes.data, l32.ctypes.data, None,
                                           lens.size, 1500, out.ctypes.data, None)
    assert rc == native.SCCSUM_EINVAL
    pl.close()
    assert ctypes.sizeof(ctypes.c_void_p) == 8


def test_host_pipeline_strided_irregular(dev):
    """gather = 2 on layouts that are only partly slot-shaped: a pitch break
    mid-batch, a packet longer than the pitch, a single-packet tail chunk and
    chunk_bytes that cut rows — every chunk either rows or as-is, all exact."""
    from seastar_amd import pipeline

    rng = np.random.default_rng(40)
    n = 700
    lens = rng.integers(20, 600, size=n).astype(np.uint32)
    lens[350] = 900  # longer than the 640-B pitch: that chunk falls back
    off = np.arange(n, dtype=np.uint64) * 640 + 64
    off[500:] += 3  # pitch break (and odd slot starts from here on)
    total = int(off[-1]) + 1024
    pool = pipeline.pinned_empty(total)
    pool[:] = rng.integers(0, 256, size=total, dtype=np.uint8)
    seeds = rng.integers(0, 65536, n).astype(np.uint32)
    want = oracle.batch_spans(pool, off, lens, seeds)
    for chunk_bytes, chunk_packets in ((1 << 20, 256), (40 * 1024, 256), (1 << 20, 699)):
        pl = pipeline.HostPipeline(0, chunk_bytes=chunk_bytes, chunk_packets=chunk_packets, depth=2)
        got, st = pl.run(native.PIPE_SPANS, pool, off, lens, seeds=seeds, status=True,
                         gather=native.GATHER_STRIDED)
        pl.close()
        assert np.array_equal(got, want), (chunk_bytes, chunk_packets)


def _frag_batch(rng, n, sizes_fn, scatter=True):
    """n packets as fragment lists; fragments placed at random (odd included)
    offsets of one buffer, in shuffled order when scatter."""
    frag_len = []
    pkt_first = [0]
    for i in range(n):
        sizes = sizes_fn(i)
        frag_len.extend(sizes)
        pkt_first.append(len(frag_len))
    frag_len = np.array(frag_len, np.uint32)
    order = rng.permutation(frag_len.size) if scatter else np.arange(frag_len.size)
    off = np.empty(frag_len.size, np.uint64)
    pos = 0
    for j in order:
        pos += int(rng.integers(0, 4))
        off[j] = pos
        pos += int(frag_len[j])
    buf = rng.integers(0, 256, size=pos + 1, dtype=np.uint8)
    return buf, off, frag_len, np.array(pkt_first, np.uint32)


@pytest.mark.parametrize("shape", ["packet_test", "odd_chains", "dpdk_segments", "single"])
def test_fragment_lists(dev, shape):
    """GPU checksummer::sum(const packet&): odd carries across fragments."""
    rng = np.random.default_rng({"packet_test": 1, "odd_chains": 2, "dpdk_segments": 3, "single": 4}[shape])
    if shape == "packet_test":  # tests/unit/packet_test.cc:32-84 sizes, with trims
        base = [[5, 31, 65, 4096, 4096], [4, 25, 36, 3072, 4096], [1, 31, 65], [5], [0, 7]]
        fn = lambda i: base[i % len(base)]
    elif shape == "odd_chains":
        fn = lambda i: list(rng.integers(0, 40, size=int(rng.integers(1, 9))))
    elif shape == "dpdk_segments":  # jumbo frames in 2048-B data rooms (dpdk.cc:147-156)
        fn = lambda i: ([2048] * (int(L) // 2048) + [int(L) % 2048]) if (L := rng.integers(64, 9001)) else [0]
    else:
        fn = lambda i: [int(rng.integers(0, 3000))]
    n = 700
    buf, off, flen, first = _frag_batch(rng, n, fn)
    seeds = rng.integers(0, 65536, size=n).astype(np.uint32)
    d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    got = batch.fragments(d, buf.size, torch.from_numpy(off.view(np.int64)).to(dev),
                          torch.from_numpy(flen.view(np.int32)).to(dev), torch.from_numpy(first.view(np.int32)).to(dev),
                          seeds=torch.from_numpy(seeds.view(np.int32)).to(dev), status=st, max_frag_len=4096)
    torch.cuda.synchronize()
    want = oracle.batch_fragments(buf, off, flen, first, seeds)
    assert np.array_equal(batch.as_u16(got), want)
    assert np.array_equal(st.cpu().numpy(), (want == 0).astype(np.uint8))
    # fragments of a contiguous packet == the contiguous span
    if shape == "odd_chains":
        got2 = batch.fragments(d, buf.size, torch.from_numpy(off.view(np.int64)).to(dev),
                               torch.from_numpy(flen.view(np.int32)).to(dev),
                               torch.from_numpy(first.view(np.int32)).to(dev))
        assert np.array_equal(batch.as_u16(got2), oracle.batch_fragments(buf, off, flen, first))


def test_fragment_lists_range(dev):
    """A fragment past bytes_len (or a bad pkt_first) marks only its packet RANGE."""
    rng = np.random.default_rng(9)
    buf, off, flen, first = _frag_batch(rng, 64, lambda i: [3, 1500, 7], scatter=False)
    off = off.copy()
    off[3 * 10 + 1] = buf.size - 100  # packet 10's middle fragment overruns
    d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
    st = torch.empty(64, dtype=torch.uint8, device=dev)
    got = batch.as_u16(batch.fragments(d, buf.size, torch.from_numpy(off.view(np.int64)).to(dev),
                                       torch.from_numpy(flen.view(np.int32)).to(dev),
                                       torch.from_numpy(first.view(np.int32)).to(dev), status=st))
    stn = st.cpu().numpy()
    assert stn[10] == 8 and got[10] == 0
    ok = np.arange(64) != 10
    want = oracle.batch_fragments(buf, off, flen, first)
    assert np.array_equal(got[ok], want[ok])
    assert np.all(stn[ok] & 8 == 0)


def _tx_frames(rng, n):
    """IPv4 frames for the tx generate path: UDP / TCP / ICMP, IHL 5..15,
    Ethernet-padded (len > ip_len), truncated (malformed), runts (< 20 B),
    segments too short for their checksum field, GARBAGE in every checksum
    field (a generate must not depend on it); IP fragments (first, middle,
    last, past the 65 535-byte limit: synth.frag_words) among atomic
    datagrams; ICMP echo requests (some with all-zero messages, whose reply
    checksum is 0xffff) among other ICMP types; random odd offsets."""
    frames = []
    fw = synth.frag_words(rng, n)
    for i in range(n):
        proto = int(rng.choice([17, 6, 1, 17, 6]))
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(6, 16))
        pay = int(rng.integers(0, 30)) if rng.random() < 0.15 else int(rng.integers(0, 3000))
        ip_len = 4 * ihl + pay
        f = rng.integers(0, 256, size=ip_len, dtype=np.uint8)
        f[0] = 0x40 | ihl
        f[2], f[3] = ip_len >> 8, ip_len & 0xFF
        f[6], f[7] = int(fw[i]) >> 8, int(fw[i]) & 0xFF
        f[9] = proto
        if proto == 1 and pay >= 1:
            f[4 * ihl] = 8 if rng.random() < 0.7 else int(rng.choice([0, 3, 11, 13, 9]))
            if rng.random() < 0.1:  # all-zero message after type / code / checksum
                f[4 * ihl + 4:] = 0
        kind = rng.random()
        if kind < 0.08:  # Ethernet padding past ip_len
            f = np.concatenate([f, rng.integers(0, 256, size=int(rng.integers(1, 40)), dtype=np.uint8)])
        elif kind < 0.14:  # truncated: ip_len > len
            f = f[: max(20, ip_len - int(rng.integers(1, 50)))]
        elif kind < 0.17:  # runt
            f = f[: int(rng.integers(0, 20))]
        frames.append(f)
    length = np.array([f.size for f in frames], np.uint32)
    off = np.empty(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 5))
        off[i] = pos
        pos += int(length[i])
    buf = rng.integers(0, 256, size=pos + 3, dtype=np.uint8)
    for i in range(n):
        buf[int(off[i]): int(off[i]) + int(length[i])] = frames[i]
    return buf, off, length


FILL_MODES = {
    "ip_l4": native.FILL_IP | native.FILL_L4,
    "l4": native.FILL_L4,
    "ip": native.FILL_IP,
    "pseudo": native.FILL_L4_PSEUDO,
    "ip_pseudo_tso": native.FILL_IP | native.FILL_L4_PSEUDO | native.FILL_TSO,
    "icmp_echo": native.FILL_ICMP_ECHO,
    "ip_l4_icmp_echo": native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO,
}


@pytest.mark.parametrize("mode", list(FILL_MODES))
def test_ipv4_fill_in_place(dev, mode, fill_passes):
    """Tx generate + in-place store == the reference writers, byte for byte."""
    m = FILL_MODES[mode]
    rng = np.random.default_rng(0xF111 + m)
    buf, off, length = _tx_frames(rng, 900)
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_fill(b, m, out2=out2, status=st)
    torch.cuda.synchronize()
    want_buf, want_out2, want_st = oracle.batch_ipv4_fill(buf, off, length, m)
    got_buf = b.data.cpu().numpy()[: buf.size]
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
    assert np.array_equal(st.cpu().numpy(), want_st)
    assert np.array_equal(got_buf, want_buf)
    # an IP fragment's bytes past its IP header are byte-identical after any
    # fill (ip.cc:244-299: L4 is summed before ipv4::send cuts the datagram)
    stn = st.cpu().numpy()
    frag = np.nonzero(stn & native.ST_IPFRAG)[0]
    assert frag.size > 50
    for i in frag:
        o, L = int(off[i]), int(length[i])
        assert np.array_equal(got_buf[o + 20:o + L], buf[o + 20:o + L]), f"fragment {i} payload written"
    assert not np.any(stn[frag] & native.ST_L4_OK)
    if m & native.FILL_ICMP_ECHO:  # echo requests became replies; every other ICMP frame is untouched
        icmp = [i for i in range(off.size) if length[i] >= 20 and buf[int(off[i]) + 9] == 1]
        replies = [i for i in icmp if stn[i] & native.ST_L4_OK]
        assert len(replies) > 20
        for i in icmp:
            o, L = int(off[i]), int(length[i])
            ihl4 = 4 * (int(buf[o]) & 0xF)
            if i in replies:
                assert buf[o + ihl4] == 8 and got_buf[o + ihl4] == 0 and got_buf[o + ihl4 + 1] == 0
            else:
                assert np.array_equal(got_buf[o + 20:o + L], buf[o + 20:o + L])
    if m & (native.FILL_L4 | native.FILL_ICMP_ECHO):
        # the filled frames verify: receive path (ip.cc:121-127, udp/tcp verify) accepts them
        got, vst = _frames(dev, got_buf, off, length)
        stored = want_st & 2 != 0
        assert np.all(vst[stored] & 2)
        if m & native.FILL_IP:
            assert np.all(vst[want_st & 1 != 0] & 1)


def test_frames_on_tx_frames(dev):
    """sccsum_ipv4_frames (the rx verify path) on the tx generator's odd
    frames — UDP / TCP / ICMP, options, Ethernet padding, truncation, runts,
    garbage checksum fields, odd offsets — against the oracle."""
    rng = np.random.default_rng(0xF222)
    buf, off, length = _tx_frames(rng, 1500)
    got, st = _frames(dev, buf, off, length)
    want, want_st = oracle.batch_ipv4(buf, off, length)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)


def _packed_tx_frames(rng, n, gaps=(0,)):
    """ihl-5 UDP / TCP frames packed back to back (gap 0 mostly), lengths at
    the whole-unit store thresholds (64, 96) and around the field offsets,
    every start alignment: neighbours share the 16-byte units holding fields."""
    choices = [20, 21, 27, 28, 29, 37, 38, 39, 40, 47, 48, 63, 64, 65, 79, 80, 95, 96, 97, 100, 128, 576, 1500]
    frames = []
    fw = synth.frag_words(rng, n, frac=0.15)
    for i in range(n):
        L = int(rng.choice(choices))
        proto = int(rng.choice([17, 6]))
        f = rng.integers(0, 256, size=L, dtype=np.uint8)
        f[0] = 0x45
        f[2], f[3] = L >> 8, L & 0xFF
        f[6], f[7] = int(fw[i]) >> 8, int(fw[i]) & 0xFF
        f[9] = proto
        frames.append(f)
    length = np.array([f.size for f in frames], np.uint32)
    off = np.empty(n, np.uint64)
    pos = 5
    for i in range(n):
        pos += int(rng.choice(gaps))
        off[i] = pos
        pos += int(length[i])
    buf = rng.integers(0, 256, size=pos + 7, dtype=np.uint8)
    for i in range(n):
        buf[int(off[i]): int(off[i]) + int(length[i])] = frames[i]
    return buf, off, length


@pytest.mark.parametrize("gaps", [(0,), (0, 0, 0, 1, 3, 16)], ids=["contiguous", "mostly_contiguous"])
def test_ipv4_fill_whole_unit_stores(dev, gaps, fill_passes):
    """In-place fill rewrites the 16-byte units holding the fields whole where
    no other frame writes their bytes: byte-exact against the oracle on packed
    frames whose neighbours share those units (short frames, lengths at the
    64 / 96-byte thresholds, every alignment, shuffled tile boundaries)."""
    rng = np.random.default_rng(0xF333 + len(gaps))
    buf, off, length = _packed_tx_frames(rng, 6000, gaps)
    m = native.FILL_IP | native.FILL_L4
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_fill(b, m, out2=out2, status=st)
    torch.cuda.synchronize()
    want_buf, want_out2, want_st = oracle.batch_ipv4_fill(buf, off, length, m)
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
    assert np.array_equal(st.cpu().numpy(), want_st)
    got_buf = b.data.cpu().numpy()[: buf.size]
    bad = np.nonzero(got_buf != want_buf)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


@pytest.mark.parametrize("shape", ["ring_overflow", "static_order", "one_wave_tiles"])
def test_ipv4_fill_tile_shapes(dev, kernel_variant, shape):
    """The in-place fill under other tile shapes: one-packet tiles on a
    1-block-per-CU grid (~50 tiles per wave), the static tile order (no
    counter slot), the plain 64-packet cap.  No out2: the generate pass hands
    its values to the store pass through the library's stream-ordered
    scratch (the production call).  Byte-exact against the oracle."""
    if kernel_variant not in (14, 15, 16):
        pytest.skip("the fill runs the flat kernel")
    lib = native.load()
    rng = np.random.default_rng(0xD2A1)
    buf, off, length = _tx_frames(rng, 50000 if shape != "one_wave_tiles" else 8000)
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    try:
        if shape == "ring_overflow":
            native.check(lib.sccsum_set_blocks_per_cu(1), "blocks")
            native.check(lib.sccsum_set_tile_packets(1), "tile packets")
        elif shape == "static_order":
            native.check(lib.sccsum_set_dynamic_tiles(0), "static")
        else:
            native.check(lib.sccsum_set_tile_bytes(0), "tile bytes")
        for _ in range(2):  # a repeated fill is idempotent
            batch.ipv4_fill(b, m)
        torch.cuda.synchronize()
    finally:
        lib.sccsum_set_blocks_per_cu(8)
        lib.sccsum_set_tile_packets(64)
        lib.sccsum_set_dynamic_tiles(1)
        lib.sccsum_set_tile_bytes(49152)
    want_buf, _, _ = oracle.batch_ipv4_fill(buf, off, length, m)
    got_buf = b.data.cpu().numpy()[: buf.size]
    bad = np.nonzero(got_buf != want_buf)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def test_ipv4_fill_full_scale_no_out2(dev, kernel_variant):
    """cfg 2 tx at full size in the production form (no out2, no status):
    every frame verifies afterwards and the fields equal classic generate
    (the values cross between the passes in the library's scratch)."""
    from seastar_amd import devsynth

    if kernel_variant in (1, 2):
        pytest.skip("the fill runs the flat kernel")

    b = devsynth.udp_frames(1 << 20, 1500, seed=78, device=dev)
    gen = batch.ipv4_frames(b).clone()  # fields are 0 here: classic generate
    f = b.data[: b.n * 1500].view(b.n, 1500)
    f[:, 10:12] = 0x5A
    f[:, 26:28] = 0xC3
    batch.ipv4_fill(b, native.FILL_IP | native.FILL_L4)
    got = torch.stack([f[:, 10:12].contiguous().view(torch.int16).view(-1),
                       f[:, 26:28].contiguous().view(torch.int16).view(-1)], dim=1)
    assert torch.equal(got, gen)
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_frames(b, status=st)
    assert int((st == 3).sum()) == b.n


def test_ipv4_fill_full_scale_udp1500(dev):
    """cfg 2 at full size: fill(IP|L4) on frames with garbage checksum fields
    stores exactly what generate-on-zeroed-fields computes, and every frame verifies."""
    from seastar_amd import devsynth

    b = devsynth.udp_frames(1 << 20, 1500, seed=77, device=dev)
    gen = batch.ipv4_frames(b).clone()  # fields are 0 here: classic generate
    f = b.data[: b.n * 1500].view(b.n, 1500)
    f[:, 10:12] = 0xA5  # garbage in both fields
    f[:, 26:28] = 0x3C
    out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
    batch.ipv4_fill(b, native.FILL_IP | native.FILL_L4, out2=out2)
    assert torch.equal(out2.view(b.n, 2), gen)
    assert torch.equal(f[:, 10:12].contiguous().view(torch.int16).view(-1), gen[:, 0].contiguous())
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_frames(b, status=st)
    assert int((st == 3).sum()) == b.n


@pytest.mark.parametrize("mode", [0, 1], ids=["dispatch", "reassembled"])
def test_rss_standalone_and_fused(dev, mode, kernel_variant):
    """Toeplitz RSS (toeplitz.hh:78-98 over the stack's forward_hash) per frame:
    sccsum_ipv4_rss and the fused sccsum_ipv4_frames_rss vs the oracle, on
    fragments, options, ICMP/other protocols, padded / truncated / short frames
    at odd offsets; the fused pass leaves the checksums and status unchanged."""
    if kernel_variant not in (1, 14, 15, 16):
        pytest.skip("RSS exercised with the simple and flat families")
    rss = json.load(open(os.path.join(GOLDEN, "rss.json")))
    buf, off, lens = synth.rss_frames(5000, seed=21)
    # the last frame ends exactly at a 16-aligned buffer end (the padded-read guard)
    end = (int(off[-1] + lens[-1]) + 15) & ~15
    lens[-1] = end - int(off[-1])
    buf = buf[:end]
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    ref2, ref_st = _frames(dev, buf, off, lens)
    for key in (batch.RSS_KEY_40, bytes.fromhex(rss["cases"][0]["key"]), bytes(range(7, 15))):
        want, want_st = oracle.batch_ipv4_rss(buf, off, lens, key=key, mode=mode)
        st = torch.empty(b.n, dtype=torch.uint8, device=dev)
        got = batch.ipv4_rss(b, key=key, mode=mode, status=st)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want)
        assert np.array_equal(st.cpu().numpy() & 4, want_st & 4)
        fst = torch.empty(b.n, dtype=torch.uint8, device=dev)
        out2, h = batch.ipv4_frames_rss(b, key=key, mode=mode, status=fst)
        torch.cuda.synchronize()
        assert np.array_equal(h.cpu().numpy().view(np.uint32), want)
        assert np.array_equal(batch.as_u16(out2), ref2) and np.array_equal(fst.cpu().numpy(), ref_st)


def test_rss_errors(dev):
    lib = native.load()
    k = (ctypes.c_uint8 * 3)(1, 2, 3)
    b = batch.PacketBatch.from_host(np.zeros(64, np.uint8), np.zeros(1, np.uint64), np.full(1, 40, np.uint32),
                                    device=dev)
    h = torch.empty(1, dtype=torch.int32, device=dev)
    args = (batch.ctypes_ptr(b.data), b.bytes_len, batch.ctypes_ptr(b.off), batch.ctypes_ptr(b.length))
    assert lib.sccsum_ipv4_rss(*args, ctypes.addressof(k), 3, 0, batch.ctypes_ptr(h), None, 1, None) == native.SCCSUM_EINVAL
    k5 = (ctypes.c_uint8 * 5)(1, 2, 3, 4, 5)
    assert lib.sccsum_ipv4_rss(*args, ctypes.addressof(k5), 5, 2, batch.ctypes_ptr(h), None, 1, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_rss(*args, ctypes.addressof(k5), 5, 0, None, None, 1, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_rss(*args, ctypes.addressof(k5), 5, 0, batch.ctypes_ptr(h), None, 1, None) == native.SCCSUM_OK
    torch.cuda.synchronize()


def test_packets_over_128k(dev, kernel_variant):
    """Packets over 128 KiB leave the fast path for the exact redo (phase D);
    their IPv4 header, pseudo-header and RSS inputs still come from the frame's
    own head units.  Mixed with short frames in one tile; verify, spans, fused
    RSS and in-place generate."""
    lens = np.array([140_000, 1500, 131_073, 131_072, 64, 200_001, 1500, 300_000, 9000, 131_200], np.uint32)
    buf, off, lens, _ = synth.mixed_udp_frames(lens.size, seed=91, max_gap=3, lengths=lens)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    got, st = _frames(dev, buf, off, lens)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)
    assert np.array_equal(_spans(dev, buf, off, lens), oracle.batch_spans(buf, off, lens))
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    want_h, _ = oracle.batch_ipv4_rss(buf, off, lens)
    out2, h = batch.ipv4_frames_rss(b)
    torch.cuda.synchronize()
    assert np.array_equal(h.cpu().numpy().view(np.uint32), want_h)
    assert np.array_equal(batch.as_u16(out2), want)
    m = native.FILL_IP | native.FILL_L4
    out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
    stf = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_fill(b, m, out2=out2, status=stf)
    torch.cuda.synchronize()
    want_buf, want_out2, want_stf = oracle.batch_ipv4_fill(buf, off, lens, m)
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
    assert np.array_equal(stf.cpu().numpy(), want_stf)
    assert np.array_equal(b.data.cpu().numpy()[: buf.size], want_buf)


def test_host_pipeline_strided_short_last_row(dev, kernel_variant):
    """gather = 2 where the caller's buffer ends right after a short last
    packet: the 2D copy reads every row W bytes wide, so that row goes in a
    chunk of its own and nothing is read past the buffer."""
    if kernel_variant not in (1, 15):
        pytest.skip("pipeline chunking is kernel independent")
    from seastar_amd import pipeline

    rng = np.random.default_rng(41)
    n = 300
    lens = rng.integers(200, 600, size=n).astype(np.uint32)
    lens[-1] = 20
    off = np.arange(n, dtype=np.uint64) * 640 + 64
    end = int(off[-1]) + 20
    pool = pipeline.pinned_empty(end + 4096)
    pool[:] = rng.integers(0, 256, size=pool.size, dtype=np.uint8)
    seeds = rng.integers(0, 65536, n).astype(np.uint32)
    want = oracle.batch_spans(pool[:end], off, lens, seeds)
    pl = pipeline.HostPipeline(0, chunk_bytes=1 << 20, chunk_packets=128, depth=2)
    got = pl.run(native.PIPE_SPANS, pool[:end], off, lens, seeds=seeds, gather=native.GATHER_STRIDED)
    pl.close()
    assert np.array_equal(got, want)


def test_many_launches_in_flight_streams_and_graphs(dev, kernel_variant):
    """Tile counters are per stream: 600 launches queued on one stream without
    a sync (past the old 256-launch ring), 24 streams interleaved, and a
    launch captured in a HIP graph and replayed (static tile order) — every
    result exact."""
    if kernel_variant not in (15, 16):
        pytest.skip("tile dequeue lives in the flat kernel")
    buf, off, lens, _ = synth.mixed_udp_frames(20_000, seed=61, max_gap=3)
    want, want_st = oracle.batch_ipv4(buf, off, lens, nthreads=8)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    outs = [torch.empty(2 * b.n, dtype=torch.int16, device=dev) for _ in range(8)]
    s0 = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s0):
        for k in range(600):
            batch.ipv4_frames(b, out2=outs[k % 8])
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
    streams = [torch.cuda.Stream(device=dev) for _ in range(24)]
    souts = [torch.empty(2 * b.n, dtype=torch.int16, device=dev) for _ in streams]
    for rep in range(5):
        for s, o in zip(streams, souts):
            batch.ipv4_frames(b, out2=o, stream=s)
    torch.cuda.synchronize()
    for o in souts:
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
    g = torch.cuda.CUDAGraph()
    gout = torch.zeros(2 * b.n, dtype=torch.int16, device=dev)
    gst = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    cs = torch.cuda.Stream(device=dev)
    with torch.cuda.graph(g, stream=cs):
        batch.ipv4_frames(b, out2=gout, status=gst, stream=cs)
    for _ in range(3):
        gout.zero_()
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(batch.as_u16(gout).reshape(-1, 2), want)
    assert np.array_equal(gst.cpu().numpy(), want_st)


@pytest.mark.parametrize("path", ["c_abi", "wrapper"])
def test_fill_without_out2_in_a_graph(dev, kernel_variant, path, fill_passes):
    """sccsum_ipv4_fill with no d_out2, captured in a HIP graph.  Through the
    C-ABI with d_out2 = NULL the library's scratch is a stream-ordered
    allocation (a graph memory node); the Python wrapper passes a scratch from
    torch's caching allocator instead.  Either way the call stays
    capturable, and each replay over freshly restored frames stores exactly
    the oracle's fields."""
    if kernel_variant not in (15, 16):
        pytest.skip("the fill runs the flat kernel")
    rng = np.random.default_rng(0x6A1)
    buf, off, length = _tx_frames(rng, 3000)
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    orig = b.data.clone()
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    want_buf, _, _ = oracle.batch_ipv4_fill(buf, off, length, m)
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cs):
        if path == "c_abi":
            batch.prepare_call("sccsum_ipv4_fill", b.data, b.bytes_len, b.off, b.length, None, None, b.n, b.max_len,
                               m)(cs)
        else:
            batch.ipv4_fill(b, m, stream=cs)
    for _ in range(3):
        b.data.copy_(orig)
        g.replay()
        torch.cuda.synchronize()
        got = b.data.cpu().numpy()[: buf.size]
        bad = np.nonzero(got != want_buf)[0]
        assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def test_multi_batch_launch(dev, kernel_variant):
    """sccsum_ipv4_frames_multi / sccsum_spans_multi: 16 independent batches in
    one launch (empty, 1 packet, 1500 B frames, Zipf frames at odd offsets,
    malformed frames, packets over 128 KiB, seeded spans) — each batch's
    outputs exactly what its own launch gives, and the oracle's."""
    rng = np.random.default_rng(71)
    items, want = [], []
    for i in range(16):
        kind = i % 5
        if kind == 0:
            buf, off, lens, _ = synth.udp_ipv4_frames(int(rng.integers(0, 3)) * 700, 1500, seed=100 + i)
        elif kind == 1:
            buf, off, lens, _ = synth.mixed_udp_frames(int(rng.integers(1, 900)), seed=200 + i, max_gap=3)
        elif kind == 2:
            buf, off, length = _tx_frames(rng, 300)
            lens = length
        elif kind == 3:
            lens = np.array([140_000, 1500, 64], np.uint32)
            buf, off, lens, _ = synth.mixed_udp_frames(3, seed=300 + i, lengths=lens)
        else:
            buf, off, lens, _ = synth.udp_ipv4_frames(1, 200, seed=400 + i)
        if lens.size == 0:
            buf, off = np.zeros(16, np.uint8), np.zeros(0, np.uint64)
        b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
        st = torch.empty(max(b.n, 1), dtype=torch.uint8, device=dev)
        items.append((b, None, st))
        want.append(oracle.batch_ipv4(buf, off, lens) if lens.size else (np.zeros((0, 2), np.uint16), np.zeros(0, np.uint8)))
    outs = batch.ipv4_frames_multi(items)
    torch.cuda.synchronize()
    for (b, _, st), o, (w, ws) in zip(items, outs, want):
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), w)
        assert np.array_equal(st[: b.n].cpu().numpy(), ws)
    # spans with seeds, 16 batches of Zipf lengths
    sitems, swant = [], []
    for i in range(16):
        lens = synth.zipf_lengths(int(rng.integers(0, 400)), seed=500 + i)
        off, total = synth.pack(lens, seed=600 + i, max_gap=5)
        buf = rng.integers(0, 256, size=max(int(total), 16), dtype=np.uint8)
        seeds = rng.integers(0, 65536, size=lens.size).astype(np.uint32)
        b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
        sd = torch.from_numpy(seeds.view(np.int32)).to(dev) if lens.size else None
        sitems.append((b, None, None, sd))
        swant.append(oracle.batch_spans(buf, off, lens, seeds) if lens.size else np.zeros(0, np.uint16))
    souts = batch.spans_multi(sitems)
    torch.cuda.synchronize()
    for o, w in zip(souts, swant):
        assert np.array_equal(batch.as_u16(o), w)


@pytest.mark.parametrize("tile_bytes,tile_packets", [(0, 64), (0, 1), (0, 7), (1500, 64), (49152, 64), (49152, 13),
                                                     (1 << 20, 64)])
def test_tile_shapes_match_oracle(dev, kernel_variant, tile_bytes, tile_packets):
    """The flat kernel's tile sizing (bytes target, packet cap) changes only
    the schedule: 1500 B frames, Zipf frames and 64 KiB spans match the
    oracle under every shape (the default is 49152 B / 64)."""
    if kernel_variant not in (15, 16):
        pytest.skip("tile shapes exercised on the default flat forms")
    lib = native.load()
    native.check(lib.sccsum_set_tile_bytes(tile_bytes), "tile_bytes")
    native.check(lib.sccsum_set_tile_packets(tile_packets), "tile_packets")
    try:
        buf, off, lens, _ = synth.udp_ipv4_frames(3000, 1500, seed=91)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        buf, off, lens, _ = synth.mixed_udp_frames(4000, seed=92, max_gap=3)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        rng = np.random.default_rng(93)
        lens = np.full(24, 65536, np.uint32)
        lens[::5] = 65535
        off, total = synth.pack(lens, seed=94, max_gap=2)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        seeds = rng.integers(0, 65536, lens.size).astype(np.uint32)
        assert np.array_equal(_spans(dev, buf, off, lens, seeds), oracle.batch_spans(buf, off, lens, seeds))
    finally:
        native.check(lib.sccsum_set_tile_bytes(49152), "tile_bytes")
        native.check(lib.sccsum_set_tile_packets(64), "tile_packets")


def test_verify_only_frames(dev, kernel_variant):
    """Frames with no d_out2 and a status array (verify only): the status bits
    equal the oracle's, single and multi launch; no d_out2 and no status is
    refused."""
    rng = np.random.default_rng(77)
    buf, off, lens = _tx_frames(rng, 700)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
    got = batch.verify_frames(b, st)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want_st)
    buf2, off2, lens2, _ = synth.mixed_udp_frames(900, seed=78, max_gap=3)
    want2, want_st2 = oracle.batch_ipv4(buf2, off2, lens2)
    b2 = batch.PacketBatch.from_host(buf2, off2, lens2, device=dev)
    st.fill_(0xEE)
    st2 = torch.full((b2.n,), 0xEE, dtype=torch.uint8, device=dev)
    o2 = torch.empty(2 * b2.n, dtype=torch.int16, device=dev)
    batch.prepare_ipv4_frames_multi([(b, None, st), (b2, o2, st2)])(torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), want_st) and np.array_equal(st2.cpu().numpy(), want_st2)
    assert np.array_equal(batch.as_u16(o2).reshape(-1, 2), want2)
    lib = native.load()
    rc = lib.sccsum_ipv4_frames(batch.ctypes_ptr(b.data), b.bytes_len, batch.ctypes_ptr(b.off),
                                batch.ctypes_ptr(b.length), None, None, b.n, b.max_len, None)
    assert rc == native.SCCSUM_EINVAL


@pytest.mark.parametrize("short", [1, 0])
def test_slot_layout_one_run_per_packet(dev, kernel_variant, short):
    """Packets in 4 KiB slots at every start alignment (mbuf-like: every
    packet its own run): lengths 0..3071 give runs of 1..193 units, so a
    run's one chunk is cut to 2, 4, 8 or 16 rows (short chunks, the default)
    or always full; spans and frames against the oracle."""
    lib = native.load()
    native.check(lib.sccsum_set_short_chunks(short), "short_chunks")
    try:
        rng = np.random.default_rng(800 + short)
        lens = np.arange(0, 3072, dtype=np.uint32)
        off = (np.arange(lens.size, dtype=np.uint64) * 4096 + 256 + (np.arange(lens.size) % 16)).astype(np.uint64)
        buf = rng.integers(0, 256, size=lens.size * 4096 + 64, dtype=np.uint8)
        seeds = rng.integers(0, 65536, lens.size).astype(np.uint32)
        assert np.array_equal(_spans(dev, buf, off, lens, seeds), oracle.batch_spans(buf, off, lens, seeds))
        fl = np.maximum(lens, 20).astype(np.uint32)
        fbuf = buf.copy()
        fw = synth.frag_words(rng, fl.size, frac=0.1)
        for i in range(fl.size):  # IPv4/UDP headers, ip_len = frame length, some fragments
            o, L = int(off[i]), int(fl[i])
            fbuf[o], fbuf[o + 2], fbuf[o + 3], fbuf[o + 9] = 0x45, L >> 8, L & 0xFF, 17
            fbuf[o + 6], fbuf[o + 7] = int(fw[i]) >> 8, int(fw[i]) & 0xFF
        got, st = _frames(dev, fbuf, off, fl)
        want, want_st = oracle.batch_ipv4(fbuf, off, fl)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
    finally:
        native.check(lib.sccsum_set_short_chunks(1), "short_chunks")


def test_slot_layout_short_slow_frames_at_the_buffer_end(dev, kernel_variant):
    """20-byte frames the fast path hands to the exact redo (options, an IP
    length that is not the frame's, fragments) in a sparse slot layout, at
    every dword phase, the last one ending exactly at bytes_len (a multiple of
    16, frame start 12 mod 16): the redo reads the header from the frame and
    must stay inside it (sccsum.h's readable extent is
    roundup(bytes_len, 16)); results against the oracle."""
    rng = np.random.default_rng(4242)
    n = 96
    fl = np.full(n, 20, dtype=np.uint32)
    off = (np.arange(n, dtype=np.uint64) * 2048 + 512 + (np.arange(n) % 16)).astype(np.uint64)
    total = int(off[-2]) + 2048
    total += (-total) % 16
    off[-1] = total - 20  # ends exactly at bytes_len
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    for i in range(n):
        o = int(off[i])
        ihl = 5 + (i % 3 == 0)                       # options claimed: 4*ihl past ip_len -> malformed
        ip_len = 20 + (i % 3 == 1) * (1 + i % 5)     # longer than the frame -> malformed
        buf[o], buf[o + 2], buf[o + 3], buf[o + 9] = 0x40 | ihl, ip_len >> 8, ip_len & 0xFF, (17, 6, 1)[i % 3]
        buf[o + 6], buf[o + 7] = (0x20 if i % 7 == 0 else 0), 0
    assert int(off[-1]) % 16 == 12 and int(off[-1]) + 20 == buf.size
    got, st = _frames(dev, buf, off, fl)
    want, want_st = oracle.batch_ipv4(buf, off, fl)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)


@pytest.mark.parametrize("bpc,tile_packets", [(8, 64), (1, 5), (3, 1)])
def test_static_tile_order_matches_oracle(dev, kernel_variant, bpc, tile_packets):
    """Static round-robin tiles (no dequeue counters: what a graph capture or a
    stream past the slot cap gets) change only the schedule: frames, a
    multi-queue launch and spans match the oracle on grids of 1-8 blocks per CU."""
    if kernel_variant not in (15, 16):
        pytest.skip("tile orders exercised on the default flat forms")
    lib = native.load()
    native.check(lib.sccsum_set_dynamic_tiles(0), "dynamic")
    native.check(lib.sccsum_set_blocks_per_cu(bpc), "blocks_per_cu")
    native.check(lib.sccsum_set_tile_packets(tile_packets), "tile_packets")
    try:
        buf, off, lens, _ = synth.mixed_udp_frames(20000, seed=700 + bpc, max_gap=3)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        items, wants = [], []
        for q, n in enumerate([5000, 3, 12000]):
            buf, off, lens, _ = synth.mixed_udp_frames(n, seed=710 + q, max_gap=1)
            items.append((batch.PacketBatch.from_host(buf, off, lens, device=dev), None,
                          torch.empty(n, dtype=torch.uint8, device=dev)))
            wants.append(oracle.batch_ipv4(buf, off, lens))
        outs = batch.ipv4_frames_multi(items)
        torch.cuda.synchronize()
        for o, it, (w, wst) in zip(outs, items, wants):
            assert np.array_equal(batch.as_u16(o).reshape(-1, 2), w)
            assert np.array_equal(it[2].cpu().numpy(), wst)
        rng = np.random.default_rng(720)
        lens = rng.integers(0, 5000, 30000).astype(np.uint32)
        off, total = synth.pack(lens, seed=721, max_gap=2)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        assert np.array_equal(_spans(dev, buf, off, lens), oracle.batch_spans(buf, off, lens))
    finally:
        native.check(lib.sccsum_set_dynamic_tiles(1), "dynamic")
        native.check(lib.sccsum_set_blocks_per_cu(8), "blocks_per_cu")
        native.check(lib.sccsum_set_tile_packets(64), "tile_packets")


@pytest.mark.parametrize("policy", [0, 1, 2, 3, 4])
def test_out_policies_match_oracle(dev, kernel_variant, policy):
    """The result stores' cache policy (sccsum_set_out_policy; nt by default)
    changes nothing in the results: frames with and without status, spans."""
    if kernel_variant not in (15, 16):
        pytest.skip("the policy applies to the flat kernel")
    lib = native.load()
    native.check(lib.sccsum_set_out_policy(policy), "out_policy")
    try:
        rng = np.random.default_rng(500 + policy)
        buf, off, lens = _tx_frames(rng, 900)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        lens = rng.integers(0, 3000, 3001).astype(np.uint32)
        off, total = synth.pack(lens, seed=501, max_gap=7)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        got, st = _spans(dev, buf, off, lens, with_status=True)
        want = oracle.batch_spans(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, (want == 0).astype(np.uint8))
    finally:
        native.check(lib.sccsum_set_out_policy(1), "out_policy")


@pytest.mark.parametrize("split,quarters,tile_packets,bpc",[(2, 4, 64, 8), (4, 4, 64, 8), (8, 4, 64, 8),
                                                             (4, 1, 7, 1), (8, 2, 13, 1), (4, 64, 64, 8),
                                                             (2, 0, 64, 8)])
def test_tail_split_matches_oracle(dev, kernel_variant, split, quarters, tile_packets, bpc):
    """The tail split (the launch's last tiles cut into sub-tiles, some of them
    empty when a queue's last tile is short) changes only the schedule: single
    and multi-queue launches of frames and spans match the oracle, with the
    split point inside the launch (small grid, 7 / 13-packet tiles) or before
    its first tile."""
    if kernel_variant not in (15, 16):
        pytest.skip("tail split exercised on the default flat forms")
    lib = native.load()
    native.check(lib.sccsum_set_tail_split(split, quarters), "tail_split")
    native.check(lib.sccsum_set_tile_packets(tile_packets), "tile_packets")
    native.check(lib.sccsum_set_blocks_per_cu(bpc), "blocks_per_cu")
    try:
        buf, off, lens, _ = synth.udp_ipv4_frames(3001, 1500, seed=191)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        buf, off, lens, _ = synth.mixed_udp_frames(5003, seed=192, max_gap=3)
        got, st = _frames(dev, buf, off, lens)
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        items, wants = [], []
        for q, n in enumerate([1, 257, 3000, 63, 1999]):
            buf, off, lens, _ = synth.mixed_udp_frames(n, seed=300 + q, max_gap=2)
            items.append((batch.PacketBatch.from_host(buf, off, lens, device=dev), None,
                          torch.empty(n, dtype=torch.uint8, device=dev)))
            wants.append(oracle.batch_ipv4(buf, off, lens))
        outs = batch.ipv4_frames_multi(items)
        torch.cuda.synchronize()
        for o, it, (w, wst) in zip(outs, items, wants):
            assert np.array_equal(batch.as_u16(o).reshape(-1), w.reshape(-1))
            assert np.array_equal(it[2].cpu().numpy(), wst)
        rng = np.random.default_rng(193)
        lens = rng.integers(0, 9000, 4001).astype(np.uint32)
        off, total = synth.pack(lens, seed=194, max_gap=5)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        seeds = rng.integers(0, 65536, lens.size).astype(np.uint32)
        assert np.array_equal(_spans(dev, buf, off, lens, seeds), oracle.batch_spans(buf, off, lens, seeds))
    finally:
        native.check(lib.sccsum_set_tail_split(1, 4), "tail_split")
        native.check(lib.sccsum_set_tile_packets(64), "tile_packets")
        native.check(lib.sccsum_set_blocks_per_cu(8), "blocks_per_cu")


@pytest.mark.parametrize("seed", [101, 202, 303])
def test_random_layouts_shuffled_overlapping(dev, kernel_variant, seed):
    """Offsets in any order: shuffled, overlapping spans (packets sharing
    bytes), duplicates, zero lengths, spans over 128 KiB (the exact redo) and
    runs broken at random — spans with seeds and frames, against the oracle."""
    rng = np.random.default_rng(seed)
    total = 3 << 20
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    n = 3000
    kinds = rng.random(n)
    lens = np.where(kinds < 0.05, 0, np.where(kinds < 0.07, rng.integers(131073, 300000, n),
                                               rng.integers(1, 9001, n))).astype(np.uint32)
    off = np.array([int(rng.integers(0, total - int(L) + 1)) for L in lens], np.uint64)
    off[10:20] = off[0]  # duplicates of one packet
    lens[10:20] = lens[0]
    order = rng.permutation(n)
    off, lens = off[order], lens[order]
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(_spans(dev, buf, off, lens, seeds), oracle.batch_spans(buf, off, lens, seeds))
    # frames: the same layout with IPv4 headers written at each start (later writes win, as on the host)
    fb = buf.copy()
    fw = synth.frag_words(rng, n, frac=0.1)
    for i in range(n):
        L = int(lens[i])
        if L >= 20:
            o = int(off[i])
            fb[o] = 0x45
            fb[o + 2], fb[o + 3] = (L >> 8) & 0xFF, L & 0xFF
            fb[o + 6], fb[o + 7] = int(fw[i]) >> 8, int(fw[i]) & 0xFF
            fb[o + 9] = 17 if i % 2 else 6
    got, st = _frames(dev, fb, off, lens)
    want, want_st = oracle.batch_ipv4(fb, off, lens)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)


@pytest.mark.parametrize("case", ["zipf_frames", "spans_zero_lengths", "spans_shuffled", "fill_tx_frames"])
def test_full_tiles_match_oracle(dev, kernel_variant, case):
    """Full 64-packet tiles.  The small cases above get tiles of a few
    packets (B = n / waves); a grid of one block per CU (1 024 waves) and
    ~100 K packets fills every tile to the cap, so runs span whole tiles,
    last tiles end ragged, and slow-path packets (IP options, over-long spans)
    sit among 63 fast ones: Zipf frames, spans with zero lengths, shuffled
    spans (one run per packet), in-place fill of the tx generator's frames.
    (This test also carried the round-2 A/B of two packets per lane,
    profiles/r02_ab_p2.log.)"""
    if kernel_variant not in (15, 16):
        pytest.skip("full tiles exercised on the default flat forms")
    lib = native.load()
    native.check(lib.sccsum_set_blocks_per_cu(1), "blocks_per_cu")
    native.check(lib.sccsum_set_tile_bytes(0 if case != "zipf_frames" else 49152), "tile_bytes")
    rng = np.random.default_rng(0x7A11)
    try:
        if case == "zipf_frames":
            buf, off, lens, _ = synth.mixed_udp_frames(150_000, seed=0x7A12, max_gap=3)
            got, st = _frames(dev, buf, off, lens)
            want, want_st = oracle.batch_ipv4(buf, off, lens)
            assert np.array_equal(got, want) and np.array_equal(st, want_st)
        elif case.startswith("spans"):
            n = 110_000
            lens = rng.integers(0, 3000, n).astype(np.uint32)
            lens[rng.random(n) < 0.05] = 0
            lens[rng.integers(0, n, 20)] = 140_000  # over kExactMax: phase D
            off, total = synth.pack(lens, seed=0x7A13, max_gap=2)
            if case == "spans_shuffled":  # every packet its own run (spans stay inside the buffer)
                order = rng.permutation(n)
                off, lens = off[order], lens[order]
            buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
            seeds = rng.integers(0, 65536, n).astype(np.uint32)
            assert np.array_equal(_spans(dev, buf, off, lens, seeds), oracle.batch_spans(buf, off, lens, seeds))
        else:
            m = native.FILL_IP | native.FILL_L4
            buf, off, length = _tx_frames(rng, 100_000)
            b = batch.PacketBatch.from_host(buf, off, length, device=dev)
            out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
            st = torch.empty(b.n, dtype=torch.uint8, device=dev)
            batch.ipv4_fill(b, m, out2=out2, status=st)
            torch.cuda.synchronize()
            want_buf, want_out2, want_st = oracle.batch_ipv4_fill(buf, off, length, m)
            assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
            assert np.array_equal(st.cpu().numpy(), want_st)
            assert np.array_equal(b.data.cpu().numpy()[: buf.size], want_buf)
    finally:
        native.check(lib.sccsum_set_blocks_per_cu(8), "blocks_per_cu")
        native.check(lib.sccsum_set_tile_bytes(49152), "tile_bytes")


@pytest.mark.parametrize("units", [1, 4, 8])
def test_run_align_matches_oracle(dev, kernel_variant, units):
    """Run extents started on 16 / 64 / 128-byte boundaries (sccsum_set_run_align;
    128 B is the default) change only which bytes a wave loads before a run's
    first packet: Zipf
    frames at odd offsets, a batch whose first packet sits in its first unit
    (the clamp), 65 535 B spans at odd offsets and shuffled spans match the
    oracle."""
    if kernel_variant not in (14, 15, 16):
        pytest.skip("run alignment applies to the flat forms")
    lib = native.load()
    native.check(lib.sccsum_set_run_align(units), "run_align")
    try:
        for gap in (0, 3):
            buf, off, lens, _ = synth.mixed_udp_frames(6000, seed=0xA11 + gap, max_gap=gap)
            got, st = _frames(dev, buf, off, lens)
            want, want_st = oracle.batch_ipv4(buf, off, lens)
            assert np.array_equal(got, want) and np.array_equal(st, want_st)
        rng = np.random.default_rng(0xA12)
        lens = np.full(40, 65535, np.uint32)
        off, total = synth.pack(lens, seed=0xA13, max_gap=5)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        assert np.array_equal(_spans(dev, buf, off, lens), oracle.batch_spans(buf, off, lens))
        lens = rng.integers(0, 2000, 20000).astype(np.uint32)
        off, total = synth.pack(lens, seed=0xA14, max_gap=2)
        order = rng.permutation(lens.size)
        off, lens = off[order], lens[order]
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        assert np.array_equal(_spans(dev, buf, off, lens), oracle.batch_spans(buf, off, lens))
        # a batch based 16 B past a 128 B boundary: the first runs' aligned start
        # would fall before the batch, so it is clamped to the batch's first unit
        buf, off, lens, _ = synth.mixed_udp_frames(3000, seed=0xA15)
        big = torch.zeros(buf.size + 64, dtype=torch.uint8, device=dev)
        big[16:16 + buf.size] = torch.from_numpy(buf).to(dev)
        b = batch.PacketBatch(data=big[16:], off=torch.from_numpy(off.astype(np.int64)).to(dev),
                              length=torch.from_numpy(lens.astype(np.int32)).to(dev), bytes_len=buf.size,
                              max_len=int(lens.max()))
        st = torch.empty(b.n, dtype=torch.uint8, device=dev)
        got = batch.as_u16(batch.ipv4_frames(b, status=st))
        torch.cuda.synchronize()
        want, want_st = oracle.batch_ipv4(buf, off, lens)
        assert np.array_equal(got, want) and np.array_equal(st.cpu().numpy(), want_st)
        # the same batch as the second queue of a multi launch: the clamp is per queue
        buf0, off0, lens0, _ = synth.mixed_udp_frames(2000, seed=0xA16)
        b0 = batch.PacketBatch.from_host(buf0, off0, lens0, device=dev)
        st0 = torch.empty(b0.n, dtype=torch.uint8, device=dev)
        st1 = torch.empty(b.n, dtype=torch.uint8, device=dev)
        o0, o1 = batch.ipv4_frames_multi([(b0, None, st0), (b, None, st1)])
        torch.cuda.synchronize()
        w0, ws0 = oracle.batch_ipv4(buf0, off0, lens0)
        assert np.array_equal(batch.as_u16(o0), w0) and np.array_equal(st0.cpu().numpy(), ws0)
        assert np.array_equal(batch.as_u16(o1), want) and np.array_equal(st1.cpu().numpy(), want_st)
    finally:
        native.check(lib.sccsum_set_run_align(8), "run_align")


def _fragmented_datagrams(rng, sizes, mtu=1500):
    """UDP / TCP datagrams of the given L4 sizes, checksummed whole by the
    oracle (udp.cc:184-195 / tcp.hh:1656-1694 run before ipv4::send) and cut
    into frames by synth.ipv4_fragment (ip.cc:283-294); the frames are packed
    at odd offsets.  Returns (buf, off, lens, dgrams) with dgrams[d] =
    (proto, src, dst, l4 bytes, [frame indices in offset order])."""
    frames, dgrams = [], []
    for d, size in enumerate(sizes):
        proto = 17 if d % 2 == 0 else 6
        src, dst = int(rng.integers(1, 2**32)), int(rng.integers(1, 2**32))
        l4 = rng.integers(0, 256, size=size, dtype=np.uint8)
        fo = 6 if proto == 17 else 16
        if proto == 17:
            l4[4], l4[5] = size >> 8, size & 0xFF
        else:
            l4[12] = 0x50
        l4[fo:fo + 2] = 0
        seed = oracle.pseudo_seed(src, dst, proto, size)
        c = oracle.batch_spans(l4, np.zeros(1, np.uint64), np.array([size], np.uint32), np.array([seed], np.uint32))
        l4[fo:fo + 2] = np.frombuffer(np.uint16(c[0]).tobytes(), np.uint8)
        idx = []
        for f in synth.ipv4_fragment(l4, proto, src, dst, mtu=mtu, ident=d):
            idx.append(len(frames))
            frames.append(f)
        dgrams.append((proto, src, dst, l4, idx))
    lens = np.array([f.size for f in frames], np.uint32)
    off = np.empty(lens.size, np.uint64)
    pos = 3
    for i in range(lens.size):
        pos += int(rng.integers(0, 4))
        off[i] = pos
        pos += int(lens[i])
    buf = rng.integers(0, 256, size=pos + 5, dtype=np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + f.size] = f
    return buf, off, lens, dgrams


DGRAM_SIZES = [8, 100, 1480, 1481, 2960, 2961, 4000, 9000, 30001, 65515, 65515, 12345]


def test_ip_fragments_rx_and_reassembled_l4(dev, kernel_variant):
    """rx (ip.cc:114-229): every fragment's IPv4 header is verified; a
    fragment claims no L4 value (SCCSUM_ST_IPFRAG, L4 word 0, never L4_OK);
    the L4 checksum of the reassembled datagram — its fragments' payloads in
    offset order, pseudo-header seed, no IP check (ip.cc:120-121) — verifies
    through sccsum_spans_desc, and a corrupted fragment fails its datagram."""
    rng = np.random.default_rng(0xF4A6)
    buf, off, lens, dgrams = _fragmented_datagrams(rng, DGRAM_SIZES)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    # the IP header checksums, as ipv4::send writes them per fragment
    batch.ipv4_fill(b, native.FILL_IP)
    torch.cuda.synchronize()
    rx = b.data.cpu().numpy()[: buf.size]
    got, st = _frames(dev, rx, off, lens)
    want, want_st = oracle.batch_ipv4(rx, off, lens)
    assert np.array_equal(got, want) and np.array_equal(st, want_st)
    for proto, src, dst, l4, idx in dgrams:
        if len(idx) == 1:
            assert st[idx[0]] == native.ST_OK | native.ST_L4_OK
        else:
            assert np.all(st[idx] == native.ST_OK | native.ST_IPFRAG) and np.all(got[idx, 1] == 0)
    # the reassembled datagrams: fragments summed where they lie (payload = frame + 20)
    base = b.data.data_ptr()
    src_a, dst_off, flen, first, doff, dlen, seeds = [], [], [], [0], [], [], []
    pos = 0
    for proto, s_ip, d_ip, l4, idx in dgrams:
        doff.append(pos)
        at = 0
        for i in idx:
            src_a.append(base + int(off[i]) + 20)
            dst_off.append(pos + at)
            flen.append(int(lens[i]) - 20)
            at += int(lens[i]) - 20
        first.append(len(src_a))
        dlen.append(at)
        seeds.append(oracle.pseudo_seed(s_ip, d_ip, proto, at))
        pos += at
    desc = torch.from_numpy(batch.make_desc(np.array(src_a, np.uint64), np.array(dst_off, np.uint32),
                                            np.array(flen, np.uint32)).view(np.uint8)).to(dev)
    args = (desc, torch.from_numpy(np.array(first, np.int32)).to(dev),
            torch.from_numpy(np.array(doff, np.int64)).to(dev), torch.from_numpy(np.array(dlen, np.int32)).to(dev),
            max(dlen))
    dst_t = torch.empty(len(dgrams), dtype=torch.uint8, device=dev)
    r = batch.spans_desc(*args, seeds=torch.from_numpy(np.array(seeds, np.uint32).view(np.int32)).to(dev),
                         status=dst_t)
    torch.cuda.synchronize()
    assert np.all(batch.as_u16(r) == 0) and np.all(dst_t.cpu().numpy() == native.ST_OK)
    # one payload byte of datagram 7's second fragment flipped: only that datagram fails
    j = dgrams[7][4][1]
    b.data[int(off[j]) + 100] ^= 0x41
    r = batch.as_u16(batch.spans_desc(*args, seeds=torch.from_numpy(np.array(seeds, np.uint32).view(np.int32)).to(dev)))
    torch.cuda.synchronize()
    assert r[7] != 0 and np.all(np.delete(r, 7) == 0)


def test_ip_fragments_fill(dev, kernel_variant):
    """tx (ip.cc:244-299): ipv4_fill over the frames of fragmented datagrams
    writes each fragment's IPv4 header checksum and nothing past its header —
    the first fragment's L4 checksum (computed over the whole datagram before
    the cut) and the later fragments' payload are byte-identical — while an
    unfragmented datagram gets both checksums; byte-exact against the oracle."""
    rng = np.random.default_rng(0xF4A7)
    buf, off, lens, dgrams = _fragmented_datagrams(rng, DGRAM_SIZES)
    for i in range(off.size):  # garbage in every checksum field a fill could write
        o = int(off[i])
        buf[o + 10:o + 12] = rng.integers(0, 256, 2)
    for proto, src, dst, l4, idx in dgrams:
        if len(idx) == 1:
            o = int(off[idx[0]]) + 20 + (6 if proto == 17 else 16)
            buf[o:o + 2] = rng.integers(0, 256, 2)
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out2 = torch.empty(2 * b.n, dtype=torch.int16, device=dev)
    st = torch.empty(b.n, dtype=torch.uint8, device=dev)
    batch.ipv4_fill(b, m, out2=out2, status=st)
    torch.cuda.synchronize()
    want_buf, want_out2, want_st = oracle.batch_ipv4_fill(buf, off, lens, m)
    got_buf = b.data.cpu().numpy()[: buf.size]
    assert np.array_equal(got_buf, want_buf)
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
    assert np.array_equal(st.cpu().numpy(), want_st)
    for proto, src, dst, l4, idx in dgrams:
        for k, i in enumerate(idx):
            o, L = int(off[i]), int(lens[i])
            if len(idx) > 1:
                assert np.array_equal(got_buf[o + 12:o + L], buf[o + 12:o + L])
        # the wire bytes after the fill are the datagram the L4 writer produced
        l4_wire = np.concatenate([got_buf[int(off[i]) + 20:int(off[i]) + int(lens[i])] for i in idx])
        assert np.array_equal(l4_wire, l4)


def test_scratch_on_a_side_stream(dev, kernel_variant):
    """ipv4_fill(FILL_L4) and fragments() on a stream that is not torch's
    current one: fragments() allocates its workspace, which is recorded on
    the launch stream, so allocations churned on the current stream meanwhile
    cannot take its block while the kernels still use it; the
    fill's values cross between its passes in the library's stream-ordered
    allocation on the launch stream.  Results byte-exact against the oracle."""
    if kernel_variant not in (1, 16):
        pytest.skip("scratch lifetime is kernel independent")
    rng = np.random.default_rng(0x5C1)
    buf, off, length = _tx_frames(rng, 4000)
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    fb, fo, fl, first = _frag_batch(rng, 3000, lambda i: [int(x) for x in rng.integers(1, 700, int(rng.integers(1, 6)))])
    d = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).to(dev)
    args = (d, fb.size, torch.from_numpy(fo.view(np.int64)).to(dev), torch.from_numpy(fl.view(np.int32)).to(dev),
            torch.from_numpy(first.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    for _ in range(3):
        batch.ipv4_fill(b, m, stream=side)
        got = batch.fragments(*args, stream=side)  # workspace allocated by the wrapper
        junk = [torch.full((1 << 20,), 7, dtype=torch.uint8, device=dev) for _ in range(8)]  # churn, current stream
        del junk
        side.synchronize()
    torch.cuda.synchronize()
    want_buf, _, _ = oracle.batch_ipv4_fill(buf, off, length, m)
    assert np.array_equal(b.data.cpu().numpy()[: buf.size], want_buf)
    assert np.array_equal(batch.as_u16(got), oracle.batch_fragments(fb, fo, fl, first))


@pytest.mark.parametrize("bpc,dynamic", [(8, 1), (1, 1), (2, 0)], ids=["grid", "one_block_per_cu", "static"])
def test_late_claim_form_matches_oracle(dev, kernel_variant, bpc, dynamic):
    """The U = 16 form reads its tile claims back a tile late for launches
    whose mean packet is 48 KiB or more (sccsum.hip flat_body LATE, cfg 4).
    Big spans and frames with tiny, empty, out-of-range and over-128 KiB
    packets among them (tiles that stream nothing claim after the run loop),
    seeds and status, on the full grid, one block per CU (more tiles per wave)
    and static tile order; and a launch with fewer tiles than waves."""
    if kernel_variant != 16:
        pytest.skip("the LATE form is the U = 16 flat kernel's")
    lib = native.load()
    native.check(lib.sccsum_set_blocks_per_cu(bpc), "blocks_per_cu")
    native.check(lib.sccsum_set_dynamic_tiles(dynamic), "dynamic")
    try:
        rng = np.random.default_rng(4000 + bpc)
        n = 1500
        lens = rng.integers(49152, 65537, n).astype(np.uint32)
        lens[rng.choice(n, 40, replace=False)] = rng.choice([0, 1, 2, 7, 19, 20, 64], 40)
        lens[rng.choice(n, 5, replace=False)] = [131_073, 140_000, 65_535, 200_001, 131_072]
        assert lens.mean() >= 49152
        off, total = synth.pack(lens, seed=4010 + bpc, max_gap=5)
        buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
        seeds = rng.integers(0, 65536, n).astype(np.uint32)
        bad = [3, 700]
        bad_off = off.copy()
        bad_off[bad] = total + 1  # out of range (the oracle has no buffer length: those two are checked apart)
        got, st = _spans(dev, buf, bad_off, lens, seeds, with_status=True)
        want = oracle.batch_spans(buf, off, lens, seeds)
        assert np.array_equal(np.delete(got, bad), np.delete(want, bad))
        assert np.array_equal(np.delete(st, bad), np.delete((want == 0).astype(np.uint8), bad))
        assert np.all(got[bad] == 0) and np.all(st[bad] == native.ST_RANGE)
        flens = np.clip(lens, 28, 65535).astype(np.uint32)  # (UDP frames: 28 B at least)
        fbuf, foff, flens, _ = synth.mixed_udp_frames(n, seed=4020 + bpc, max_gap=3, lengths=flens)
        got, st = _frames(dev, fbuf, foff, flens)
        want, want_st = oracle.batch_ipv4(fbuf, foff, flens)
        assert np.array_equal(got, want) and np.array_equal(st, want_st)
        small = lens[:37]  # fewer tiles than waves
        o2, t2 = synth.pack(small, seed=4030, max_gap=1)
        b2 = rng.integers(0, 256, size=int(t2), dtype=np.uint8)
        assert np.array_equal(_spans(dev, b2, o2, small), oracle.batch_spans(b2, o2, small))
    finally:
        native.check(lib.sccsum_set_blocks_per_cu(8), "blocks_per_cu")
        native.check(lib.sccsum_set_dynamic_tiles(1), "dynamic")
