"""Synthetic packet batches shaped like the native stack's traffic.

Frames are built byte-for-byte the way the reference builds them:
  IPv4 header  src/net/ip.cc:249-269  (ver 4, ihl 5, dscp/ecn 0, total length,
               id 0, frag 0, ttl 64, proto, csum 0, src, dst — network order)
  UDP header   src/net/udp.cc:178-182 (ports, length = UDP header + payload,
               cksum 0 from the value-initialised header, packet.hh:586-589)
  TCP header   include/seastar/net/tcp.hh:1621-1651, written by tcp_hdr::write
               (:261-282) with checksum 0 and data_offset = (20+options)/4.
Payload bytes are random.  Everything is deterministic in `seed`.
"""
from __future__ import annotations

import numpy as np

PROTO_TCP = 6
PROTO_UDP = 17
IPV4_HDR = 20
UDP_HDR = 8
TCP_HDR = 20


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def _put_be16(frames: np.ndarray, col: int, vals) -> None:
    vals = np.asarray(vals, dtype=np.uint32)
    frames[:, col] = (vals >> 8) & 0xFF
    frames[:, col + 1] = vals & 0xFF


def _put_be32(frames: np.ndarray, col: int, vals) -> None:
    vals = np.asarray(vals, dtype=np.uint64)
    for k in range(4):
        frames[:, col + k] = (vals >> (24 - 8 * k)) & 0xFF


def write_ipv4_header(frames: np.ndarray, total_len, proto: int, src, dst) -> None:
    """ipv4::send's header (ip.cc:249-269) into frames[:, 0:20], csum = 0."""
    frames[:, 0] = 0x45  # ver 4, ihl 5
    frames[:, 1] = 0
    _put_be16(frames, 2, total_len)
    frames[:, 4:8] = 0  # id 0, frag 0
    frames[:, 8] = 64
    frames[:, 9] = proto
    frames[:, 10:12] = 0
    _put_be32(frames, 12, src)
    _put_be32(frames, 16, dst)


def udp_ipv4_frames(n: int, frame_len: int = 1500, seed: int = 0x5EA57A2C):
    """n equal-length IPv4/UDP frames packed back to back; checksum fields 0.

    Returns (buf, off, length, meta) with meta = dict(src, dst) host-order."""
    assert frame_len >= IPV4_HDR + UDP_HDR
    rng = _rng(seed)
    frames = rng.integers(0, 256, size=(n, frame_len), dtype=np.uint8)
    src = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    dst = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    write_ipv4_header(frames, frame_len, PROTO_UDP, src, dst)
    _put_be16(frames, 20, rng.integers(1024, 65536, size=n))
    _put_be16(frames, 22, rng.integers(1, 65536, size=n))
    _put_be16(frames, 24, frame_len - IPV4_HDR)
    frames[:, 26:28] = 0
    off = np.arange(n, dtype=np.uint64) * frame_len
    length = np.full(n, frame_len, dtype=np.uint32)
    return frames.reshape(-1), off, length, {"src": src, "dst": dst}


def tcp_segments(n: int, seg_len: int, seed: int = 0x5EA57A2C, options_len: int = 0):
    """n TCP segments (header + options + payload, no IP header) packed back to
    back, checksum 0; meta has the host-order addresses for the pseudo-header."""
    assert seg_len >= TCP_HDR + options_len and options_len % 4 == 0
    rng = _rng(seed)
    segs = rng.integers(0, 256, size=(n, seg_len), dtype=np.uint8)
    _put_be16(segs, 0, rng.integers(1, 65536, size=n))
    _put_be16(segs, 2, rng.integers(1, 65536, size=n))
    _put_be32(segs, 4, rng.integers(0, 2**32, size=n, dtype=np.uint64))
    _put_be32(segs, 8, rng.integers(0, 2**32, size=n, dtype=np.uint64))
    segs[:, 12] = ((TCP_HDR + options_len) // 4) << 4
    segs[:, 13] = 0x10  # ACK
    _put_be16(segs, 14, rng.integers(0, 65536, size=n))
    segs[:, 16:18] = 0
    segs[:, 18:20] = 0
    if options_len:
        segs[:, TCP_HDR:TCP_HDR + options_len] = 1  # NOP options
    src = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    dst = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    off = np.arange(n, dtype=np.uint64) * seg_len
    length = np.full(n, seg_len, dtype=np.uint32)
    return segs.reshape(-1), off, length, {"src": src, "dst": dst}


def zipf_lengths(n: int, seed: int, s: float = 1.2, lo: int = 64, hi: int = 9000) -> np.ndarray:
    """L = lo-1+k, k ~ Zipf(s) on {1 .. hi-lo+1} (SURVEY.md §8(d) cfg 3)."""
    rng = _rng(seed)
    kmax = hi - lo + 1
    k = np.arange(1, kmax + 1, dtype=np.float64)
    p = k ** (-s)
    p /= p.sum()
    draw = rng.choice(kmax, size=n, p=p) + 1
    return (lo - 1 + draw).astype(np.uint32)


def pack(lengths: np.ndarray, align: int = 1, seed: int | None = None, max_gap: int = 0):
    """Offsets for packing `lengths` back to back, each start rounded up to
    `align`, optionally with random 0..max_gap byte gaps (odd starts)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    gaps = np.zeros(lengths.size, dtype=np.uint64)
    if max_gap:
        gaps = _rng(seed or 1).integers(0, max_gap + 1, size=lengths.size).astype(np.uint64)
    off = np.empty(lengths.size, dtype=np.uint64)
    pos = 0
    a = int(align)
    for i, (L, g) in enumerate(zip(lengths.tolist(), gaps.tolist())):
        pos += g
        pos = (pos + a - 1) // a * a
        off[i] = pos
        pos += L
    return off, pos


def mixed_udp_frames(n: int, seed: int = 0x5EA57A2C, align: int = 1, max_gap: int = 0,
                     lengths: np.ndarray | None = None):
    """IPv4/UDP frames with Zipf lengths 64..9000 (cfg 3), packed at `align`."""
    rng = _rng(seed)
    if lengths is None:
        lengths = zipf_lengths(n, seed)
    off, total = pack(lengths, align=align, seed=seed + 1, max_gap=max_gap)
    buf = rng.integers(0, 256, size=int(total), dtype=np.uint8)
    src = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    dst = rng.integers(1, 2**32, size=n, dtype=np.uint64)
    sport = rng.integers(1024, 65536, size=n)
    dport = rng.integers(1, 65536, size=n)
    for i in range(n):
        o, L = int(off[i]), int(lengths[i])
        f = buf[o:o + L].reshape(1, L)
        write_ipv4_header(f, [L], PROTO_UDP, [src[i]], [dst[i]])
        _put_be16(f, 20, [sport[i]])
        _put_be16(f, 22, [dport[i]])
        _put_be16(f, 24, [L - IPV4_HDR])
        f[:, 26:28] = 0
    return buf, off, lengths.astype(np.uint32), {"src": src, "dst": dst}


def store_ipv4_checksums(buf: np.ndarray, off: np.ndarray, out2: np.ndarray) -> None:
    """Write computed (IP, L4) checksums into the frames' fields: IP +10,
    UDP +20+6 or TCP +20+16 (ihl 5 frames; header proto picks the L4)."""
    for i in range(off.size):
        o = int(off[i])
        buf[o + 10:o + 12] = np.frombuffer(np.uint16(out2[i, 0]).tobytes(), np.uint8)
        proto = int(buf[o + 9])
        pos = o + 20 + (16 if proto == PROTO_TCP else 6)
        buf[pos:pos + 2] = np.frombuffer(np.uint16(out2[i, 1]).tobytes(), np.uint8)


def frag_words(rng: np.random.Generator, n: int, frac: float = 0.3) -> np.ndarray:
    """IPv4 flags + fragment-offset words (header bytes 6-7, ip.hh:388-391)
    for n frames: atomic datagrams (0, or DF alone) and, with probability
    `frac`, fragments as ipv4::send cuts a datagram (ip.cc:283-294): a first
    fragment (MF, offset 0), a middle one (MF, offset k), a last one (offset
    k, MF clear), and offsets near the top whose offset + length passes the
    65 535-byte datagram limit (ip.cc:141-144)."""
    w = np.where(rng.random(n) < 0.5, 0, 0x4000).astype(np.uint32)  # DF alone is still atomic
    kind = rng.random(n)
    frag = kind < frac
    sub = rng.integers(0, 4, n)
    k = rng.integers(1, 0x2000, n).astype(np.uint32)
    fw = np.select([sub == 0, sub == 1, sub == 2], [0x2000 + 0 * k, 0x2000 | (k & 0x1ff), k & 0x1ff],
                   default=0x1f00 | (k & 0xff))
    w = np.where(frag, fw | (w & 0x4000 & np.where(sub == 2, 0xFFFF, 0)), w)
    return w.astype(np.uint32)


def ipv4_fragment(datagram_l4: np.ndarray, proto: int, src: int, dst: int, mtu: int = 1500,
                  ident: int = 0) -> list[np.ndarray]:
    """ipv4::send (src/net/ip.cc:244-299) of one L4 datagram (header +
    payload, its checksum already in place): cut into pieces of at most
    mtu - 20 bytes when it does not fit (needs_frag, ip.cc:100-111), each
    prepended with its own IPv4 header (ihl 5, id `ident`, MF on all but the
    last, offset in 8-byte units, ttl 64; header checksum 0).  Returns the
    frames.  (With mtu - 20 a multiple of 8, every offset is exact.)"""
    data = np.asarray(datagram_l4, dtype=np.uint8)
    room = mtu - IPV4_HDR
    if data.size + IPV4_HDR <= mtu:
        cuts = [(0, data.size)]
    else:
        cuts = [(o, min(room, data.size - o)) for o in range(0, data.size, room)]
    frames = []
    for k, (o, L) in enumerate(cuts):
        f = np.zeros((1, IPV4_HDR + L), np.uint8)
        write_ipv4_header(f, [IPV4_HDR + L], proto, [src], [dst])
        _put_be16(f, 4, [ident])
        more = k + 1 < len(cuts)
        _put_be16(f, 6, [(0x2000 if more else 0) | ((o // 8) if len(cuts) > 1 else 0)])
        f[0, IPV4_HDR:] = data[o:o + L]
        frames.append(f.reshape(-1))
    return frames


def rss_frames(n: int, seed: int = 0x55):
    """A varied IPv4 batch for RSS hashing (forward_hash edge cases): UDP, TCP,
    ICMP and other protocols; fragments (MF set / nonzero offset); IP options
    (ihl 5-8); Ethernet-style padding (len > ip total length) and truncation;
    frames of 0-19 bytes and just below / at the TCP and UDP header bounds;
    packed back to back at odd offsets.  Returns (buf, off, length)."""
    rng = _rng(seed)
    lens = rng.choice([8, 19, 20, 27, 28, 39, 40, 44, 60, 64, 100, 576, 1500], size=n).astype(np.uint32)
    off, total = pack(lens, seed=seed + 1, max_gap=3)
    buf = rng.integers(0, 256, size=int(total) + 64, dtype=np.uint8)
    protos = rng.choice([PROTO_UDP, PROTO_TCP, 1, 47], size=n, p=[0.4, 0.4, 0.1, 0.1])
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        if L < 20:
            continue
        f = buf[o:o + L]
        ihl = int(rng.choice([5, 5, 5, 6, 8]))
        f[0] = 0x40 | ihl
        ip_len = L if rng.random() < 0.7 else int(rng.integers(20, L + 40))
        f[2], f[3] = (ip_len >> 8) & 0xFF, ip_len & 0xFF
        frag = 0
        r = rng.random()
        if r < 0.15:
            frag = 0x2000  # MF
        elif r < 0.25:
            frag = int(rng.integers(1, 0x2000))  # nonzero offset
        elif r < 0.3:
            frag = 0x4000  # DF only: still atomic
        f[6], f[7] = (frag >> 8) & 0xFF, frag & 0xFF
        f[9] = int(protos[i])
    return buf, off, lens
