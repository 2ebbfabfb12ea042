"""Device-side synthetic batches for full-size tests and bench.py.

Same frame layout as synth.py (src/net/ip.cc:249-269, src/net/udp.cc:178-182),
generated directly in HBM with torch so that a 1.5 GB batch never crosses
PCIe.  Only data generation uses torch ops; checksums come from libsccsum.
"""
from __future__ import annotations

import torch

from .batch import PacketBatch


def _round16(n: int) -> int:
    return (n + 15) & ~15


def random_bytes(nbytes: int, g: torch.Generator, device, chunk: int = 1 << 30) -> torch.Tensor:
    """nbytes random bytes in HBM, generated in 1 GiB pieces (torch's RNG
    kernels are happiest below 2^31 elements)."""
    data = torch.empty(nbytes, dtype=torch.uint8, device=device)
    for s in range(0, nbytes, chunk):
        e = min(nbytes, s + chunk)
        data[s:e].random_(0, 256, generator=g)
    return data


def _be16(x: torch.Tensor) -> torch.Tensor:
    return torch.stack([(x >> 8) & 0xFF, x & 0xFF], dim=1).to(torch.uint8)


def _be32(x: torch.Tensor) -> torch.Tensor:
    return torch.stack([(x >> 24) & 0xFF, (x >> 16) & 0xFF, (x >> 8) & 0xFF, x & 0xFF], dim=1).to(torch.uint8)


def udp_frames(n: int, frame_len: int, seed: int, device) -> PacketBatch:
    """n IPv4/UDP frames of frame_len bytes back to back, checksum fields 0."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    total = n * frame_len
    data = torch.randint(0, 256, (_round16(total),), dtype=torch.uint8, device=device, generator=g)
    f = data[:total].view(n, frame_len)
    src = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    dst = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    f[:, 0] = 0x45
    f[:, 1] = 0
    f[:, 2:4] = _be16(torch.full((n,), frame_len, dtype=torch.int64, device=device))
    f[:, 4:8] = 0
    f[:, 8] = 64
    f[:, 9] = 17
    f[:, 10:12] = 0
    f[:, 12:16] = _be32(src)
    f[:, 16:20] = _be32(dst)
    f[:, 24:26] = _be16(torch.full((n,), frame_len - 20, dtype=torch.int64, device=device))
    f[:, 26:28] = 0
    off = torch.arange(n, dtype=torch.int64, device=device) * frame_len
    length = torch.full((n,), frame_len, dtype=torch.int32, device=device)
    return PacketBatch(data=data, off=off, length=length, bytes_len=total, max_len=frame_len)


def _frame_view(b: PacketBatch) -> torch.Tensor:
    L = b.max_len
    return b.data[: b.n * L].view(b.n, L)


def store_checksums(b: PacketBatch, out2: torch.Tensor) -> PacketBatch:
    """Copy of an equal-length UDP batch with (IP, UDP) checksums stored in
    their fields (IP +10, UDP +26), i.e. a received batch that verifies."""
    data = b.data.clone()
    nb = PacketBatch(data=data, off=b.off, length=b.length, bytes_len=b.bytes_len, max_len=b.max_len)
    f = _frame_view(nb)
    raw = out2.contiguous().view(torch.uint8).view(b.n, 4)
    f[:, 10:12] = raw[:, 0:2]
    f[:, 26:28] = raw[:, 2:4]
    return nb


def corrupt(b: PacketBatch, idx: torch.Tensor, byte: int) -> None:
    """Flip bits of payload byte `byte` in frames idx (in place)."""
    f = _frame_view(b)
    f[idx, byte] ^= 0x5A


def tcp_segments(n: int, seg_len: int, seed: int, device):
    """n TCP segments (20 B header, checksum 0, payload random) back to back;
    returns (batch, seeds): seeds = pseudo-header partial sums exactly as
    tcp_pseudo_header_checksum leaves them (ip.hh:70-75, len as uint16_t),
    folded to 16 bits."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    total = n * seg_len
    data = random_bytes(_round16(total), g, device)
    f = data[:total].view(n, seg_len)
    f[:, 12] = (20 // 4) << 4
    f[:, 13] = 0x10
    f[:, 16:18] = 0
    src = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    dst = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    s = src + dst + 6 + (seg_len & 0xFFFF)
    for _ in range(3):
        s = (s & 0xFFFF) + (s >> 16)
    off = torch.arange(n, dtype=torch.int64, device=device) * seg_len
    length = torch.full((n,), seg_len, dtype=torch.int32, device=device)
    b = PacketBatch(data=data, off=off, length=length, bytes_len=total, max_len=seg_len)
    return b, s.to(torch.int32)


def store_tcp_checksums(b: PacketBatch, out: torch.Tensor) -> None:
    """tcp_hdr::write_nbo_checksum (tcp.hh:283-285) for every segment, in place."""
    f = _frame_view(b)
    f[:, 16:18] = out.contiguous().view(torch.uint8).view(b.n, 2)


def mixed_frames(lengths, seed: int, device, align: int = 1) -> PacketBatch:
    """IPv4/UDP frames of the given lengths packed back to back (align 1: odd
    offsets included) or each starting on an `align`-byte boundary, built in
    HBM: random payload (and gap bytes), headers per ip.cc:249-269."""
    import numpy as np

    lengths = np.asarray(lengths, dtype=np.int64)
    n = lengths.size
    pitch = (lengths + align - 1) // align * align
    off = np.concatenate([[0], np.cumsum(pitch)[:-1]])
    total = int(off[-1] + lengths[-1]) if n else 0
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    data = torch.randint(0, 256, (_round16(total),), dtype=torch.uint8, device=device, generator=g)
    o = torch.from_numpy(off).to(device)
    L = torch.from_numpy(lengths).to(device)

    def put(k: int, vals):
        data[o + k] = vals.to(torch.uint8) if torch.is_tensor(vals) else torch.full_like(o, vals, dtype=torch.uint8)

    src = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    dst = torch.randint(1, 2**31, (n,), dtype=torch.int64, device=device, generator=g)
    put(0, 0x45)
    put(1, 0)
    put(2, (L >> 8) & 0xFF)
    put(3, L & 0xFF)
    for k in (4, 5, 6, 7, 10, 11, 26, 27):
        put(k, 0)
    put(8, 64)
    put(9, 17)
    for i in range(4):
        put(12 + i, (src >> (24 - 8 * i)) & 0xFF)
        put(16 + i, (dst >> (24 - 8 * i)) & 0xFF)
    put(24, ((L - 20) >> 8) & 0xFF)
    put(25, (L - 20) & 0xFF)
    return PacketBatch(data=data, off=o, length=L.to(torch.int32), bytes_len=total, max_len=int(lengths.max()))
