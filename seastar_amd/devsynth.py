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
