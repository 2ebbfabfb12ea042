"""Sharding a packet batch across GPUs.

Packets are independent, so a batch splits into G contiguous index ranges of
about equal BYTES (prefix sum of the lengths), one per GPU / rank, with no
data-path collective: each rank uploads and checksums its own range, and the
(2-4 B per packet) results come back by index.  This mirrors Seastar's own
scaling — shard-per-core with flows steered by RSS — one shard per device.
"""
from __future__ import annotations

import numpy as np


def partition_by_bytes(lengths: np.ndarray, world: int) -> np.ndarray:
    """Boundaries b[0..world] (b[0]=0, b[world]=n): rank r owns [b[r], b[r+1])."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = lengths.size
    if world < 1:
        raise ValueError("world must be >= 1")
    prefix = np.concatenate([[0], np.cumsum(lengths, dtype=np.uint64)])
    total = int(prefix[-1])
    b = np.empty(world + 1, dtype=np.int64)
    b[0], b[world] = 0, n
    for r in range(1, world):
        # first packet whose start reaches r/world of the bytes
        b[r] = int(np.searchsorted(prefix[:-1], total * r // world, side="left")) if total else n * r // world
    return np.maximum.accumulate(b)


def shard(buf: np.ndarray, off: np.ndarray, length: np.ndarray, rank: int, world: int):
    """Rank's slice of a host batch: (bytes, rebased offsets, lengths, (lo, hi)).

    The byte slice covers [min off, max off+len) of the rank's packets, so a
    rank uploads only what it checksums."""
    b = partition_by_bytes(length, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    o = np.asarray(off[lo:hi], dtype=np.uint64)
    ln = np.asarray(length[lo:hi], dtype=np.uint32)
    if hi == lo:
        return np.zeros(0, np.uint8), o, ln, (lo, hi)
    start = int(o.min())
    end = int((o + ln.astype(np.uint64)).max())
    return np.ascontiguousarray(buf[start:end]), o - np.uint64(start), ln, (lo, hi)


def assemble(parts: list, n: int, width: int = 1, dtype=np.uint16) -> np.ndarray:
    """Concatenate per-rank results [(lo, hi, values)] back into index order."""
    out = np.zeros((n, width) if width > 1 else n, dtype=dtype)
    for lo, hi, vals in parts:
        out[lo:hi] = vals
    return out
