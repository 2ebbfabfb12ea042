"""Op-sequence cases for the reference checksummer driver
(oracle/ref/checksummer_ref.cc) and their replay on the oracle — TEST
INFRASTRUCTURE: shared by tests/golden/make_ref_accum.py (which runs the
REFERENCE build and writes tests/golden/ref_accum.json) and
tests/test_ref_pinning.py (which replays every case on the oracle).

A case is a string of whitespace-separated ops (see the driver's header):
u8:V u16:V u32:V, ph:SRC:DST:PROTO:LEN, x:HEX, rep:V:N, g:SEED:LEN:FILL.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def splitmix_bytes(seed: int, n: int) -> bytes:
    """The driver's generator: little-endian bytes of successive
    splitmix64(seed) outputs, truncated to n."""
    words = (n + 7) // 8
    if words == 0:
        return b""
    with np.errstate(over="ignore"):
        s = (np.uint64(seed) + np.arange(1, words + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = s
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:n]


def op_bytes(tok: str) -> bytes | None:
    """The bytes a byte op feeds, or None for a scalar op."""
    f = tok.split(":")
    if f[0] == "x":
        return bytes.fromhex(f[1])
    if f[0] == "rep":
        return bytes([int(f[1])]) * int(f[2])
    if f[0] == "g":
        seed, n, fill = int(f[1]), int(f[2]), int(f[3])
        return splitmix_bytes(seed, n) if fill == 0 else (b"\0" if fill == 1 else b"\xff") * n
    return None


def fold_get(csum: int) -> int:
    """checksummer::get() (src/net/ip_checksum.cc:55-62) statement by
    statement on an accumulator value: 128 -> 64 bits twice with end-around
    carry, four 16-bit lanes, two more folds, complement, htons (the uint16_t
    value on a little-endian host)."""
    c1 = (csum & M64) + (csum >> 64)
    c = ((c1 & M64) + (c1 >> 64)) & M64
    c = (c & 0xFFFF) + ((c >> 16) & 0xFFFF) + ((c >> 32) & 0xFFFF) + (c >> 48)
    c = (c & 0xFFFF) + (c >> 16)
    c = (c & 0xFFFF) + (c >> 16)
    v = ~c & 0xFFFF
    return ((v & 0xFF) << 8) | (v >> 8)
