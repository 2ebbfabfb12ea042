"""ctypes wrapper of the ORACLE (oracle/sccsum_oracle.c) — TEST INFRASTRUCTURE
ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker / CPU baseline, never by the product (seastar_amd/)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(ORACLE_DIR, "build", "libsccsum_oracle.so")


class Checksummer(ctypes.Structure):
    _fields_ = [("csum_lo", ctypes.c_uint64), ("csum_hi", ctypes.c_int64), ("odd", ctypes.c_int),
                ("_pad", ctypes.c_int * 3)]

    @property
    def csum(self) -> int:
        return (self.csum_hi << 64) | self.csum_lo


_lib = None
_P = ctypes.c_void_p


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        cs = ctypes.POINTER(Checksummer)
        protos = {
            "oracle_init": (None, [cs]),
            "oracle_sum_bytes": (None, [cs, _P, ctypes.c_size_t]),
            "oracle_sum_u8": (None, [cs, ctypes.c_uint8]),
            "oracle_sum_u16": (None, [cs, ctypes.c_uint16]),
            "oracle_sum_u32": (None, [cs, ctypes.c_uint32]),
            "oracle_get": (ctypes.c_uint16, [cs]),
            "oracle_sum_fragments": (None, [cs, _P, _P, ctypes.c_size_t]),
            "oracle_ip_checksum": (ctypes.c_uint16, [_P, ctypes.c_size_t]),
            "oracle_pseudo_header": (None, [cs, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint16]),
            "oracle_fold_seed": (ctypes.c_uint32, [cs]),
            "oracle_batch_spans": (None, [_P, _P, _P, _P, _P, ctypes.c_uint64, ctypes.c_int]),
            "oracle_batch_ipv4": (None, [_P, _P, _P, _P, _P, ctypes.c_uint64, ctypes.c_int]),
            "oracle_batch_ipv4_cpus": (None, [_P, _P, _P, _P, _P, ctypes.c_uint64, _P, ctypes.c_int]),
            "oracle_batch_fragments": (None, [_P, _P, _P, _P, _P, _P, ctypes.c_uint64]),
            "oracle_batch_ipv4_fill": (None, [_P, _P, _P, _P, _P, ctypes.c_uint64, ctypes.c_uint32]),
            "oracle_toeplitz": (ctypes.c_uint32, [_P, ctypes.c_size_t, _P, ctypes.c_size_t]),
            "oracle_batch_ipv4_rss": (None, [_P, _P, _P, ctypes.c_uint64, _P, ctypes.c_size_t, ctypes.c_int, _P,
                                             _P]),
        }
        for name, (res, args) in protos.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _addr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def ip_checksum(data: bytes | np.ndarray) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return int(lib().oracle_ip_checksum(_addr(a) if a.size else None, a.size))


def new() -> Checksummer:
    c = Checksummer()
    # the C struct holds an __int128 (16-byte alignment); pymalloc blocks are
    # 16-aligned on x86-64, check rather than assume
    assert ctypes.addressof(c) % 16 == 0
    lib().oracle_init(ctypes.byref(c))
    return c


def sum_bytes(c: Checksummer, data) -> None:
    a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8))
    lib().oracle_sum_bytes(ctypes.byref(c), _addr(a) if a.size else None, a.size)


def get(c: Checksummer) -> int:
    return int(lib().oracle_get(ctypes.byref(c)))


def pseudo_seed(src: int, dst: int, proto: int, length: int) -> int:
    c = new()
    lib().oracle_pseudo_header(ctypes.byref(c), src, dst, proto, length & 0xFFFF)
    return int(lib().oracle_fold_seed(ctypes.byref(c)))


def batch_spans(buf: np.ndarray, off: np.ndarray, length: np.ndarray, seeds: np.ndarray | None = None,
                nthreads: int = 1) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    seeds = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint16)
    lib().oracle_batch_spans(_addr(buf), _addr(off), _addr(length), _addr(seeds), _addr(out), off.size, nthreads)
    return out


def batch_ipv4(buf: np.ndarray, off: np.ndarray, length: np.ndarray, nthreads: int = 1, cpus=None):
    """Returns (out2 [n,2] uint16, status [n] uint8).  With `cpus`, one thread
    per listed CPU, each pinned to it (nthreads is then len(cpus))."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out2 = np.empty((off.size, 2), dtype=np.uint16)
    status = np.empty(off.size, dtype=np.uint8)
    if cpus is not None:
        c = np.ascontiguousarray(cpus, dtype=np.int32)
        lib().oracle_batch_ipv4_cpus(_addr(buf), _addr(off), _addr(length), _addr(out2), _addr(status), off.size,
                                     _addr(c), c.size)
    else:
        lib().oracle_batch_ipv4(_addr(buf), _addr(off), _addr(length), _addr(out2), _addr(status), off.size,
                                nthreads)
    return out2, status


def batch_fragments(buf, frag_off, frag_len, pkt_first, seeds=None) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    frag_off = np.ascontiguousarray(frag_off, dtype=np.uint64)
    frag_len = np.ascontiguousarray(frag_len, dtype=np.uint32)
    pkt_first = np.ascontiguousarray(pkt_first, dtype=np.uint32)
    seeds = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    n = pkt_first.size - 1
    out = np.empty(n, dtype=np.uint16)
    lib().oracle_batch_fragments(_addr(buf), _addr(frag_off), _addr(frag_len), _addr(pkt_first), _addr(seeds),
                                 _addr(out), n)
    return out


def batch_ipv4_fill(buf, off, length, mode):
    """Tx generate in place on a COPY of buf: returns (frames, out2 [n,2], status)."""
    buf = np.array(buf, dtype=np.uint8, copy=True)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    n = off.size
    out2 = np.empty(2 * n, dtype=np.uint16)
    st = np.empty(n, dtype=np.uint8)
    lib().oracle_batch_ipv4_fill(_addr(buf), _addr(off), _addr(length), _addr(out2), _addr(st), n, mode)
    return buf, out2.reshape(n, 2), st


# Mellanox driver key the reference ships as its default (toeplitz.hh:52-58)
RSS_KEY_40 = bytes.fromhex("d181c62cf7f4db5b1983a2fc943e1adbd9389e6bd1039c2ca74499ad593d56d9f3253c062adc1ffc")


def toeplitz(key: bytes, data: bytes) -> int:
    kb = np.frombuffer(bytes(key), np.uint8)
    db = np.frombuffer(bytes(data), np.uint8) if data else np.zeros(1, np.uint8)
    return int(lib().oracle_toeplitz(_addr(kb), kb.size, _addr(db), len(data)))


def batch_ipv4_rss(buf, off, length, key: bytes = RSS_KEY_40, mode: int = 0):
    """(hash u32 [n], status u8 [n]) per frame, as oracle_ipv4_rss."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    kb = np.frombuffer(bytes(key), np.uint8)
    h = np.empty(off.size, dtype=np.uint32)
    st = np.empty(off.size, dtype=np.uint8)
    lib().oracle_batch_ipv4_rss(_addr(buf), _addr(off), _addr(length), off.size, _addr(kb), kb.size, mode,
                                _addr(h), _addr(st))
    return h, st
