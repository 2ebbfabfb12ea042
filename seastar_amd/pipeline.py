"""Host-memory batches through the GPU (sccsum_pipeline_* in include/sccsum.h):
the end-to-end path of BASELINE cfg 5 — DPDK-mbuf-shaped pinned host buffers,
hipMemcpyAsync in and out on side streams, overlapped with the kernels."""
from __future__ import annotations

import bisect
import ctypes
import threading
import weakref

import numpy as np

from . import native

MBUF_SLOT = 128 + 128 + 2048  # rte_mbuf + headroom + data room (src/net/dpdk.cc:139-156)
MBUF_DATA_OFF = 256


class _PinnedBlock:
    """Owner of one sccsum_host_alloc block, exposed through the array
    interface: numpy arrays made from it (and every view of those) hold a
    reference to the block, so the memory is freed only when the last of them
    is gone."""

    def __init__(self, nbytes: int):
        self._lib = native.load()
        p = ctypes.c_void_p()
        native.check(self._lib.sccsum_host_alloc(ctypes.byref(p), max(int(nbytes), 1)), "sccsum_host_alloc")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.__array_interface__ = {"data": (self.ptr, False), "shape": (self.nbytes,), "typestr": "|u1",
                                    "version": 3}
        _register(self)

    def __del__(self):
        _unregister(self.ptr)
        self._lib.sccsum_host_free(self.ptr)


# live pinned blocks by start address, for is_pinned (mapped burst submits)
_pinned_lock = threading.Lock()
_pinned_starts: list[int] = []
_pinned_blocks: dict[int, weakref.ref] = {}


def _register(b: _PinnedBlock) -> None:
    with _pinned_lock:
        bisect.insort(_pinned_starts, b.ptr)
        _pinned_blocks[b.ptr] = weakref.ref(b)


def _unregister(ptr: int) -> None:
    with _pinned_lock:
        i = bisect.bisect_left(_pinned_starts, ptr)
        if i < len(_pinned_starts) and _pinned_starts[i] == ptr:
            del _pinned_starts[i]
        _pinned_blocks.pop(ptr, None)


def is_pinned(a: np.ndarray) -> bool:
    """a's bytes lie inside one live pinned_empty block (device-readable at
    the same address: what a zero-copy burst submit needs)."""
    if a.size == 0:
        return True
    lo = a.ctypes.data
    hi = lo + a.nbytes
    with _pinned_lock:
        i = bisect.bisect_right(_pinned_starts, lo) - 1
        if i < 0:
            return False
        b = _pinned_blocks[_pinned_starts[i]]()
        return b is not None and hi <= b.ptr + b.nbytes


def pinned_empty(nbytes: int) -> np.ndarray:
    """uint8 array in page-locked host memory, freed when the array and every
    view of it are gone."""
    return np.asarray(_PinnedBlock(nbytes))


def mbuf_pool(frames: np.ndarray, lengths: np.ndarray, offsets: np.ndarray):
    """Place each packet in its own mbuf-shaped slot of a pinned pool: packet i
    at slot i + 256 (after the rte_mbuf header and headroom).  Returns
    (pool, off, len)."""
    n = lengths.size
    if n and int(np.max(lengths)) > MBUF_SLOT - MBUF_DATA_OFF:
        raise ValueError("a packet longer than one mbuf data room (2048 B) needs a segment chain")
    pool = pinned_empty(n * MBUF_SLOT)
    pool[:] = 0
    off = np.arange(n, dtype=np.uint64) * MBUF_SLOT + MBUF_DATA_OFF
    for i in range(n):
        L = int(lengths[i])
        o = int(offsets[i])
        pool[int(off[i]):int(off[i]) + L] = frames[o:o + L]
    return pool, off, lengths.astype(np.uint32)


class HostPipeline:
    def __init__(self, device: int = 0, chunk_bytes: int = 64 << 20, chunk_packets: int = 1 << 16, depth: int = 3):
        self._lib = native.load()
        h = ctypes.c_void_p()
        native.check(self._lib.sccsum_pipeline_create(device, chunk_bytes, chunk_packets, depth, ctypes.byref(h)),
                     "sccsum_pipeline_create")
        self._h = h

    def run(self, mode: int, buf: np.ndarray, off: np.ndarray, length: np.ndarray, seeds: np.ndarray | None = None,
            status: bool = False, gather: int = 0, max_len: int = 0):
        """gather: 0 = copy chunks as they lie, 1 = pack on the host first,
        2 = one 2D DMA of each slot's packet bytes, 3 = no copies: the kernel
        reads the packets in place (buf must be pinned: pinned_empty)
        (native.GATHER_*)."""
        # the native side reads buf.size bytes at buf's address and n entries of
        # every metadata array: a strided / wider-typed buf or a short array
        # would be read past its end
        if not (isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags.c_contiguous):
            raise ValueError("buf must be a contiguous uint8 array")
        if gather == native.GATHER_ZERO_COPY and buf.size and not is_pinned(buf):
            raise ValueError("zero-copy pipeline runs need a pinned buffer (pinned_empty)")
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.size
        sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
        if length.size != n or (sd is not None and sd.size != n):
            raise ValueError(f"off, length and seeds need one entry per packet ({n})")
        width = 2 if mode == native.PIPE_IPV4 else 1
        out = np.empty((n, width) if width == 2 else n, dtype=np.uint16)
        st = np.empty(n, dtype=np.uint8) if status else None
        code = self._lib.sccsum_pipeline_run(
            self._h, mode, int(gather), buf.ctypes.data if buf.size else None, buf.size, off.ctypes.data,
            length.ctypes.data, None if sd is None else sd.ctypes.data, n, max_len,
            out.ctypes.data, None if st is None else st.ctypes.data)
        native.check(code, "sccsum_pipeline_run")
        return (out, st) if status else out

    def close(self):
        if self._h:
            self._lib.sccsum_pipeline_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
