"""Burst queue (sccsum_burst_* in include/sccsum.h): the batching hook at the
qp boundary.  Packets are submitted from host memory one at
a time, as qp::poll_tx (src/net/net.cc:81-105) and the DPDK rx loop
(src/net/dpdk.cc:2190-2204) hand them over; the queue accumulates them into GPU
batches and completes them asynchronously through a callback on the polling
thread, like a reactor poller (include/seastar/core/internal/poll.hh:26-29)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import native, pipeline

DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                           ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint8))


class BurstQueue:
    """mode: native.PIPE_SPANS (seeded sums, one result per packet) or
    native.PIPE_IPV4 (frames, two results per packet).  on_done(first_ticket,
    results, status) gets numpy copies of each completed batch, in submit
    order; without it the results are collected in self.results /
    self.status by ticket."""

    def __init__(self, mode: int, device: int = 0, batch_bytes: int = 1 << 20, batch_packets: int = 1024,
                 max_delay_ns: int = 50_000, depth: int = 4, on_done=None):
        self._lib = native.load()
        self._h = None
        self.mode = mode
        self.width = 2 if mode == native.PIPE_IPV4 else 1
        self.results: dict[int, np.ndarray] = {}
        self.status: dict[int, int] = {}
        self.batches = 0
        self._user = on_done
        self._held: dict[int, list] = {}  # mapped submits: fragment arrays kept alive until completion
        self._cb = DONE_FN(self._done)  # lives as long as the queue
        h = ctypes.c_void_p()
        native.check(self._lib.sccsum_burst_create(device, mode, batch_bytes, batch_packets, max_delay_ns, depth,
                                                   ctypes.cast(self._cb, ctypes.c_void_p), None, ctypes.byref(h)),
                     "sccsum_burst_create")
        self._h = h

    def _done(self, _user, first, count, res, st):
        r = np.ctypeslib.as_array(res, shape=(count * self.width,)).copy()
        s = np.ctypeslib.as_array(st, shape=(count,)).copy()
        if self.width == 2:
            r = r.reshape(count, 2)
        self.batches += 1
        for k in range(count):
            self._held.pop(first + k, None)
        if self._user is not None:
            self._user(int(first), r, s)
            return
        for k in range(count):
            self.results[first + k] = r[k]
            self.status[first + k] = int(s[k])

    def submit(self, fragments, seed: int = 0, mapped: bool = False) -> int | None:
        """Stage one packet given as a list of uint8 arrays / bytes (its
        fragments, in order); returns its ticket, or None when every slot is
        in flight (poll, then retry).  mapped=True: zero-copy
        (sccsum_burst_submit_mapped) — the arrays must be views of pinned
        memory (pipeline.pinned_empty) and stay untouched until completion."""
        bufs = [np.ascontiguousarray(np.frombuffer(f, np.uint8) if isinstance(f, (bytes, bytearray)) else f,
                                     dtype=np.uint8) for f in fragments]
        if mapped:
            # the device reads these bytes at their host address: they must be
            # contiguous views of a live pinned block (pipeline.pinned_empty);
            # pageable memory would fault the GPU
            for f in fragments:
                if not (isinstance(f, np.ndarray) and f.dtype == np.uint8 and f.flags.c_contiguous):
                    raise ValueError("mapped fragments must be contiguous uint8 views of pinned memory")
                if not pipeline.is_pinned(f):
                    raise ValueError("mapped fragments must lie in pinned memory (pipeline.pinned_empty)")
        frags = (native.Fragment * max(len(bufs), 1))()
        for j, b in enumerate(bufs):
            frags[j].base = b.ctypes.data if b.size else None
            frags[j].size = b.size
        ticket = ctypes.c_uint64()
        fn = self._lib.sccsum_burst_submit_mapped if mapped else self._lib.sccsum_burst_submit
        code = fn(self._h, ctypes.cast(frags, ctypes.c_void_p), len(bufs), seed, ctypes.byref(ticket))
        if code == native.SCCSUM_EBUSY:
            return None
        native.check(code, "sccsum_burst_submit")
        if mapped:
            self._held[ticket.value] = bufs
        return ticket.value

    def poll(self) -> bool:
        did = ctypes.c_int()
        native.check(self._lib.sccsum_burst_poll(self._h, ctypes.byref(did)), "sccsum_burst_poll")
        return bool(did.value)

    def drain(self) -> None:
        native.check(self._lib.sccsum_burst_drain(self._h), "sccsum_burst_drain")

    def close(self):
        if self._h:
            self._lib.sccsum_burst_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
