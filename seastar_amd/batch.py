"""Device-resident packet batches and the launch wrappers over the C-ABI.

A batch is the layout the kernels consume (DESIGN.md "Data layout in HBM"):
one byte buffer holding every packet back to back (any alignment), padded to
a multiple of 16 bytes, plus an offset (u64) / length (u32) array.  torch
tensors only hold the device memory and give the stream; the arithmetic is in
libsccsum.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import native


def _round16(n: int) -> int:
    return (n + 15) & ~15


@dataclass
class PacketBatch:
    data: torch.Tensor  # uint8, len >= round16(bytes_len), device
    off: torch.Tensor  # int64 [n], device
    length: torch.Tensor  # int32 [n], device
    bytes_len: int
    max_len: int

    def __post_init__(self):
        # the kernels trust these: a short buffer or a mistyped array would be
        # read (or, for in-place fill, written) past its end on the device
        d, o, ln = self.data, self.off, self.length
        if d.dtype != torch.uint8 or d.dim() != 1 or not d.is_contiguous():
            raise ValueError("PacketBatch.data must be a contiguous 1-D uint8 tensor")
        if not (0 <= int(self.bytes_len) and _round16(int(self.bytes_len)) <= d.numel()):
            raise ValueError(f"PacketBatch.data holds {d.numel()} bytes; bytes_len {self.bytes_len} needs "
                             f"{_round16(int(self.bytes_len))} (padded to 16)")
        if o.dtype != torch.int64 or o.dim() != 1 or not o.is_contiguous():
            raise ValueError("PacketBatch.off must be a contiguous 1-D int64 tensor")
        if ln.dtype != torch.int32 or ln.dim() != 1 or not ln.is_contiguous() or ln.numel() != o.numel():
            raise ValueError("PacketBatch.length must be a contiguous 1-D int32 tensor with one entry per offset")
        if o.device != d.device or ln.device != d.device:
            raise ValueError("PacketBatch tensors must be on one device")
        if int(self.max_len) < 0:
            raise ValueError("PacketBatch.max_len must be >= 0 (0 = unknown)")

    @property
    def n(self) -> int:
        return int(self.off.numel())

    @property
    def device(self) -> torch.device:
        return self.data.device

    @staticmethod
    def from_host(buf: np.ndarray, off: np.ndarray, length: np.ndarray, device="cuda") -> "PacketBatch":
        buf = np.ascontiguousarray(buf, dtype=np.uint8).ravel()
        bytes_len = int(buf.size)
        padded = np.zeros(_round16(bytes_len) or 16, dtype=np.uint8)
        padded[:bytes_len] = buf
        off = np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)
        length = np.ascontiguousarray(length, dtype=np.uint32).view(np.int32)
        max_len = int(length.view(np.uint32).max()) if length.size else 0
        return PacketBatch(
            data=torch.from_numpy(padded).to(device),
            off=torch.from_numpy(off.copy()).to(device),
            length=torch.from_numpy(length.copy()).to(device),
            bytes_len=bytes_len,
            max_len=max_len,
        )


def _ptr(t):
    return None if t is None else ctypes_ptr(t)


def _need(t: torch.Tensor | None, numel: int, dtype: torch.dtype, what: str, device: torch.device) -> None:
    """A caller-supplied array the kernel reads or writes numel elements of."""
    if t is None:
        return
    if t.dtype != dtype or not t.is_contiguous() or t.numel() < numel or t.device != device:
        raise ValueError(f"{what}: need a contiguous {dtype} tensor of >= {numel} elements on {device}, got "
                         f"{t.dtype} x {t.numel()} on {t.device}")


def ctypes_ptr(t: torch.Tensor) -> int:
    if not t.is_cuda:
        raise ValueError("sccsum kernels need device tensors")
    return t.data_ptr()


def _stream(stream) -> int | None:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def _scratch(numel: int, device, stream, dtype=torch.uint8) -> torch.Tensor:
    """A buffer the library fills or reads for kernels queued on `stream`
    (scratch, or an output the caller did not pass).  It is allocated on
    `stream` itself, so the caching allocator hands out a block whose earlier
    users on that stream are ordered before the launch (a block freed on
    another stream could still be read there when the kernel overwrites it,
    ADVICE r03), and it is recorded on torch's current stream, where the
    caller reads the results, so it is not reused before that stream is done
    with it either."""
    if stream is None or not torch.device(device).type == "cuda":
        return torch.empty(numel, dtype=dtype, device=device)
    with torch.cuda.stream(stream):
        t = torch.empty(numel, dtype=dtype, device=device)
    cur = torch.cuda.current_stream(t.device)
    if cur != stream:
        t.record_stream(cur)
    return t


def spans(batch: PacketBatch, seeds: torch.Tensor | None = None, out: torch.Tensor | None = None,
          status: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """sccsum_spans: one network-order uint16 checksum per span (int16 tensor)."""
    lib = native.load()
    n = batch.n
    if out is None:
        out = _scratch(max(n, 1), batch.device, stream, torch.int16)
    _need(out, n, torch.int16, "out", batch.device)
    _need(seeds, n, torch.int32, "seeds", batch.device)
    _need(status, n, torch.uint8, "status", batch.device)
    code = lib.sccsum_spans(
        ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off), ctypes_ptr(batch.length),
        _ptr(seeds), ctypes_ptr(out), _ptr(status), n, batch.max_len, _stream(stream),
    )
    native.check(code, "sccsum_spans")
    return out[:n]


def ipv4_frames(batch: PacketBatch, out2: torch.Tensor | None = None, status: torch.Tensor | None = None,
                stream=None) -> torch.Tensor:
    """sccsum_ipv4_frames: [n, 2] int16 (IPv4 header checksum, L4 checksum)."""
    lib = native.load()
    n = batch.n
    if out2 is None:
        out2 = _scratch(max(2 * n, 2), batch.device, stream, torch.int16)
    _need(out2, 2 * n, torch.int16, "out2", batch.device)
    _need(status, n, torch.uint8, "status", batch.device)
    code = lib.sccsum_ipv4_frames(
        ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off), ctypes_ptr(batch.length),
        ctypes_ptr(out2), _ptr(status), n, batch.max_len, _stream(stream),
    )
    native.check(code, "sccsum_ipv4_frames")
    return out2[: 2 * n].view(n, 2) if n else out2[:0].view(0, 2)


def verify_frames(batch: PacketBatch, status: torch.Tensor, stream=None) -> torch.Tensor:
    """sccsum_ipv4_frames in verify-only form (no d_out2): per-frame status
    bits only — what the reference's verify keeps of the sum (ip.cc:121-127,
    tcp.hh:876-883: drop when get() != 0).  Returns status[:n]."""
    lib = native.load()
    n = batch.n
    if status is None:
        raise ValueError("verify_frames needs a status tensor")
    _need(status, n, torch.uint8, "status", batch.device)
    code = lib.sccsum_ipv4_frames(
        ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off), ctypes_ptr(batch.length),
        None, ctypes_ptr(status), n, batch.max_len, _stream(stream),
    )
    native.check(code, "sccsum_ipv4_frames")
    return status[:n]


def _multi(fn, name, items, max_len, stream, width, with_seed):
    lib = native.load()
    if len(items) > native.MAX_BATCHES:
        raise ValueError(f"at most {native.MAX_BATCHES} batches per launch")
    arr = (native.Batch * max(len(items), 1))()
    outs, rows = [], []
    for i, it in enumerate(items):  # every batch checked before any address is taken
        b, out, status = it[0], it[1], it[2]
        seeds = it[3] if len(it) > 3 else None
        if seeds is not None and not with_seed:
            raise ValueError(f"{name}: frames take no seeds")
        _need(out, width * b.n, torch.int16, f"batch {i} out", b.device)
        _need(seeds, b.n, torch.int32, f"batch {i} seeds", b.device)
        _need(status, b.n, torch.uint8, f"batch {i} status", b.device)
        rows.append((b, out, status, seeds))
    for i, (b, out, status, seeds) in enumerate(rows):
        if out is None:
            out = _scratch(max(width * b.n, width), b.device, stream, torch.int16)
        arr[i] = native.Batch(ctypes_ptr(b.data), b.bytes_len, ctypes_ptr(b.off), ctypes_ptr(b.length), _ptr(seeds),
                              ctypes_ptr(out), _ptr(status), b.n)
        outs.append(out)
    native.check(fn(ctypes.cast(arr, ctypes.c_void_p), len(items), max_len, _stream(stream)), name)
    return outs


def ipv4_frames_multi(items, stream=None) -> list:
    """sccsum_ipv4_frames_multi: items = [(PacketBatch, out2 | None, status | None), ...]
    (<= 16) in ONE launch; returns the [n, 2] int16 outputs per batch."""
    ml = max((it[0].max_len for it in items), default=0)
    outs = _multi(native.load().sccsum_ipv4_frames_multi, "sccsum_ipv4_frames_multi", items, ml, stream, 2, False)
    return [o[: 2 * it[0].n].view(it[0].n, 2) for o, it in zip(outs, items)]


def prepare_ipv4_frames_multi(items):
    """A prebuilt sccsum_ipv4_frames_multi launch over fixed batches and
    outputs: returns launch(stream) that only crosses the C-ABI (no argument
    marshalling per call), for callers that relaunch the same batch set."""
    lib = native.load()
    if not items or len(items) > native.MAX_BATCHES:
        raise ValueError(f"1..{native.MAX_BATCHES} batches per launch")
    arr = (native.Batch * len(items))()
    for i, (b, out, status) in enumerate(items):  # every batch checked before any address is taken
        # out None: a verify-only batch (status bits only)
        if out is None and status is None:
            raise ValueError(f"batch {i}: give out2, status or both")
        _need(out, 2 * b.n, torch.int16, f"batch {i} out2", b.device)
        _need(status, b.n, torch.uint8, f"batch {i} status", b.device)
    for i, (b, out, status) in enumerate(items):
        arr[i] = native.Batch(ctypes_ptr(b.data), b.bytes_len, ctypes_ptr(b.off), ctypes_ptr(b.length), None,
                              _ptr(out), _ptr(status), b.n)
    ml = max(it[0].max_len for it in items)
    fn, ptr, nb = lib.sccsum_ipv4_frames_multi, ctypes.cast(arr, ctypes.c_void_p), len(items)

    def launch(stream):
        code = fn(ptr, nb, ml, stream.cuda_stream)
        if code:
            native.check(code, "sccsum_ipv4_frames_multi")

    launch.keep = (arr, items)  # the descriptors and tensors outlive the closure's callers
    return launch


def prepare_call(name: str, *args):
    """A prebuilt C-ABI call: tensors become device addresses once; the
    returned launch(stream) appends the stream handle and calls `name`."""
    lib = native.load()
    fn = getattr(lib, name)
    conv = tuple(ctypes_ptr(a) if isinstance(a, torch.Tensor) else a for a in args)

    def launch(stream):
        code = fn(*conv, stream.cuda_stream)
        if code:
            native.check(code, name)

    launch.keep = args
    return launch


def spans_multi(items, stream=None) -> list:
    """sccsum_spans_multi: items = [(PacketBatch, out | None, status | None[, seeds int32]), ...]."""
    ml = max((it[0].max_len for it in items), default=0)
    outs = _multi(native.load().sccsum_spans_multi, "sccsum_spans_multi", items, ml, stream, 1, True)
    return [o[: it[0].n] for o, it in zip(outs, items)]


def ipv4_fill(batch: PacketBatch, mode: int = native.FILL_IP | native.FILL_L4, out2: torch.Tensor | None = None,
              status: torch.Tensor | None = None, stream=None) -> torch.Tensor | None:
    """sccsum_ipv4_fill: generate checksums and store them in batch.data in
    place.  FILL_L4 / FILL_ICMP_ECHO read every byte: up to 524 288 frames
    (sccsum_set_fill_single_max) in one pass whose tiles store the fields
    themselves, a larger fill as two kernels on the stream (the generate pass
    into out2, then the field-store pass); the header-only modes read only
    the headers.  out2 / status are optional reports of what was stored;
    without out2 the generate pass's words go through a scratch buffer from
    torch's caching allocator (not the library's stream-ordered hipMallocAsync,
    which sits outside torch's pool and can fail when torch has cached most of
    HBM).  Returns the [n, 2] values stored when out2 is given
    (else None)."""
    lib = native.load()
    n = batch.n
    _need(out2, 2 * n, torch.int16, "out2", batch.device)
    _need(status, n, torch.uint8, "status", batch.device)
    vals = out2
    if vals is None and mode & (native.FILL_L4 | native.FILL_ICMP_ECHO) and n:
        vals = _scratch(2 * n, batch.device, stream, torch.int16)
    code = lib.sccsum_ipv4_fill(
        ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off), ctypes_ptr(batch.length),
        _ptr(vals), _ptr(status), n, batch.max_len, mode, _stream(stream),
    )
    native.check(code, "sccsum_ipv4_fill")
    return None if out2 is None else out2[: 2 * n].view(n, 2)


# The reference's default RSS key (Mellanox driver key, toeplitz.hh:52-58).
RSS_KEY_40 = bytes.fromhex("d181c62cf7f4db5b1983a2fc943e1adbd9389e6bd1039c2ca74499ad593d56d9f3253c062adc1ffc")


def _key(key: bytes):
    kb = bytes(key)
    return (ctypes.c_uint8 * len(kb)).from_buffer_copy(kb), len(kb)


def ipv4_rss(batch: PacketBatch, key: bytes = RSS_KEY_40, mode: int = native.RSS_DISPATCH,
             hash_out: torch.Tensor | None = None, status: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """sccsum_ipv4_rss: the Toeplitz RSS hash of every frame (int32 tensor [n])."""
    lib = native.load()
    n = batch.n
    if hash_out is None:
        hash_out = _scratch(max(n, 1), batch.device, stream, torch.int32)
    _need(hash_out, n, torch.int32, "hash_out", batch.device)
    _need(status, n, torch.uint8, "status", batch.device)
    kb, kl = _key(key)
    code = lib.sccsum_ipv4_rss(ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off),
                               ctypes_ptr(batch.length), ctypes.addressof(kb), kl, mode, ctypes_ptr(hash_out),
                               _ptr(status), n, _stream(stream))
    native.check(code, "sccsum_ipv4_rss")
    return hash_out[:n]


def ipv4_frames_rss(batch: PacketBatch, key: bytes = RSS_KEY_40, mode: int = native.RSS_DISPATCH,
                    out2: torch.Tensor | None = None, status: torch.Tensor | None = None,
                    hash_out: torch.Tensor | None = None, stream=None):
    """sccsum_ipv4_frames_rss: ([n, 2] int16 checksums, [n] int32 RSS hashes) in one pass."""
    lib = native.load()
    n = batch.n
    if out2 is None:
        out2 = _scratch(max(2 * n, 2), batch.device, stream, torch.int16)
    if hash_out is None:
        hash_out = _scratch(max(n, 1), batch.device, stream, torch.int32)
    _need(out2, 2 * n, torch.int16, "out2", batch.device)
    _need(hash_out, n, torch.int32, "hash_out", batch.device)
    _need(status, n, torch.uint8, "status", batch.device)
    kb, kl = _key(key)
    code = lib.sccsum_ipv4_frames_rss(
        ctypes_ptr(batch.data), batch.bytes_len, ctypes_ptr(batch.off), ctypes_ptr(batch.length), ctypes_ptr(out2),
        _ptr(status), n, batch.max_len, ctypes.addressof(kb), kl, mode, ctypes_ptr(hash_out), _stream(stream))
    native.check(code, "sccsum_ipv4_frames_rss")
    return (out2[: 2 * n].view(n, 2) if n else out2[:0].view(0, 2)), hash_out[:n]


def fragments(data: torch.Tensor, bytes_len: int, frag_off: torch.Tensor, frag_len: torch.Tensor,
              pkt_first: torch.Tensor, seeds: torch.Tensor | None = None, out: torch.Tensor | None = None,
              status: torch.Tensor | None = None, max_frag_len: int = 0, stream=None) -> torch.Tensor:
    """sccsum_fragments: one checksum per fragment-list packet (int16 tensor)."""
    lib = native.load()
    n = int(pkt_first.numel()) - 1
    nfrag = int(frag_off.numel())
    if out is None:
        out = _scratch(max(n, 1), data.device, stream, torch.int16)
    dev = data.device
    if n < 0:
        raise ValueError("pkt_first needs n + 1 entries")
    _need(frag_off, nfrag, torch.int64, "frag_off", dev)
    _need(frag_len, nfrag, torch.int32, "frag_len", dev)
    _need(pkt_first, n + 1, torch.int32, "pkt_first", dev)
    _need(seeds, n, torch.int32, "seeds", dev)
    _need(out, n, torch.int16, "out", dev)
    _need(status, n, torch.uint8, "status", dev)
    ws = _scratch(int(lib.sccsum_fragments_workspace(nfrag)), data.device, stream)
    code = lib.sccsum_fragments(
        ctypes_ptr(data), bytes_len, ctypes_ptr(frag_off), ctypes_ptr(frag_len), nfrag, ctypes_ptr(pkt_first),
        _ptr(seeds), ctypes_ptr(out), _ptr(status), n, max_frag_len, ctypes_ptr(ws), _stream(stream))
    native.check(code, "sccsum_fragments")
    return out[:n]


DESC_DTYPE = np.dtype([("src", "<u8"), ("dst_off", "<u4"), ("len", "<u4")])  # sccsum_gather_desc


def make_desc(src, dst_off, length) -> np.ndarray:
    """sccsum_gather_desc records: src = absolute device-readable addresses
    (0 = in the stage buffer at dst_off), dst_off = the fragment's position in
    the packet layout (packet offset + offset inside the packet), length."""
    d = np.zeros(len(length), dtype=DESC_DTYPE)
    d["src"] = src
    d["dst_off"] = dst_off
    d["len"] = length
    return d


def _desc_call(name, desc, first, off, length, max_len, width, seeds, stage, out, status, stream):
    lib = native.load()
    n = int(off.numel())
    dev = off.device
    if int(first.numel()) != n + 1 or first.dtype != torch.int32 or (desc is not None and desc.dtype != torch.uint8):
        raise ValueError(f"{name}: first must be int32 [n + 1] and desc uint8 records (or None: no fragments)")
    if out is None:
        out = _scratch(max(width * n, width), dev, stream, torch.int16)
    _need(length, n, torch.int32, "length", dev)
    _need(seeds, n, torch.int32, "seeds", dev)
    _need(out, width * n, torch.int16, "out", dev)
    _need(status, n, torch.uint8, "status", dev)
    args = [_ptr(desc), ctypes_ptr(first), ctypes_ptr(off), ctypes_ptr(length)]
    if width == 1:
        args.append(_ptr(seeds))
    args += [None if stage is None else ctypes_ptr(stage), ctypes_ptr(out), _ptr(status), n, max_len, _stream(stream)]
    native.check(getattr(lib, name)(*args), name)
    return out


def spans_desc(desc: torch.Tensor, first: torch.Tensor, off: torch.Tensor, length: torch.Tensor, max_len: int,
               seeds: torch.Tensor | None = None, stage: torch.Tensor | None = None, out: torch.Tensor | None = None,
               status: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """sccsum_spans_desc: packets as fragment lists summed where the fragments
    lie (desc = make_desc records as a uint8 device tensor, first = int32
    [n + 1]); one int16 checksum per packet."""
    n = int(off.numel())
    return _desc_call("sccsum_spans_desc", desc, first, off, length, max_len, 1, seeds, stage, out, status,
                      stream)[:n]


def ipv4_frames_desc(desc: torch.Tensor, first: torch.Tensor, off: torch.Tensor, length: torch.Tensor, max_len: int,
                     stage: torch.Tensor | None = None, out2: torch.Tensor | None = None,
                     status: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """sccsum_ipv4_frames_desc: frames as fragment lists; [n, 2] int16."""
    n = int(off.numel())
    out2 = _desc_call("sccsum_ipv4_frames_desc", desc, first, off, length, max_len, 2, None, stage, out2, status,
                      stream)
    return out2[: 2 * n].view(n, 2) if n else out2[:0].view(0, 2)


def read_probe(buf: torch.Tensor, nbytes: int, sink: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Stream-read nbytes of buf with the kernels' load shape (HBM ceiling probe)."""
    lib = native.load()
    if sink is None:
        sink = torch.zeros(lib.sccsum_read_probe_blocks(), dtype=torch.int64, device=buf.device)
    native.check(lib.sccsum_read_probe(ctypes_ptr(buf), nbytes & ~15, ctypes_ptr(sink), _stream(stream)),
                 "sccsum_read_probe")
    return sink


def as_u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint16)


def pseudo_seed(src_host: int, dst_host: int, proto: int, length: int) -> int:
    return int(native.load().sccsum_pseudo_seed(src_host, dst_host, proto, length & 0xFFFF))


class Engine:
    """sccsum_engine_*: ONE resident grid that takes steps (up to 4 batches
    each: a step's tx and rx halves, a shard's rx queues) while it runs, so the
    launch's ramp, drain and kernel boundary are paid once per run instead of
    once per step (include/sccsum.h, "Resident engine").

        eng = Engine(device=0, frames=True, ring_slots=1024, max_in_flight=2)
        eng.start(stream)
        step = eng.submit([(tx, out2, None), (rx, None, status)])   # like prepare_ipv4_frames_multi's items
        eng.wait(step)                                               # results readable by a D2H copy
        eng.finish(); stream.synchronize()                           # wait on the last step, then stop

    A run takes any number of steps: their descriptors cycle through a ring
    of ring_slots slots (max_steps is its old name).  Any number of threads
    may submit into a running engine and wait on its steps (the shards of one
    GPU); start / stop / finish / close belong to its owner.  max_in_flight
    is shared by every producer; producer_in_flight (0: none) also limits each
    submitting thread's own steps not yet done.

    fill=True (frames): the run also takes in-place fills, each as a generate
    step and a store step (sccsum_engine_submit_fill):
        step = eng.submit_fill([(frames, out2, status)], FILL_IP | FILL_L4)

    A step's tensors must stay alive (and unmodified) until its wait returns;
    submit keeps a reference until then.  One engine runs per device at a time
    (start raises SccsumError(SCCSUM_EBUSY) while another engine's run holds
    it); while it runs, every other kernel on the device waits for its stop."""

    def __init__(self, device: int = 0, frames: bool = True, max_steps: int | None = None, max_in_flight: int = 2,
                 fill: bool = False, ring_slots: int | None = None, idle_ms: int = 0, dep_ms: int = 0,
                 producer_in_flight: int = 0):
        import threading

        self._lib = native.load()
        h = ctypes.c_void_p()
        mode = (native.PIPE_IPV4 if frames else native.PIPE_SPANS) | (native.ENGINE_FILL if fill else 0)
        ring = ring_slots if ring_slots is not None else (max_steps if max_steps is not None else 1024)
        opts = native.EngineOpts(int(ring), int(max_in_flight), int(idle_ms), int(dep_ms), int(producer_in_flight))
        if ring <= 0 or max_in_flight <= 0:  # (0 would mean "the default" to the C-ABI)
            raise ValueError("ring_slots and max_in_flight must be >= 1")
        if hasattr(self._lib, "sccsum_engine_create_opts"):
            native.check(self._lib.sccsum_engine_create_opts(int(device), mode, ctypes.byref(opts), ctypes.byref(h)),
                         "sccsum_engine_create_opts")
        else:  # an ABI 3 build under A/B (SCCSUM_LIB + SCCSUM_ABI_ANY): its runs end at ring_slots steps
            native.check(self._lib.sccsum_engine_create(int(device), mode, int(ring), int(max_in_flight),
                                                         ctypes.byref(h)), "sccsum_engine_create")
        self._h = h
        self.frames = frames
        self.fill = fill
        self.max_in_flight = int(max_in_flight)
        self._keep: dict[int, tuple] = {}
        self._mu = threading.Lock()  # _keep and _last: producers may be several threads
        self._last = -1  # the run's latest step
        self._stream = None

    def start(self, stream=None):
        s = torch.cuda.current_stream() if stream is None else stream
        native.check(self._lib.sccsum_engine_start(self._h, s.cuda_stream), "sccsum_engine_start")
        self._stream = s
        with self._mu:
            self._keep.clear()
            self._last = -1

    def prepare(self, items, fill_mode: int = 0):
        """A step's descriptor array, checked once (items as for
        prepare_ipv4_frames_multi: (PacketBatch, out | None, status | None
        [, seeds])); submit_prepared(prep) then only crosses the C-ABI.
        fill_mode != 0: an in-place fill of the items (out2 required)."""
        if not items or len(items) > native.ENGINE_MAX_BATCHES:
            raise ValueError(f"1..{native.ENGINE_MAX_BATCHES} batches per step")
        if fill_mode and not self.fill:
            raise ValueError("fill steps need Engine(..., fill=True)")
        width = 2 if self.frames else 1
        parts = []
        for i, it in enumerate(items):  # every item is checked before any is built
            b, out, status = it[0], it[1], it[2]
            seeds = it[3] if len(it) > 3 else None
            if self.frames and seeds is not None:
                raise ValueError("frames take no seeds")
            if fill_mode and out is None:
                raise ValueError(f"batch {i}: a fill step needs out2 (the values pass through it)")
            if out is None and status is None:
                raise ValueError(f"batch {i}: give out, status or both")
            _need(out, width * b.n, torch.int16, f"batch {i} out", b.device)
            _need(status, b.n, torch.uint8, f"batch {i} status", b.device)
            _need(seeds, b.n, torch.int32, f"batch {i} seeds", b.device)
            parts.append((b, out, status, seeds))
        arr = (native.Batch * len(items))()
        for i, (b, out, status, seeds) in enumerate(parts):
            arr[i] = native.Batch(ctypes_ptr(b.data), b.bytes_len, ctypes_ptr(b.off), ctypes_ptr(b.length),
                                  _ptr(seeds), _ptr(out), _ptr(status), b.n)
        return (arr, len(items), max(b.max_len for b, _, _, _ in parts), items, int(fill_mode))

    def submit_prepared(self, prep, timeout_s: float = 10.0) -> int:
        arr, nb, ml, items, fill_mode = prep
        step = ctypes.c_uint64()
        if fill_mode:
            native.check(self._lib.sccsum_engine_submit_fill(self._h, ctypes.cast(arr, ctypes.c_void_p), nb, ml,
                                                              fill_mode, int(timeout_s * 1e9), ctypes.byref(step)),
                         "sccsum_engine_submit_fill")
        else:
            native.check(self._lib.sccsum_engine_submit(self._h, ctypes.cast(arr, ctypes.c_void_p), nb, ml,
                                                         int(timeout_s * 1e9), ctypes.byref(step)),
                         "sccsum_engine_submit")
        s = step.value
        with self._mu:
            self._keep[s] = prep
            self._last = max(self._last, s)
            if len(self._keep) > 4 * self.max_in_flight + 8:
                # done: a step max_in_flight (+ 1 for a fill's pair) before the newest was waited for by a submit
                for k in [k for k in self._keep if k + self.max_in_flight + 1 < self._last]:
                    del self._keep[k]
        return s

    def submit(self, items, timeout_s: float = 10.0) -> int:
        return self.submit_prepared(self.prepare(items), timeout_s)

    def submit_fill(self, items, mode: int = native.FILL_IP | native.FILL_L4, timeout_s: float = 10.0) -> int:
        """In-place fill of items [(PacketBatch, out2, status | None), ...]:
        returns the store step, done once the frames hold their checksums."""
        return self.submit_prepared(self.prepare(items, fill_mode=mode), timeout_s)

    def wait(self, step: int, timeout_s: float = 10.0) -> None:
        native.check(self._lib.sccsum_engine_wait(self._h, int(step), int(timeout_s * 1e9)), "sccsum_engine_wait")

    @property
    def last_step(self) -> int:
        """The run's latest submitted step (-1: none yet)."""
        return self._last

    def stop(self) -> None:
        native.check(self._lib.sccsum_engine_stop(self._h), "sccsum_engine_stop")

    def finish(self, timeout_s: float = 10.0) -> None:
        """Stop the run, then wait until its latest step is done: a give-up
        (EIDLE) or fault (EFAULT) raises here instead of passing unseen
        (a timed run that only stopped never looked).  The stop
        comes first because the grid leaves once its published steps are done:
        stopped after the wait, it left ~20 us later per run, the time for a
        waiting wave to poll the host and see the stop
        (profiles/r06_run_cost.log)."""
        self.stop()
        if self._last >= 0:
            self.wait(self._last, timeout_s)

    def close(self) -> None:
        """Destroy the engine (stopping and synchronising a running one).
        Raises SccsumError when its last run left a published step undone
        (SCCSUM_EIDLE / SCCSUM_EFAULT from sccsum_engine_destroy)."""
        if self._h:
            h, self._h = self._h, None
            self._keep.clear()
            native.check(self._lib.sccsum_engine_destroy(h), "sccsum_engine_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
