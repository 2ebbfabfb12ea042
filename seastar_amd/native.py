"""ctypes binding of the C-ABI in include/sccsum.h (libsccsum.so).

There is no fallback: if the library is missing or fails to load, every entry
point raises.  torch is imported before the library is opened so that both
share one HIP runtime (torch ships its own libamdhip64.so.7; our library's
NEEDED entry then resolves to the already-loaded copy).
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libsccsum.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "sccsum.h")
DIAG_HEADER_PATH = os.path.join(REPO_DIR, "include", "sccsum_diag.h")

SCCSUM_OK = 0
SCCSUM_EINVAL = -1
SCCSUM_ENODEV = -2
SCCSUM_EBUSY = -3
SCCSUM_EIDLE = -4
SCCSUM_EFAULT = -5
ST_OK = 0x01
ST_L4_OK = 0x02
ST_MALFORMED = 0x04
ST_RANGE = 0x08
ST_IPFRAG = 0x10
FILL_IP = 0x01
FILL_L4 = 0x02
FILL_L4_PSEUDO = 0x04
FILL_TSO = 0x08
FILL_ICMP_ECHO = 0x10
ABI_VERSION = 4


class SccsumError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        msg = what
        try:
            msg = f"{what}: {load().sccsum_strerror(code).decode()} ({code})"
        except Exception:  # noqa: BLE001 - best effort message
            msg = f"{what}: error {code}"
        super().__init__(msg)


_LIB = None

_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_vp = ctypes.c_void_p

_PROTOS = {
    "sccsum_abi_version": (ctypes.c_int, []),
    "sccsum_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "sccsum_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "sccsum_device_numa_node": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "sccsum_init": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_pseudo_seed": (_u32, [_u32, _u32, ctypes.c_uint8, ctypes.c_uint16]),
    "sccsum_spans": (ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, _vp, _u64, _u32, _vp]),
    "sccsum_ipv4_frames": (ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u64, _u32, _vp]),
    "sccsum_spans_multi": (ctypes.c_int, [_vp, _u32, _u32, _vp]),
    "sccsum_ipv4_frames_multi": (ctypes.c_int, [_vp, _u32, _u32, _vp]),
    "sccsum_sync": (ctypes.c_int, [_vp]),
    "sccsum_fragments": (ctypes.c_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp, _vp, _u64, _u32, _vp, _vp]),
    "sccsum_fragments_workspace": (_u64, [_u64]),
    "sccsum_ipv4_fill": (ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u64, _u32, _u32, _vp]),
    "sccsum_ipv4_rss": (ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _u32, ctypes.c_int, _vp, _vp, _u64, _vp]),
    "sccsum_ipv4_frames_rss": (ctypes.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u64, _u32, _vp, _u32, ctypes.c_int,
                                               _vp, _vp]),
    "sccsum_set_kernel_variant": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_blocks_per_cu": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_group_units": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_tile_packets": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_dynamic_tiles": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_tile_bytes": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_tail_split": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "sccsum_set_out_policy": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_engine_write_through": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_short_chunks": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_run_align": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_read_probe": (ctypes.c_int, [_vp, _u64, _vp, _vp]),
    "sccsum_read_probe_blocks": (ctypes.c_int, []),
    "sccsum_pipeline_create": (ctypes.c_int, [ctypes.c_int, _u64, _u32, ctypes.c_int, ctypes.POINTER(_vp)]),
    "sccsum_pipeline_run": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, _u64, _vp, _vp, _vp, _u64, _u32,
                                           _vp, _vp]),
    "sccsum_pipeline_destroy": (ctypes.c_int, [_vp]),
    "sccsum_burst_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _u64, _u32, _u64, ctypes.c_int, _vp, _vp,
                                           ctypes.POINTER(_vp)]),
    "sccsum_burst_submit": (ctypes.c_int, [_vp, _vp, _u32, _u32, ctypes.POINTER(_u64)]),
    "sccsum_burst_submit_mapped": (ctypes.c_int, [_vp, _vp, _u32, _u32, ctypes.POINTER(_u64)]),
    "sccsum_gather": (ctypes.c_int, [_vp, _u64, _vp, _vp]),
    "sccsum_spans_desc": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32, _vp]),
    "sccsum_ipv4_frames_desc": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32, _vp]),
    "sccsum_set_burst_fused": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_burst_poll": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "sccsum_burst_drain": (ctypes.c_int, [_vp]),
    "sccsum_burst_destroy": (ctypes.c_int, [_vp]),
    "sccsum_host_alloc": (ctypes.c_int, [ctypes.POINTER(_vp), _u64]),
    "sccsum_host_free": (ctypes.c_int, [_vp]),
    "sccsum_engine_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _u32, _u32, ctypes.POINTER(_vp)]),
    "sccsum_engine_create_opts": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(_vp)]),
    "sccsum_engine_start": (ctypes.c_int, [_vp, _vp]),
    "sccsum_engine_submit": (ctypes.c_int, [_vp, _vp, _u32, _u32, _u64, ctypes.POINTER(_u64)]),
    "sccsum_engine_submit_fill": (ctypes.c_int, [_vp, _vp, _u32, _u32, _u32, _u64, ctypes.POINTER(_u64)]),
    "sccsum_set_engine_idle_ms": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_engine_sync_every": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_set_fill_single_max": (ctypes.c_int, [ctypes.c_int]),
    "sccsum_engine_wait": (ctypes.c_int, [_vp, _u64, _u64]),
    "sccsum_engine_stop": (ctypes.c_int, [_vp]),
    "sccsum_engine_destroy": (ctypes.c_int, [_vp]),
}
PIPE_SPANS = 0
PIPE_IPV4 = 1
ENGINE_FILL = 0x100
GATHER_NONE = 0
GATHER_HOST = 1
GATHER_STRIDED = 2
GATHER_ZERO_COPY = 3
RSS_DISPATCH = 0
RSS_REASSEMBLED = 1


class Batch(ctypes.Structure):
    """sccsum_batch: one batch of a multi-batch launch."""
    _fields_ = [("d_bytes", ctypes.c_void_p), ("bytes_len", ctypes.c_uint64), ("d_off", ctypes.c_void_p),
                ("d_len", ctypes.c_void_p), ("d_seed", ctypes.c_void_p), ("d_out", ctypes.c_void_p),
                ("d_status", ctypes.c_void_p), ("n", ctypes.c_uint64)]


MAX_BATCHES = 16
FILL_SINGLE_MAX = 524288  # in-place fills of at most this many frames run in one pass (sccsum_diag.h)
ENGINE_MAX_BATCHES = 4


class EngineOpts(ctypes.Structure):
    """sccsum_engine_opts: a resident engine's limits (0 = the default)."""
    _fields_ = [("ring_slots", ctypes.c_uint32), ("max_in_flight", ctypes.c_uint32), ("idle_ms", ctypes.c_uint32),
                ("dep_ms", ctypes.c_uint32), ("producer_in_flight", ctypes.c_uint32)]


class Fragment(ctypes.Structure):
    """sccsum_fragment: the layout of seastar::net::fragment (packet.hh:43-46)."""
    _fields_ = [("base", ctypes.c_void_p), ("size", ctypes.c_size_t)]


def header_symbols() -> list[str]:
    """Every function declared in include/sccsum.h and include/sccsum_diag.h."""
    text = open(HEADER_PATH).read() + open(DIAG_HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sccsum_[a-z0-9_]+)\s*\(", text)))


def load():
    """Open libsccsum.so (raises if it is missing: there is no CPU fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  -- share torch's HIP runtime (see module doc)

    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    # SCCSUM_LIB: diagnostic override (A/B builds of the same ABI); still a native library, never a fallback
    lib = ctypes.CDLL(os.environ.get("SCCSUM_LIB", LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    # SCCSUM_ABI_ANY=1: diagnostic A/B against an older build (another ABI version; entry points it
    # lacks stay unbound); only ever set together with SCCSUM_LIB by tools/gpu_session.sh's lib: step
    any_abi = bool(os.environ.get("SCCSUM_ABI_ANY")) and "SCCSUM_LIB" in os.environ
    for name, (res, args) in _PROTOS.items():
        if any_abi and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sccsum_abi_version() != ABI_VERSION and not any_abi:
        raise RuntimeError(f"libsccsum ABI version {lib.sccsum_abi_version()} != {ABI_VERSION}: rebuild it")
    _LIB = lib
    return lib


def check(code: int, what: str) -> None:
    if code != SCCSUM_OK:
        raise SccsumError(code, what)
