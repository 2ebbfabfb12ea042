"""The C-ABI library loads and exports every symbol include/sccsum.h declares,
plus the kept C++ per-packet API symbols; host-only entry
points behave (no compute calls: no GPU here)."""
import subprocess

import numpy as np

import oracle
from seastar_amd import native

CXX_API_SYMBOLS = [
    "_ZN7seastar3net11ip_checksumEPKvm",  # ip_checksum(void const*, unsigned long)
    "_ZN7seastar3net11checksummer3sumEPKcm",  # checksummer::sum(char const*, unsigned long)
    "_ZNK7seastar3net11checksummer3getEv",  # checksummer::get() const
]


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_symbols_exported():
    syms = native.header_symbols()
    assert len(syms) >= 10
    exported = _exported()
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_cxx_api_symbols_exported():
    exported = _exported()
    assert all(s in exported for s in CXX_API_SYMBOLS)


def test_library_loads_and_binds_every_symbol():
    lib = native.load()
    for s in native.header_symbols():
        assert hasattr(lib, s)
    assert lib.sccsum_abi_version() == native.ABI_VERSION == 4
    assert lib.sccsum_strerror(0) == b"success"
    assert lib.sccsum_strerror(native.SCCSUM_EINVAL) == b"invalid argument"


def test_pseudo_seed_matches_oracle():
    rng = np.random.default_rng(0)
    lib = native.load()
    for _ in range(2000):
        src, dst = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
        proto = int(rng.choice([6, 17, 1, 255]))
        length = int(rng.integers(0, 65537))
        assert lib.sccsum_pseudo_seed(src, dst, proto, length & 0xFFFF) == oracle.pseudo_seed(src, dst, proto,
                                                                                              length)


def test_argument_validation_without_device():
    lib = native.load()
    assert lib.sccsum_spans(None, 0, None, None, None, None, None, 0, 0, None) == 0
    assert lib.sccsum_ipv4_frames(None, 0, None, None, None, None, 0, 0, None) == 0
    assert lib.sccsum_spans(None, 64, None, None, None, None, None, 3, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_frames(None, 64, None, None, None, None, 3, 0, None) == native.SCCSUM_EINVAL
    # misaligned offset array
    assert lib.sccsum_spans(16, 64, 0x1004, 0x2000, None, 0x3000, None, 3, 0, None) == native.SCCSUM_EINVAL
    # misaligned out2 for frames (needs 4-byte alignment)
    assert lib.sccsum_ipv4_frames(16, 64, 0x1000, 0x2000, 0x3002, None, 3, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_read_probe(None, 16, None, None) == native.SCCSUM_EINVAL
    # fragment lists: empty is a no-op; missing workspace / misaligned workspace rejected
    assert lib.sccsum_fragments(None, 0, None, None, 0, None, None, None, None, 0, 0, None, None) == 0
    assert lib.sccsum_fragments(16, 64, 0x1000, 0x2000, 4, 0x3000, None, 0x4000, None, 2, 0, None, None) \
        == native.SCCSUM_EINVAL
    assert lib.sccsum_fragments(16, 64, 0x1000, 0x2000, 4, 0x3000, None, 0x4000, None, 2, 0, 0x5008, None) \
        == native.SCCSUM_EINVAL
    assert lib.sccsum_fragments_workspace(0) >= 16
    assert lib.sccsum_fragments_workspace(1000) >= 3 * 1000
    # in-place fill: mode checks come first, then n == 0 is a no-op
    F = native
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, F.FILL_L4 | F.FILL_L4_PSEUDO, None) \
        == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, F.FILL_IP | F.FILL_TSO, None) \
        == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, 0x20, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, F.FILL_ICMP_ECHO | F.FILL_L4_PSEUDO,
                                None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, F.FILL_ICMP_ECHO, None) == 0
    assert lib.sccsum_ipv4_fill(None, 64, None, None, None, None, 3, 0, F.FILL_ICMP_ECHO, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 0, None, None, None, None, 0, 0, F.FILL_IP | F.FILL_L4, None) == 0
    assert lib.sccsum_ipv4_fill(None, 64, None, None, None, None, 3, 0, F.FILL_IP, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_fill(None, 64, None, None, None, None, 3, 0, F.FILL_L4, None) == native.SCCSUM_EINVAL


def test_rss_argument_validation_without_device():
    lib = native.load()
    assert lib.sccsum_ipv4_rss(None, 0, None, None, None, 0, 0, None, None, 0, None) == 0  # n = 0: nothing to do
    assert lib.sccsum_ipv4_rss(None, 0, None, None, None, 0, 0, None, None, 1, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_frames_rss(None, 0, None, None, None, None, 1, 0, None, 40, 0, None, None) \
        == native.SCCSUM_EINVAL


def test_burst_argument_validation_without_device():
    import ctypes

    from seastar_amd import burst

    lib = native.load()
    out = ctypes.c_void_p()
    fn = burst.DONE_FN(lambda *a: None)
    cb = ctypes.cast(fn, ctypes.c_void_p)
    for args in ((0, 7, 1 << 20, 64, 0, 2),     # mode
                 (0, 0, 1 << 20, 64, 0, 0),     # depth 0
                 (0, 0, 1 << 20, 64, 0, 65),    # depth > 64
                 (0, 0, 1 << 20, 0, 0, 2),      # no packets per batch
                 (0, 1, 32, 64, 0, 2),          # batch under 64 bytes
                 (0, 1, 1 << 32, 64, 0, 2)):    # batch offsets are 32-bit: 4 GiB is too large
        assert lib.sccsum_burst_create(*args, cb, None, ctypes.byref(out)) == native.SCCSUM_EINVAL
    assert lib.sccsum_burst_create(0, 0, 1 << 20, 64, 0, 2, None, None, ctypes.byref(out)) == native.SCCSUM_EINVAL
    assert lib.sccsum_burst_submit(None, None, 0, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_burst_submit_mapped(None, None, 0, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_gather(None, 0, None, None) == native.SCCSUM_OK  # nothing to do
    assert lib.sccsum_gather(None, 1, None, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_gather(ctypes.c_void_p(12), 1, ctypes.c_void_p(64), None) == native.SCCSUM_EINVAL  # desc align
    assert lib.sccsum_burst_poll(None, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_burst_drain(None) == native.SCCSUM_EINVAL
    assert lib.sccsum_burst_destroy(None) == native.SCCSUM_OK
    assert lib.sccsum_strerror(native.SCCSUM_EBUSY).startswith(b"busy: every batch slot")
    assert ctypes.sizeof(native.Fragment) == 16  # char* base; size_t size (packet.hh:43-46)


def test_multi_batch_argument_validation_without_device():
    import ctypes

    lib = native.load()
    arr = (native.Batch * 17)()
    assert ctypes.sizeof(native.Batch) == 64
    assert lib.sccsum_ipv4_frames_multi(None, 0, 0, None) == native.SCCSUM_OK  # nothing to do
    assert lib.sccsum_spans_multi(ctypes.cast(arr, ctypes.c_void_p), 16, 0, None) == native.SCCSUM_OK  # all empty
    assert lib.sccsum_spans_multi(ctypes.cast(arr, ctypes.c_void_p), 17, 0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_multi(None, 2, 0, None) == native.SCCSUM_EINVAL
    arr[0] = native.Batch(16, 64, 0x1000, 0x2000, 0x3000, 0x4000, None, 3)
    # frames take no seeds
    assert lib.sccsum_ipv4_frames_multi(ctypes.cast(arr, ctypes.c_void_p), 1, 0, None) == native.SCCSUM_EINVAL
    arr[0] = native.Batch(17, 64, 0x1000, 0x2000, None, 0x4000, None, 3)  # misaligned bytes
    assert lib.sccsum_spans_multi(ctypes.cast(arr, ctypes.c_void_p), 1, 0, None) == native.SCCSUM_EINVAL


def test_desc_argument_validation_without_device():
    """sccsum_*_desc refuse null / misaligned arrays before any device call."""
    lib = native.load()
    p = 0x10000
    assert lib.sccsum_ipv4_frames_desc(None, None, None, None, None, None, None, 0, 0, None) == native.SCCSUM_OK
    # a NULL descriptor array is accepted (no packet has fragments), the other arrays are still checked
    assert lib.sccsum_ipv4_frames_desc(None, p, p, p, None, p + 2, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_frames_desc(None, None, p, p, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_frames_desc(p, None, p, p, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p + 4, p, p, p, None, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p, p + 2, p, p, None, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p, p, p + 4, p, None, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p, p, p, p + 1, None, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p, p, p, p, p + 2, None, p, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_spans_desc(p, p, p, p, None, None, p + 1, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_ipv4_frames_desc(p, p, p, p, None, p + 2, None, 4, 64, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_set_burst_fused(3) == native.SCCSUM_EINVAL
    assert lib.sccsum_set_burst_fused(2) == native.SCCSUM_OK


def test_engine_opts_layout_matches_the_header(tmp_path):
    """native.EngineOpts (ctypes) against sccsum_engine_opts as a C compiler
    lays it out from include/sccsum.h: size and every field's offset (a field
    added on one side only would shift the limits the engine reads)."""
    import ctypes
    import os

    src = tmp_path / "opts.c"
    fields = [name for name, _ in native.EngineOpts._fields_]
    body = "\n".join(f'    printf("{f} %zu\\n", offsetof(sccsum_engine_opts, {f}));' for f in fields)
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include <sccsum.h>\n"
                   "int main(void) {\n    printf(\"size %zu\\n\", sizeof(sccsum_engine_opts));\n"
                   f"{body}\n    return 0;\n}}\n")
    exe = str(tmp_path / "opts")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(repo, "include"), str(src), "-o", exe], check=True)
    got = dict(line.split() for line in subprocess.run([exe], check=True, capture_output=True,
                                                        text=True).stdout.splitlines())
    assert int(got["size"]) == ctypes.sizeof(native.EngineOpts)
    for f in fields:
        assert int(got[f]) == getattr(native.EngineOpts, f).offset, f
