"""Generate tests/golden/vectors.json: expected checksums derived from the
REFERENCE build of struct checksummer (oracle/_ref/checksummer_ref, see
make_ref_accum.py) — each input is pushed through the reference's inline
members (a pseudo-header through sum_many exactly as ip.hh:70-75 calls it,
bytes through sum(uint8_t)) and folded by get() (ip_checksum.cc:55-62, the one
restated step: ref_cases.fold_get).  The oracle must agree on every value
before the file is written.  The GPU tests check the kernels against it as
data.  Needs /root/reference (build container only); the JSON travels.

Frames follow the reference's rx path (ip.cc:114-140, 220-225: header sum
over sizeof(ip_hdr) = 20 bytes, L4 over [4*ihl, min(ip_len, len)) seeded with
the pseudo-header of that length as uint16_t, tcp.hh:876-883) — restated here
in Python to build the op strings.

usage: python tests/golden/make_vectors.py   (deterministic)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)

import oracle  # noqa: E402
from make_ref_accum import run_ref  # noqa: E402
from ref_cases import fold_get  # noqa: E402
from seastar_amd import synth  # noqa: E402


def ref_results(lines):
    return [fold_get(c) for c, _ in run_ref(lines)]


def frame_ops(f: bytes):
    """(ip ops, l4 ops, status bits) of one frame, or None for a short one."""
    n = len(f)
    if n < 20:
        return None
    ihl, ip_len, proto = f[0] & 0xF, (f[2] << 8) | f[3], f[9]
    st = 4 if n < ip_len else 0
    l4_off, l4_end = 4 * ihl, min(ip_len, n)
    if l4_off > l4_end:
        st |= 4
        l4 = b""
    else:
        l4 = f[l4_off:l4_end]
    src, dst = int.from_bytes(f[12:16], "big"), int.from_bytes(f[16:20], "big")
    return f"x:{f[:20].hex()}", f"ph:{src}:{dst}:{proto}:{len(l4) & 0xFFFF} x:{l4.hex()}", st


def main():
    rng = np.random.default_rng(0x5EA57A2C)
    buf = rng.integers(0, 256, size=4096 + 16, dtype=np.uint8)
    spans = []
    # every length 0..80 at start offsets 0..3 (head/tail/odd handling)
    for a in range(4):
        for n in range(81):
            spans.append((a, n, 0))
    # longer, odd and seeded
    for a, n in [(0, 1500), (1, 1500), (3, 1499), (5, 2048), (7, 4095), (0, 4096)]:
        spans.append((a, n, 0))
    for i in range(40):
        a, n = int(rng.integers(0, 16)), int(rng.integers(0, 4000))
        spans.append((a, n, int(rng.integers(0, 65536))))
    # a seed is the folded pseudo-header value a checksummer holds (< 2^16):
    # from a fresh checksummer sum(uint32_t(seed)) sets csum = seed exactly
    lines = [f"u32:{s} x:{buf[a:a + n].tobytes().hex()}" for a, n, s in spans]
    special_in = {"zeros_1500": "g:0:1500:1", "ones_1500": "g:0:1500:2", "zeros_odd_1501": "g:0:1501:1"}
    fbuf, foff, flen, meta = synth.udp_ipv4_frames(64, 200, seed=99)
    fops = [frame_ops(fbuf[int(o):int(o) + int(n)].tobytes()) for o, n in zip(foff, flen)]
    res = ref_results(lines + list(special_in.values()) + [x for ip, l4, _ in fops for x in (ip, l4)])
    out = res[:len(spans)]
    special = dict(zip(special_in, res[len(spans):len(spans) + 3]))
    fr = res[len(spans) + 3:]
    fout = [[fr[2 * i], fr[2 * i + 1]] for i in range(len(fops))]
    fst = [st | (1 if a == 0 else 0) | (2 if b == 0 else 0) for (_, _, st), (a, b) in zip(fops, fout)]

    # the oracle agrees on every value (the checker the GPU tests also use)
    off = np.array([s[0] for s in spans], np.uint64)
    lens = np.array([s[1] for s in spans], np.uint32)
    seeds = np.array([s[2] for s in spans], np.uint32)
    assert np.array_equal(oracle.batch_spans(buf, off, lens, seeds), np.array(out, np.uint16))
    o2, ost = oracle.batch_ipv4(fbuf, foff, flen)
    assert np.array_equal(o2, np.array(fout, np.uint16)) and np.array_equal(ost, np.array(fst, np.uint8))
    assert special == {"zeros_1500": oracle.ip_checksum(bytes(1500)), "ones_1500": oracle.ip_checksum(b"\xff" * 1500),
                       "zeros_odd_1501": oracle.ip_checksum(bytes(1501))}
    doc = {
        "generator": "tests/golden/make_vectors.py: reference build of struct checksummer "
                     "(oracle/_ref/checksummer_ref) + the get() fold; oracle agrees on every value",
        "span_buffer_hex": buf.tobytes().hex(),
        "spans": [{"off": int(o), "len": int(n), "seed": int(s), "out": int(r)}
                  for o, n, s, r in zip(off, lens, seeds, out)],
        "special": special,
        "frames": {"buffer_hex": fbuf.tobytes().hex(), "frame_len": 200, "out": fout, "status": fst},
    }
    json.dump(doc, open(os.path.join(HERE, "vectors.json"), "w"))
    print(f"{len(spans)} spans, {len(fout)} frames -> vectors.json")


if __name__ == "__main__":
    main()
