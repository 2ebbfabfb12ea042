"""Generate tests/golden/vectors.json from the oracle (oracle/sccsum_oracle.c).

The oracle is pinned by tests/golden/kat.json (reference outputs recorded in
SURVEY.md §8(c) + RFC 1071/791 vectors) and by an independent closed form
(tests/test_oracle.py); these vectors freeze its outputs on edge cases so the
GPU tests can check the kernels against data, not only against a live oracle.

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

import oracle  # noqa: E402
from seastar_amd import synth  # noqa: E402


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
    off = np.array([s[0] for s in spans], np.uint64)
    lens = np.array([s[1] for s in spans], np.uint32)
    seeds = np.array([s[2] for s in spans], np.uint32)
    out = oracle.batch_spans(buf, off, lens, seeds)
    special = {
        "zeros_1500": oracle.ip_checksum(bytes(1500)),
        "ones_1500": oracle.ip_checksum(b"\xff" * 1500),
        "zeros_odd_1501": oracle.ip_checksum(bytes(1501)),
    }
    fbuf, foff, flen, meta = synth.udp_ipv4_frames(64, 200, seed=99)
    fout, fst = oracle.batch_ipv4(fbuf, foff, flen)
    doc = {
        "generator": "tests/golden/make_vectors.py (oracle/sccsum_oracle.c)",
        "span_buffer_hex": buf.tobytes().hex(),
        "spans": [{"off": int(o), "len": int(n), "seed": int(s), "out": int(r)}
                  for o, n, s, r in zip(off, lens, seeds, out)],
        "special": special,
        "frames": {"buffer_hex": fbuf.tobytes().hex(), "frame_len": 200,
                   "out": [[int(a), int(b)] for a, b in fout], "status": [int(x) for x in fst]},
    }
    json.dump(doc, open(os.path.join(HERE, "vectors.json"), "w"))
    print(f"{len(spans)} spans, {len(fout)} frames -> vectors.json")


if __name__ == "__main__":
    main()
