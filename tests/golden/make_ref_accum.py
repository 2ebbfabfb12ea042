"""Generate tests/golden/ref_accum.json: checksummer accumulator states
computed by the REFERENCE's own struct checksummer
(include/seastar/net/ip_checksum.hh:35-69: sum(uint8_t/uint16_t/uint32_t),
sum_many), built where it lies by `make -C oracle ref`
(oracle/ref/checksummer_ref.cc -> oracle/_ref/checksummer_ref).  Needs
/root/reference, so it runs in the build container only; the JSON travels.

Corpus (every case starts from a fresh checksummer):
  - every length 0..4096 of splitmix bytes; all-zero / all-0xff spans of
    0..64 bytes and of MTU / jumbo / 64 KiB lengths;
  - the known-answer inputs of tests/golden/kat.json;
  - packet_test.cc:32-84's fragment chain (5/31/65/4096/4096 bytes of
    'a'/'b'/'c'/'c'/'d', trimmed by 1, 6, 29, 1024, then 9 'z' + 7 'x'
    appended), with the fragment sizes each state has;
  - pseudo-headers exactly as ip.hh:70-75 calls sum_many, including the
    uint16_t length wrap (65536 -> 0) and a pseudo-header after an odd byte,
    followed by payload;
  - random sequences of all the ops.

usage: python tests/golden/make_ref_accum.py   (deterministic)
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "checksummer_ref")
sys.path.insert(0, HERE)

from ref_cases import fold_get  # noqa: E402


def packet_test_chain():
    """(case ops, fragment sizes) after each step of packet_test.cc:32-84."""
    frags = [(ord("a"), 5), (ord("b"), 31), (ord("c"), 65), (ord("c"), 4096), (ord("d"), 4096)]
    out = []

    def emit():
        out.append((" ".join(f"rep:{v}:{n}" for v, n in frags if n), [n for _, n in frags if n]))

    emit()
    for trim in (1, 6, 29, 1024):  # packet::trim_front (packet.hh:545-565)
        while trim:
            v, n = frags[0]
            k = min(n, trim)
            trim -= k
            frags[0] = (v, n - k)
            if frags[0][1] == 0:
                frags.pop(0)
        emit()
    frags += [(ord("z"), 9), (ord("x"), 7)]  # p.append(p2)
    emit()
    return out


def cases():
    rng = np.random.default_rng(0x5EA57A2C)
    cs = []  # (ops, frags or None, tag)
    for n in range(4097):
        cs.append((f"g:{1000 + n}:{n}:0", None, "len"))
    for n in list(range(65)) + [1499, 1500, 1501, 4095, 4096, 9000, 65535, 65536]:
        cs.append((f"g:0:{n}:1", None, "zeros"))
        cs.append((f"g:0:{n}:2", None, "ones"))
    kat = json.load(open(os.path.join(HERE, "kat.json")))
    for k in kat["ip_checksum"]:
        cs.append((f"x:{k['hex']}" if k["hex"] else "", None, "kat:" + k["name"]))
    for ops, fr in packet_test_chain():
        cs.append((ops, fr, "packet_test"))
    for i in range(400):
        src, dst = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
        proto = int(rng.choice([6, 17, 1, 255]))
        ln = int(rng.choice([0, 8, 1480, 65516, 65535, 65536, 65537, int(rng.integers(0, 70000))]))
        pre = "u8:%d " % int(rng.integers(0, 256)) if i % 7 == 3 else ""
        payload = min(ln & 0xFFFF, 3000) if i % 2 else int(rng.integers(0, 64))
        cs.append((f"{pre}ph:{src}:{dst}:{proto}:{ln} g:{50000 + i}:{payload}:0", None, "pseudo"))
    for i in range(1500):
        ops = []
        for _ in range(int(rng.integers(1, 13))):
            k = int(rng.integers(0, 6))
            if k == 0:
                ops.append(f"u8:{int(rng.integers(0, 256))}")
            elif k == 1:
                ops.append(f"u16:{int(rng.integers(0, 65536))}")
            elif k == 2:
                ops.append(f"u32:{int(rng.integers(0, 2**32, dtype=np.uint64))}")
            elif k == 3:
                src, dst = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
                ops.append(f"ph:{src}:{dst}:{int(rng.choice([6, 17]))}:{int(rng.integers(0, 65537))}")
            elif k == 4:
                ops.append("x:" + rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes().hex())
            else:
                ops.append(f"g:{90000 + i}:{int(rng.integers(0, 300))}:0")
        cs.append((" ".join(ops), None, "mixed"))
    return cs


def run_ref(lines):
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    out = subprocess.run([REF], input="".join(line + "\n" for line in lines), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    assert len(out) == len(lines)
    res = []
    for line in out:
        h, odd = line.split()
        res.append((int(h, 16), int(odd)))
    return res


def main():
    cs = cases()
    states = run_ref([c[0] for c in cs])
    doc = {
        "source": "reference build: struct checksummer inline members of include/seastar/net/ip_checksum.hh:35-69 "
                  "(oracle/ref/checksummer_ref.cc -> oracle/_ref/checksummer_ref, g++ -std=c++20 -O2); "
                  "byte ops fed through sum(uint8_t)",
        "fold": "get = ip_checksum.cc:55-62 applied to csum (a restatement: that TU does not build here)",
        "cases": [{"ops": ops, "tag": tag, "csum": format(cs_, "x"), "odd": odd, "get": fold_get(cs_),
                   **({"frags": fr} if fr else {})}
                  for (ops, fr, tag), (cs_, odd) in zip(cs, states)],
    }
    with open(os.path.join(HERE, "ref_accum.json"), "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"{len(cs)} cases -> ref_accum.json")


if __name__ == "__main__":
    main()
