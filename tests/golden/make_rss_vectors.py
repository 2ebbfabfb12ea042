"""Generate tests/golden/rss.json: Toeplitz hash vectors computed by the
REFERENCE's own toeplitz_hash (include/seastar/net/toeplitz.hh:78-98), built
where it lies by `make -C oracle ref` (oracle/ref/toeplitz_ref.cc driver ->
oracle/_ref/toeplitz_ref).  Needs /root/reference, so it runs in the build
container only; the JSON travels.

Cases: the Microsoft RSS verification suite (published key, 5 IPv4 flows,
IP-only and IP+TCP ports, published hashes — checked here against the
reference build), then random data of 0..16 bytes under the reference's two
default keys (40-byte Mellanox, 52-byte i40e) and under short 4..16-byte keys
(the `(i + 4) < key.size()` edge of toeplitz.hh:93).

usage: python tests/golden/make_rss_vectors.py   (deterministic)
"""
import json
import os
import socket
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "toeplitz_ref")

MS_KEY = "6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa"
# (destination, dst port, source, src port, IPv4-only hash, IPv4+TCP hash): the published table
MS_FLOWS = [
    ("161.142.100.80", 1766, "66.9.149.187", 2794, 0x323E8FC2, 0x51CCC178),
    ("65.69.140.83", 4739, "199.92.111.2", 14230, 0xD718262A, 0xC626B0EA),
    ("12.22.207.184", 38024, "24.19.198.95", 12898, 0xD2D0A5DE, 0x5C2B394A),
    ("209.142.163.6", 2217, "38.27.205.30", 48228, 0x82989176, 0xAFC7327F),
    ("202.188.127.2", 1303, "153.39.163.191", 44251, 0x5D1809C5, 0x10E828A2),
]
KEY40 = "d181c62cf7f4db5b1983a2fc943e1adbd9389e6bd1039c2ca74499ad593d56d9f3253c062adc1ffc"  # toeplitz.hh:52-58
KEY52 = ("4439796bb54c5023b675ea5b124f9f30b8a2c03ddfdc4d02a08c9b334af64a4c05c6fa343958d8557d99583ae138c92e"
         "81150366")  # toeplitz.hh:63-71


def ref_hashes(cases):
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    inp = "".join(f"{k} {d or '-'}\n" for k, d in cases)
    out = subprocess.run([REF], input=inp, capture_output=True, text=True, check=True).stdout.split()
    return [int(h, 16) for h in out]


def main():
    cases, expect = [], []
    for dst, dport, src, sport, h_ip, h_tcp in MS_FLOWS:
        ipd = socket.inet_aton(src) + socket.inet_aton(dst)
        cases.append((MS_KEY, ipd.hex()))
        expect.append(h_ip)
        cases.append((MS_KEY, (ipd + struct.pack(">HH", sport, dport)).hex()))
        expect.append(h_tcp)
    rng = np.random.default_rng(0x7E0)
    for key in (KEY40, KEY52):
        for n in list(range(0, 17)) + [8, 12, 12, 12, 8]:
            cases.append((key, rng.integers(0, 256, n, dtype=np.uint8).tobytes().hex()))
            expect.append(None)
    for klen in (4, 5, 8, 12, 15, 16):
        key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes().hex()
        for n in (0, 4, 8, 12, 13, 16):
            cases.append((key, rng.integers(0, 256, n, dtype=np.uint8).tobytes().hex()))
            expect.append(None)
    got = ref_hashes(cases)
    for (k, d), e, g in zip(cases, expect, got):
        assert e is None or e == g, f"reference build disagrees with the published vector: {k} {d} {g:08x} {e:08x}"
    doc = {
        "source": "reference build: include/seastar/net/toeplitz.hh via oracle/ref/toeplitz_ref.cc; "
                  "MS RSS verification suite rows checked against their published hashes",
        "cases": [{"key": k, "data": d, "hash": g} for (k, d), g in zip(cases, got)],
    }
    with open(os.path.join(HERE, "rss.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
