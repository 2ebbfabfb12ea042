"""Pins the oracle to the REFERENCE's own code (tests/golden/ref_accum.json).

ref_accum.json holds accumulator states (csum, odd) that the reference's
struct checksummer — include/seastar/net/ip_checksum.hh:35-69, compiled where
it lies by `make -C oracle ref` — reached on 6 155 op sequences
(tests/golden/make_ref_accum.py).  Here:

1. the oracle replays every sequence: its inline-member restatements
   (oracle_sum_u8/u16/u32, oracle_pseudo_header) must reach the reference's
   exact state; its byte loop (oracle_sum_bytes, the BE 64-bit word loop of
   src/net/ip_checksum.cc:31-53, fed at odd alignments and cut into
   fragments) must reach a state with the same residue mod 65535, the same
   zero-ness and the same odd flag — which is everything get() depends on;
2. oracle_get on the reference's state equals the fixture's `get`, and the
   oracle's own result equals it too: only the 8-line fold of
   ip_checksum.cc:55-62 remains a restatement (that TU needs boost/fmt);
3. the REPO's replacement header (include/seastar/net/ip_checksum.hh), driven
   by the same driver source, reproduces every state exactly — with
   /root/reference present also through its `__has_include(<seastar/net/
   packet.hh>)` branch against the reference's real packet.hh.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, GOLDEN)
from ref_cases import fold_get, op_bytes  # noqa: E402

DOC = json.load(open(os.path.join(GOLDEN, "ref_accum.json")))
CASES = DOC["cases"]
REF_INCLUDE = "/root/reference/include"


def _set_csum(c: oracle.Checksummer, v: int) -> None:
    c.csum_lo = v & ((1 << 64) - 1)
    c.csum_hi = v >> 64


def _replay(ops: str, frags, rng) -> tuple[oracle.Checksummer, bool]:
    L = oracle.lib()
    c = oracle.new()
    scalar_only = True
    nbyte_ops = 0
    for tok in ops.split():
        b = op_bytes(tok)
        if b is None:
            f = tok.split(":")
            if f[0] == "u8":
                L.oracle_sum_u8(ctypes.byref(c), int(f[1]))
            elif f[0] == "u16":
                L.oracle_sum_u16(ctypes.byref(c), int(f[1]))
            elif f[0] == "u32":
                L.oracle_sum_u32(ctypes.byref(c), int(f[1]))
            else:
                assert f[0] == "ph"
                L.oracle_pseudo_header(ctypes.byref(c), int(f[1]), int(f[2]), int(f[3]), int(f[4]) & 0xFFFF)
            continue
        scalar_only = False
        if frags is None:  # random cut points: the odd carry across fragments
            k = int(rng.integers(0, 4)) if len(b) > 1 else 0
            cuts = sorted(set(int(x) for x in rng.integers(1, max(len(b), 2), k))) if k else []
            pieces = [b[i:j] for i, j in zip([0] + cuts, cuts + [len(b)])]
        else:  # packet_test chains: one byte op per fragment, as the packet holds them
            assert len(b) == frags[nbyte_ops]
            pieces = [b]
        nbyte_ops += 1
        for p in pieces:
            if not p:
                continue
            a = int(rng.integers(0, 16))  # odd / unaligned starts for the 8-byte loads
            buf = np.zeros(len(p) + 32, np.uint8)
            buf[a:a + len(p)] = np.frombuffer(p, np.uint8)
            L.oracle_sum_bytes(ctypes.byref(c), buf.ctypes.data + a, len(p))
    return c, scalar_only


def test_fixture_covers_the_corpus():
    tags = {c["tag"].split(":")[0] for c in CASES}
    assert {"len", "zeros", "ones", "kat", "packet_test", "pseudo", "mixed"} <= tags
    assert sum(c["tag"] == "len" for c in CASES) == 4097
    # the uint16_t pseudo-header length wrap is in the corpus (ip.hh:70-75)
    assert any(":65536 " in c["ops"] for c in CASES if c["tag"] == "pseudo")


def test_oracle_reaches_reference_states():
    rng = np.random.default_rng(11)
    exact = 0
    for case in CASES:
        ref = int(case["csum"], 16)
        c, scalar_only = _replay(case["ops"], case.get("frags"), rng)
        ctx = case["ops"][:80]
        assert int(c.odd) == case["odd"], ctx
        if scalar_only:
            assert c.csum == ref, ctx  # the inline members: exact state
            exact += 1
        else:
            assert c.csum % 65535 == ref % 65535 and (c.csum == 0) == (ref == 0), ctx
        assert oracle.get(c) == case["get"], ctx
    assert exact > 100


def test_fold_on_reference_states():
    """oracle_get (ip_checksum.cc:55-62 in C) on the reference's exact states
    == the fixture's get == fold_get (the same 8 lines in Python)."""
    for case in CASES:
        ref = int(case["csum"], 16)
        c = oracle.new()
        _set_csum(c, ref)
        assert oracle.get(c) == case["get"] == fold_get(ref), case["ops"][:80]


def test_known_answers_through_reference_states():
    kat = {k["name"]: k for k in json.load(open(os.path.join(GOLDEN, "kat.json")))["ip_checksum"]}
    seen = 0
    for case in CASES:
        if case["tag"].startswith("kat:"):
            k = kat[case["tag"][4:]]
            assert case["get"] == int.from_bytes(bytes.fromhex(k["result_bytes"]), "little"), k["name"]
            seen += 1
    assert seen == len(kat)


def _driver(tmp_path, name, includes):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++20", "-O2", "-Wall", *[a for i in includes for a in ("-I", i)],
           os.path.join(REPO, "oracle", "ref", "checksummer_ref.cc"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def _run(exe):
    inp = "".join(c["ops"] + "\n" for c in CASES)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    return [(int(h, 16), int(o)) for h, o in (line.split() for line in out)]


def _expect():
    return [(int(c["csum"], 16), c["odd"]) for c in CASES]


def test_repo_header_reproduces_reference_states(tmp_path):
    """The replacement header's inline members, standalone (no packet.hh)."""
    got = _run(_driver(tmp_path, "ours", [os.path.join(REPO, "include")]))
    assert got == _expect()


@pytest.mark.skipif(not os.path.isdir(REF_INCLUDE), reason="needs /root/reference (build container only)")
def test_repo_header_inside_reference_tree(tmp_path):
    """The replacement header first on the include path, the reference tree
    after it: its __has_include branch pulls in the real packet.hh."""
    inc = [os.path.join(REPO, "include"), REF_INCLUDE]
    deps = subprocess.run(["g++", "-std=c++20", "-M", "-I", inc[0], "-I", inc[1],
                           os.path.join(REPO, "oracle", "ref", "checksummer_ref.cc")],
                          capture_output=True, text=True, check=True).stdout
    assert os.path.join(REPO, "include", "seastar", "net", "ip_checksum.hh") in deps
    assert os.path.join(REF_INCLUDE, "seastar", "net", "packet.hh") in deps
    assert os.path.join(REF_INCLUDE, "seastar", "net", "ip_checksum.hh") not in deps
    exe = _driver(tmp_path, "ours_in_tree", inc)
    assert _run(exe) == _expect()


@pytest.mark.skipif(not os.path.isdir(REF_INCLUDE), reason="needs /root/reference (build container only)")
def test_reference_build_reproduces_fixture():
    """The committed fixture is what the reference build prints today."""
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    assert _run(os.path.join(REPO, "oracle", "_ref", "checksummer_ref")) == _expect()
