"""The fourth exported symbol of the kept API:
checksummer::sum(const packet&) — seastar_amd/csrc/checksummer_packet.cc,
replacing src/net/ip_checksum.cc:64-68 — built against the reference's own
packet type (include/seastar/net/packet.hh, where it lies) and checked against
the oracle on packet_test.cc's chains and random fragment lists
(tests/cpp/packet_ref.cc).  Needs /root/reference: build container only."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_INCLUDE = "/root/reference/include"
SYM = "_ZN7seastar3net11checksummer3sumERKNS0_6packetE"  # seastar::net::checksummer::sum(packet const&)

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_INCLUDE), reason="needs /root/reference (build container only)")


def _cxx(tmp_path, *args):
    cmd = ["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-I", os.path.join(REPO, "include"), "-I", REF_INCLUDE,
           "-I", os.path.join(REPO, "oracle"), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    return r


def test_packet_symbol_built(tmp_path):
    obj = str(tmp_path / "checksummer_packet.o")
    _cxx(tmp_path, "-fPIC", "-c", os.path.join(REPO, "seastar_amd", "csrc", "checksummer_packet.cc"), "-o", obj)
    out = subprocess.run(["nm", "--defined-only", obj], capture_output=True, text=True, check=True).stdout
    assert SYM in {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_sum_packet_matches_oracle(tmp_path):
    oobj = str(tmp_path / "oracle.o")
    subprocess.run(["gcc", "-O2", "-c", os.path.join(REPO, "oracle", "sccsum_oracle.c"), "-o", oobj], check=True)
    exe = str(tmp_path / "packet_ref")
    _cxx(tmp_path, os.path.join(REPO, "tests", "cpp", "packet_ref.cc"),
         os.path.join(REPO, "seastar_amd", "csrc", "checksummer.cc"),
         os.path.join(REPO, "seastar_amd", "csrc", "checksummer_packet.cc"), oobj, "-o", exe, "-lpthread")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    # all four out-of-line symbols of SURVEY.md §8(b) are in the linked program
    out = subprocess.run(["nm", "--defined-only", exe], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for s in (SYM, "_ZN7seastar3net11ip_checksumEPKvm", "_ZN7seastar3net11checksummer3sumEPKcm",
              "_ZNK7seastar3net11checksummer3getEv"):
        assert s in syms, s
