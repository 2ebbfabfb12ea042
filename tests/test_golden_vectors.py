"""Committed golden vectors (tests/golden/vectors.json): the oracle still
reproduces them (CPU), and the HIP kernels match them (GPU)."""
import json
import os

import numpy as np
import pytest

import oracle

V = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")))


def _spans():
    buf = np.frombuffer(bytes.fromhex(V["span_buffer_hex"]), np.uint8)
    off = np.array([s["off"] for s in V["spans"]], np.uint64)
    lens = np.array([s["len"] for s in V["spans"]], np.uint32)
    seeds = np.array([s["seed"] for s in V["spans"]], np.uint32)
    want = np.array([s["out"] for s in V["spans"]], np.uint16)
    return buf, off, lens, seeds, want


def _frames():
    f = V["frames"]
    buf = np.frombuffer(bytes.fromhex(f["buffer_hex"]), np.uint8)
    n = len(f["out"])
    off = np.arange(n, dtype=np.uint64) * f["frame_len"]
    lens = np.full(n, f["frame_len"], np.uint32)
    return buf, off, lens, np.array(f["out"], np.uint16), np.array(f["status"], np.uint8)


def test_oracle_reproduces_vectors():
    buf, off, lens, seeds, want = _spans()
    assert np.array_equal(oracle.batch_spans(buf, off, lens, seeds), want)
    fb, fo, fl, fw, fs = _frames()
    out, st = oracle.batch_ipv4(fb, fo, fl)
    assert np.array_equal(out, fw) and np.array_equal(st, fs)
    assert oracle.ip_checksum(bytes(1500)) == V["special"]["zeros_1500"] == 0xFFFF
    assert oracle.ip_checksum(b"\xff" * 1500) == V["special"]["ones_1500"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2, 15, 16])
def test_kernels_match_vectors(dev, variant):
    import torch

    from seastar_amd import batch, native

    lib = native.load()
    native.check(lib.sccsum_set_kernel_variant(variant), "variant")
    try:
        buf, off, lens, seeds, want = _spans()
        b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
        sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
        got = batch.as_u16(batch.spans(b, seeds=sd))
        assert np.array_equal(got, want)
        fb, fo, fl, fw, fs = _frames()
        b = batch.PacketBatch.from_host(fb, fo, fl, device=dev)
        st = torch.empty(b.n, dtype=torch.uint8, device=dev)
        got = batch.as_u16(batch.ipv4_frames(b, status=st))
        assert np.array_equal(got, fw) and np.array_equal(st.cpu().numpy(), fs)
    finally:
        native.check(lib.sccsum_set_kernel_variant(0), "variant")
