"""The Python launch wrappers refuse arrays the kernels would read or write
past their ends (no device needed: the checks run before any launch)."""
import numpy as np
import pytest
import torch

from seastar_amd import batch


def _cpu_batch(n=8, frame=100, pad=0):
    total = n * frame
    return batch.PacketBatch(data=torch.zeros(((total + 15) & ~15) + pad, dtype=torch.uint8),
                             off=torch.arange(n, dtype=torch.int64) * frame,
                             length=torch.full((n,), frame, dtype=torch.int32), bytes_len=total, max_len=frame)


def test_packet_batch_accepts_the_kernel_layout():
    b = _cpu_batch()
    assert b.n == 8 and b.bytes_len == 800
    b = batch.PacketBatch.from_host(np.arange(37, dtype=np.uint8), np.array([0, 5], np.uint64),
                                    np.array([5, 32], np.uint32), device="cpu")
    assert b.data.numel() == 48 and b.max_len == 32


@pytest.mark.parametrize("bad", ["short_data", "data_dtype", "off_dtype", "len_dtype", "len_count", "data_2d",
                                 "negative_max_len", "strided_off"])
def test_packet_batch_refuses_bad_arrays(bad):
    n, frame = 8, 100
    kw = dict(data=torch.zeros(800, dtype=torch.uint8), off=torch.arange(n, dtype=torch.int64) * frame,
              length=torch.full((n,), frame, dtype=torch.int32), bytes_len=n * frame, max_len=frame)
    if bad == "short_data":
        kw["bytes_len"] = 801  # needs 816 padded bytes
    elif bad == "data_dtype":
        kw["data"] = torch.zeros(800, dtype=torch.int8)
    elif bad == "off_dtype":
        kw["off"] = kw["off"].to(torch.int32)
    elif bad == "len_dtype":
        kw["length"] = kw["length"].to(torch.int64)
    elif bad == "len_count":
        kw["length"] = kw["length"][:-1]
    elif bad == "data_2d":
        kw["data"] = kw["data"].view(8, 100)
    elif bad == "negative_max_len":
        kw["max_len"] = -1
    elif bad == "strided_off":
        kw["off"] = (torch.arange(2 * n, dtype=torch.int64) * frame)[::2]
    with pytest.raises(ValueError):
        batch.PacketBatch(**kw)


def test_wrappers_refuse_short_outputs():
    b = _cpu_batch()
    with pytest.raises(ValueError, match="out"):
        batch.spans(b, out=torch.empty(7, dtype=torch.int16))
    with pytest.raises(ValueError, match="seeds"):
        batch.spans(b, seeds=torch.zeros(8, dtype=torch.int64))
    with pytest.raises(ValueError, match="out2"):
        batch.ipv4_frames(b, out2=torch.empty(15, dtype=torch.int16))
    with pytest.raises(ValueError, match="status"):
        batch.ipv4_frames(b, status=torch.empty(7, dtype=torch.uint8))
    with pytest.raises(ValueError, match="status"):
        batch.verify_frames(b, torch.empty(8, dtype=torch.int8))
    with pytest.raises(ValueError, match="out2"):
        batch.ipv4_fill(b, out2=torch.empty(4, dtype=torch.int16))
    with pytest.raises(ValueError, match="hash_out"):
        batch.ipv4_rss(b, hash_out=torch.empty(7, dtype=torch.int32))
    with pytest.raises(ValueError, match="batch 1 status"):
        batch.ipv4_frames_multi([(b, None, None), (b, None, torch.empty(3, dtype=torch.uint8))])
    with pytest.raises(ValueError, match="batch 0"):
        batch.prepare_ipv4_frames_multi([(b, None, None)])
    with pytest.raises(ValueError, match="pkt_first"):
        batch.fragments(b.data, b.bytes_len, b.off, b.length, torch.arange(4, dtype=torch.int64))
    with pytest.raises(ValueError, match="frag_len"):
        batch.fragments(b.data, b.bytes_len, b.off, b.length[:5], torch.arange(4, dtype=torch.int32))


def test_host_pipeline_refuses_mismatched_arrays():
    """HostPipeline.run checks its host arrays before the native call (the
    pipeline object here is never created on a device)."""
    from seastar_amd import native, pipeline

    pl = pipeline.HostPipeline.__new__(pipeline.HostPipeline)
    pl._lib, pl._h = native.load(), None
    buf = np.zeros(4096, np.uint8)
    off = np.array([0, 100, 200], np.uint64)
    lens = np.array([50, 50, 50], np.uint32)
    with pytest.raises(ValueError, match="one entry per packet"):
        pl.run(native.PIPE_IPV4, buf, off, lens[:2])
    with pytest.raises(ValueError, match="one entry per packet"):
        pl.run(native.PIPE_SPANS, buf, off, lens, seeds=np.zeros(2, np.uint32))
    with pytest.raises(ValueError, match="contiguous uint8"):
        pl.run(native.PIPE_IPV4, buf.view(np.uint32), off, lens)
    with pytest.raises(ValueError, match="contiguous uint8"):
        pl.run(native.PIPE_IPV4, buf[::2], off, lens)
