"""Host-side checks of the resident engine's Python wrapper (batch.Engine,
DESIGN.md §5.11) that need no device: a step's items are validated before
anything crosses the C-ABI (the C side's own argument checks run in
tests/cpp/abi_validate.cc)."""
import pytest
import torch

from seastar_amd import batch, native


def _engine(frames: bool, fill: bool = False) -> batch.Engine:
    e = object.__new__(batch.Engine)  # no device here: skip sccsum_engine_create
    e.frames, e.fill, e.max_in_flight, e._keep, e._h = frames, fill, 2, {}, None
    return e


def _batch(n=4, step=64):
    return batch.PacketBatch(data=torch.zeros(n * step + 16, dtype=torch.uint8),
                             off=torch.arange(n, dtype=torch.int64) * step,
                             length=torch.full((n,), step, dtype=torch.int32), bytes_len=n * step, max_len=step)


def test_step_holds_one_to_four_batches():
    e, b = _engine(True), _batch()
    st = torch.zeros(4, dtype=torch.uint8)
    with pytest.raises(ValueError, match="batches per step"):
        e.prepare([])
    with pytest.raises(ValueError, match="batches per step"):
        e.prepare([(b, None, st)] * (native.ENGINE_MAX_BATCHES + 1))


def test_items_are_checked_before_the_c_abi():
    b = _batch()
    with pytest.raises(ValueError, match="give out, status or both"):
        _engine(True).prepare([(b, None, None)])
    with pytest.raises(ValueError, match="frames take no seeds"):
        _engine(True).prepare([(b, torch.zeros(8, dtype=torch.int16), None, torch.zeros(4, dtype=torch.int32))])
    with pytest.raises(ValueError, match="batch 0 out"):  # frames write 2 values per frame
        _engine(True).prepare([(b, torch.zeros(4, dtype=torch.int16), None)])
    with pytest.raises(ValueError, match="batch 1 status"):
        _engine(False).prepare([(b, torch.zeros(4, dtype=torch.int16), None),
                                (b, None, torch.zeros(3, dtype=torch.uint8))])
    with pytest.raises(ValueError, match="batch 0 seeds"):
        _engine(False).prepare([(b, torch.zeros(4, dtype=torch.int16), None, torch.zeros(4, dtype=torch.int64))])
    # well-formed items on host tensors: refused for their memory, not their shape
    with pytest.raises(ValueError, match="device tensors"):
        _engine(True).prepare([(b, torch.zeros(8, dtype=torch.int16), torch.zeros(4, dtype=torch.uint8))])


def test_fill_steps_need_a_fill_engine_and_out2():
    b = _batch()
    st = torch.zeros(4, dtype=torch.uint8)
    with pytest.raises(ValueError, match="fill=True"):
        _engine(True).prepare([(b, torch.zeros(8, dtype=torch.int16), st)], fill_mode=native.FILL_L4)
    with pytest.raises(ValueError, match="needs out2"):
        _engine(True, fill=True).prepare([(b, None, st)], fill_mode=native.FILL_L4)
    with pytest.raises(ValueError, match="device tensors"):  # well-formed: refused for host memory only
        _engine(True, fill=True).prepare([(b, torch.zeros(8, dtype=torch.int16), st)], fill_mode=native.FILL_L4)


def test_close_without_a_handle_is_a_no_op():
    e = _engine(True)
    e.close()
    e.close()
