"""Host-side checks of the resident engine's Python wrapper (batch.Engine,
DESIGN.md §5.11) that need no device: a step's items are validated before
anything crosses the C-ABI (the C side's own argument checks run in
tests/cpp/abi_validate.cc)."""
import pytest
import torch

from seastar_amd import batch, native


def _engine(frames: bool, fill: bool = False, lib=None) -> batch.Engine:
    import threading

    e = object.__new__(batch.Engine)  # no device here: skip sccsum_engine_create
    e.frames, e.fill, e.max_in_flight, e._keep, e._h = frames, fill, 2, {}, None
    e._mu, e._last, e._lib = threading.Lock(), -1, lib
    return e


class _FakeLib:
    """Stands in for libsccsum's engine entry points: records the calls and
    returns the codes a run that went wrong would."""

    def __init__(self, destroy=0, wait=0, stop=0):
        self.codes = {"destroy": destroy, "wait": wait, "stop": stop}
        self.calls = []

    def sccsum_engine_destroy(self, h):
        self.calls.append(("destroy", h))
        return self.codes["destroy"]

    def sccsum_engine_wait(self, h, step, timeout_ns):
        self.calls.append(("wait", step))
        return self.codes["wait"]

    def sccsum_engine_stop(self, h):
        self.calls.append(("stop", h))
        return self.codes["stop"]


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


@pytest.mark.parametrize("code", [native.SCCSUM_EIDLE, native.SCCSUM_EFAULT])
def test_close_raises_when_the_run_left_a_step_undone(code):
    """sccsum_engine_destroy's report of a run that left a
    published step undone (SCCSUM_EIDLE, SCCSUM_EFAULT) raises from close()
    instead of being dropped; the handle is released either way, and a
    second close is a no-op."""
    lib = _FakeLib(destroy=code)
    e = _engine(True, lib=lib)
    e._h = 0x1234
    with pytest.raises(native.SccsumError) as err:
        e.close()
    assert err.value.code == code
    assert lib.calls == [("destroy", 0x1234)] and e._h is None
    e.close()
    assert lib.calls == [("destroy", 0x1234)]
    ok = _FakeLib()
    e2 = _engine(True, lib=ok)
    e2._h = 0x99
    e2.close()
    assert ok.calls == [("destroy", 0x99)]


def test_finish_stops_then_waits_on_the_last_step():
    """finish(): stop (the grid leaves once its published steps are done),
    then wait on the run's latest step — a give-up seen by the wait, or
    reported by the stop itself, raises."""
    lib = _FakeLib()
    e = _engine(True, lib=lib)
    e._h, e._last = 0x10, 41
    e.finish()
    assert lib.calls == [("stop", 0x10), ("wait", 41)]
    bad = _FakeLib(wait=native.SCCSUM_EIDLE)
    e = _engine(True, lib=bad)
    e._h, e._last = 0x11, 7
    with pytest.raises(native.SccsumError) as err:
        e.finish()
    assert err.value.code == native.SCCSUM_EIDLE
    assert bad.calls == [("stop", 0x11), ("wait", 7)]
    gave_up = _FakeLib(stop=native.SCCSUM_EFAULT)
    e = _engine(True, lib=gave_up)
    e._h, e._last = 0x13, 3
    with pytest.raises(native.SccsumError) as err:
        e.finish()
    assert err.value.code == native.SCCSUM_EFAULT
    assert gave_up.calls == [("stop", 0x13)]
    none = _FakeLib()
    e = _engine(True, lib=none)
    e._h = 0x12
    e.finish()  # no step submitted: nothing to wait on
    assert none.calls == [("stop", 0x12)]
