"""The resident engine (sccsum_engine_*, include/sccsum.h "Resident engine";
DESIGN.md §5.11): steps streamed into one running grid give, step by step,
exactly what one multi launch per step gives — and the oracle — for frames
(verify-only halves included) and seeded spans; pacing by max_in_flight; runs
stopped and started again; empty steps; a grid left idle leaves on its own.
While a grid runs it holds every CU, so the tests launch no other kernel
until it has stopped (results are compared afterwards)."""
import numpy as np
import pytest
import torch

import oracle
from seastar_amd import batch, native, synth

pytestmark = pytest.mark.gpu


def _frames_step(rng, dev, kind):
    if kind == 0:
        buf, off, lens, _ = synth.udp_ipv4_frames(int(rng.integers(200, 3000)), 1500, seed=int(rng.integers(1 << 30)))
    elif kind == 1:
        buf, off, lens, _ = synth.mixed_udp_frames(int(rng.integers(100, 4000)), seed=int(rng.integers(1 << 30)),
                                                   max_gap=3)
    else:  # the tx generator's odd frames: options, padding, truncation, runts, fragments
        n = int(rng.integers(50, 900))
        lens = rng.integers(0, 2200, n).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 5, n))[:-1]]).astype(np.uint64)
        buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 8, dtype=np.uint8)
        for i in range(n):
            o, L = int(off[i]), int(lens[i])
            if L >= 20:
                ihl = 5 + int(rng.integers(0, 3))
                ipl = L if rng.random() < 0.8 else max(0, L - int(rng.integers(0, 9)))
                buf[o], buf[o + 2], buf[o + 3] = 0x40 | ihl, ipl >> 8, ipl & 0xFF
                buf[o + 6], buf[o + 7] = (0x20 if rng.random() < 0.1 else 0), 0
                buf[o + 9] = (17, 6, 1)[int(rng.integers(0, 3))]
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    return b, want, want_st


def test_engine_frames_steps_match_oracle_and_multi(dev):
    """40 steps of 1-4 frame batches each (UDP 1500 B, Zipf frames at odd
    offsets, odd frames), some batches verify-only (status bits alone),
    through one run with 2 steps in flight: every step's outputs equal the
    oracle's and one multi launch's."""
    rng = np.random.default_rng(0xE1)
    steps = []
    for s in range(40):
        items, wants = [], []
        for q in range(int(rng.integers(1, 5))):
            b, want, want_st = _frames_step(rng, dev, int(rng.integers(0, 3)))
            verify_only = rng.random() < 0.3
            out = None if verify_only else torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
            st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
            items.append((b, out, st))
            wants.append((want, want_st))
        steps.append((items, wants))
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, max_steps=64, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    ids = [eng.submit(items) for items, _ in steps]
    for i in ids:
        eng.wait(i)
    eng.stop()
    stream.synchronize()
    for items, wants in steps:
        for (b, out, st), (want, want_st) in zip(items, wants):
            if out is not None:
                assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)
            assert np.array_equal(st.cpu().numpy(), want_st)
    # the same steps as multi launches: identical bits
    for items, _ in steps[:8]:
        outs = batch.ipv4_frames_multi([(b, None, None) for b, _, _ in items])
        torch.cuda.synchronize()
        for (b, out, st), o in zip(items, outs):
            if out is not None:
                assert torch.equal(out.view(-1, 2), o)
    eng.close()


def test_engine_spans_with_seeds(dev):
    """Seeded spans (the cfg 4 shape, smaller): steps of Zipf spans and 64 KiB
    segments with pseudo-header seeds, against the oracle."""
    rng = np.random.default_rng(0xE2)
    eng = batch.Engine(0, frames=False, max_steps=32, max_in_flight=3)
    stream = torch.cuda.Stream(device=dev)
    steps = []
    for s in range(12):
        if s % 3 == 2:
            n = 48
            lens = np.full(n, 65536 - (s % 2), dtype=np.uint32)
        else:
            n = int(rng.integers(100, 5000))
            lens = synth.zipf_lengths(n, seed=int(rng.integers(1 << 30)))
        off, total = synth.pack(lens, seed=int(rng.integers(1 << 30)), max_gap=5)
        buf = rng.integers(0, 256, total, dtype=np.uint8)
        seeds = rng.integers(0, 65536, n).astype(np.uint32)
        b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
        sd = torch.from_numpy(seeds.view(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        steps.append(((b, out, st, sd), oracle.batch_spans(buf, off, lens, seeds)))
    torch.cuda.synchronize()
    eng.start(stream)
    ids = [eng.submit([item]) for item, _ in steps]
    eng.wait(ids[-1])
    eng.stop()
    stream.synchronize()
    for (b, out, st, sd), want in steps:
        got = batch.as_u16(out)
        assert np.array_equal(got, want)
        assert np.array_equal(st.cpu().numpy(), (want == 0).astype(np.uint8))
    eng.close()


def test_engine_runs_restart_and_limits(dev):
    """A run takes at most max_steps steps (then EBUSY); stop and start begin a
    new run on the same engine; empty steps complete at once and the grid walks
    past them; wait on a step never submitted is refused."""
    rng = np.random.default_rng(0xE3)
    b, want, want_st = _frames_step(rng, dev, 0)
    eng = batch.Engine(0, frames=True, max_steps=5, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    empty = batch.PacketBatch(data=torch.zeros(16, dtype=torch.uint8, device=dev),
                              off=torch.zeros(0, dtype=torch.int64, device=dev),
                              length=torch.zeros(0, dtype=torch.int32, device=dev), bytes_len=0, max_len=0)
    outs = []
    for run in range(3):
        o = [torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev) for _ in range(4)]
        torch.cuda.synchronize()
        eng.start(stream)
        ids = [eng.submit([(b, o[0], None)]), eng.submit([(empty, None, torch.empty(1, dtype=torch.uint8,
                                                                                       device=dev))]),
               eng.submit([(b, o[1], None), (b, o[2], None)]), eng.submit([(b, o[3], None)])]
        eng.submit([(empty, None, torch.empty(1, dtype=torch.uint8, device=dev))])
        with pytest.raises(native.SccsumError) as e:  # the 6th step of a 5-step run
            eng.submit([(b, o[0], None)])
        assert e.value.code == native.SCCSUM_EBUSY
        for i in ids:
            eng.wait(i)
        with pytest.raises(native.SccsumError):
            eng.wait(99)
        eng.stop()
        stream.synchronize()
        outs.extend(o)
    for o in outs:
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
    eng.close()


def test_engine_grid_left_idle_leaves_on_its_own(dev):
    """A run started and never given a step nor a stop: its grid gives up after
    its idle limit (1 s), the stream drains, and the run reports SCCSUM_EIDLE;
    a new run then works."""
    rng = np.random.default_rng(0xE4)
    b, want, _ = _frames_step(rng, dev, 0)
    eng = batch.Engine(0, frames=True, max_steps=4, max_in_flight=1)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    eng.start(stream)
    stream.synchronize()  # returns once every wave has waited out the idle limit
    with pytest.raises(native.SccsumError) as e:
        eng.submit([(b, torch.empty(2 * b.n, dtype=torch.int16, device=dev), None)])
    assert e.value.code == native.SCCSUM_EIDLE
    with pytest.raises(native.SccsumError):
        eng.stop()
    out = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    eng.start(stream)
    eng.wait(eng.submit([(b, out, None)]))
    eng.stop()
    stream.synchronize()
    assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)
    eng.close()


def test_engine_large_steps_property(dev):
    """Bench-sized steps (2 x 262 144 x 1500 B frames, tx + verify-only rx) for
    16 steps over 4 rotated batch pairs: every rx frame verifies except the
    corrupted ones, and every tx output equals a multi launch's."""
    from seastar_amd import devsynth

    n = 262144
    R = 4
    txs = [devsynth.udp_frames(n, 1500, seed=900 + r, device=dev) for r in range(R)]
    ref = [batch.ipv4_frames(t) for t in txs]
    rxs = [devsynth.store_checksums(t, f) for t, f in zip(txs, ref)]
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    bad = torch.randperm(n, device=dev, generator=g)[: n // 100]
    for rx in rxs:
        devsynth.corrupt(rx, bad, byte=700)
    outs = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(R)]
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, max_steps=64, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    preps = [eng.prepare([(txs[r], outs[r], None), (rxs[r], None, sts[r])]) for r in range(R)]
    eng.start(stream)
    for k in range(16):
        eng.submit_prepared(preps[k % R])
    eng.stop()
    stream.synchronize()
    for r in range(R):
        assert torch.equal(outs[r].view(-1, 2), ref[r])
        assert int(((sts[r] & 2) == 0).sum()) == bad.numel()
    eng.close()


def test_engine_results_readable_while_the_grid_runs(dev):
    """The header's promise: a step's results may be read as soon as its wait
    returns, while the grid still runs (a host copy on another stream goes
    through a copy engine, not a kernel that would queue behind the grid)."""
    rng = np.random.default_rng(0xE5)
    items = []
    for _ in range(3):
        b, want, want_st = _frames_step(rng, dev, 0)
        items.append((b, torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev), want))
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, max_steps=8, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    eng.start(stream)
    ids = [eng.submit([(b, out, None)]) for b, out, _ in items]
    got = []
    for i, (b, out, want) in zip(ids, items):
        eng.wait(i)
        with torch.cuda.stream(side):
            host = out.to("cpu", non_blocking=False)
        got.append((host, want))
    eng.stop()  # raises SccsumError(EIDLE) if a copy had queued behind the grid past its idle limit
    stream.synchronize()
    for host, want in got:
        assert np.array_equal(host.numpy().view(np.uint16).reshape(-1, 2), want)
    eng.close()
