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
    eng = batch.Engine(0, frames=True, ring_slots=64, max_in_flight=2)
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
    eng = batch.Engine(0, frames=False, ring_slots=32, max_in_flight=3)
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


def test_engine_runs_restart_and_outlast_their_ring(dev):
    """A run takes any number of steps: with a ring of 5 (rounded up to 8)
    descriptor slots, 3 runs of 30 steps each (real and empty ones) all
    complete exact (ABI 4; a run of max_steps steps used to end in EBUSY);
    stop and start begin a new run on the same engine; empty steps complete at
    once and the grid walks past them; wait on a step never submitted is
    refused."""
    rng = np.random.default_rng(0xE3)
    b, want, want_st = _frames_step(rng, dev, 0)
    eng = batch.Engine(0, frames=True, ring_slots=5, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    empty = batch.PacketBatch(data=torch.zeros(16, dtype=torch.uint8, device=dev),
                              off=torch.zeros(0, dtype=torch.int64, device=dev),
                              length=torch.zeros(0, dtype=torch.int32, device=dev), bytes_len=0, max_len=0)
    empty_st = torch.empty(1, dtype=torch.uint8, device=dev)
    outs = []
    for run in range(3):
        o = [torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev) for _ in range(20)]
        torch.cuda.synchronize()
        eng.start(stream)
        ids = []
        for k in range(10):
            ids.append(eng.submit([(b, o[2 * k], None)]))
            ids.append(eng.submit([(empty, None, empty_st)]))
            ids.append(eng.submit([(b, o[2 * k + 1], None), (empty, None, empty_st)]))
        assert ids == list(range(30))
        for i in ids:
            eng.wait(i)
        with pytest.raises(native.SccsumError) as e:
            eng.wait(99)
        assert e.value.code == native.SCCSUM_EINVAL
        eng.finish()
        stream.synchronize()
        outs.extend(o)
    for o in outs:
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
    eng.close()


def test_engine_grid_left_idle_leaves_on_its_own(dev):
    """A run started and never given a step nor a stop: its grid gives up after
    its idle limit (1 s), the stream drains, and a submit reports SCCSUM_EIDLE
    (stop does not: no published step was lost); a new run then works."""
    rng = np.random.default_rng(0xE4)
    b, want, _ = _frames_step(rng, dev, 0)
    eng = batch.Engine(0, frames=True, ring_slots=4, max_in_flight=1)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    eng.start(stream)
    stream.synchronize()  # returns once every wave has waited out the idle limit
    with pytest.raises(native.SccsumError) as e:
        eng.submit([(b, torch.empty(2 * b.n, dtype=torch.int16, device=dev), None)])
    assert e.value.code == native.SCCSUM_EIDLE
    eng.stop()  # the give-up left no published step undone: nothing lost, 0
    out = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    eng.start(stream)
    eng.wait(eng.submit([(b, out, None)]))
    eng.stop()
    stream.synchronize()
    assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)
    eng.close()


def test_engine_large_steps_property(dev):
    """Bench-sized steps (2 x 524 288 x 1500 B frames, tx + verify-only rx) for
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
    eng = batch.Engine(0, frames=True, ring_slots=64, max_in_flight=2)
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
    eng = batch.Engine(0, frames=True, ring_slots=8, max_in_flight=2)
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


# ---- in-place fill through the engine (sccsum_engine_submit_fill) ---------------

ENGINE_FILL_MODES = {
    "ip_l4": native.FILL_IP | native.FILL_L4,
    "l4": native.FILL_L4,
    "icmp_echo": native.FILL_ICMP_ECHO,
    "ip_l4_icmp_echo": native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO,
}


@pytest.mark.parametrize("mode", list(ENGINE_FILL_MODES))
def test_engine_fill_steps_match_oracle(dev, mode, fill_passes):
    """Fill steps (generate, then the store step that waits for it) of the tx
    generator's odd frames — UDP / TCP / ICMP, options, padding, truncation,
    runts, IP fragments, garbage checksum fields, odd offsets — among verify
    steps of other batches, in one run: every filled buffer is byte-exact
    against the oracle's writers (ip.cc:266-278, udp.cc:184-195,
    tcp.hh:1656-1694, ip.cc:464-474), with its out2 values and status; each
    batch is filled again later in the same run, into fresh out2 / status
    (generate tiles then read bytes that store tiles of the same grid wrote):
    the oracle's second fill of its own first result — the same bytes (a fill
    is idempotent), and the values and status bits that second fill reports
    (an echo request answered by the first fill is a reply the second leaves
    alone); the verify steps equal the oracle too."""
    from test_gpu_parity import _tx_frames

    m = ENGINE_FILL_MODES[mode]
    rng = np.random.default_rng(0xEF00 + m)
    fills, verifies = [], []
    for k in range(6):
        items = []
        for q in range(int(rng.integers(1, 4))):
            buf, off, length = _tx_frames(rng, int(rng.integers(100, 1200)))
            b = batch.PacketBatch.from_host(buf, off, length, device=dev)
            out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
            st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev) if q != 1 else None
            want1 = oracle.batch_ipv4_fill(buf, off, length, m)
            want2 = oracle.batch_ipv4_fill(want1[0], off, length, m)
            again = (torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev),
                     torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev))
            items.append((b, out2, st, want1, again, want2))
        fills.append(items)
        b, want, want_st = _frames_step(rng, dev, int(rng.integers(0, 3)))
        out = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
        verifies.append((b, out, want))
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=64, max_in_flight=4)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    ids = []
    for items, (vb, vout, _) in zip(fills, verifies):
        ids.append(eng.submit_fill([(it[0], it[1], it[2]) for it in items], m))
        ids.append(eng.submit([(vb, vout, None)]))
    for items in fills:  # again
        ids.append(eng.submit_fill([(it[0], it[4][0], it[4][1]) for it in items], m))
    for i in ids:
        eng.wait(i)
    eng.stop()
    stream.synchronize()
    for items in fills:
        for b, out2, st, want1, (out2b, stb), want2 in items:
            got = b.data.cpu().numpy()[: b.bytes_len]
            assert np.array_equal(want2[0], want1[0])  # the oracle's own fill is idempotent
            bad = np.nonzero(got != want1[0])[0]
            assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
            assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want1[1])
            if st is not None:
                assert np.array_equal(st.cpu().numpy(), want1[2])
            assert np.array_equal(batch.as_u16(out2b).reshape(-1, 2), want2[1])
            assert np.array_equal(stb.cpu().numpy(), want2[2])
    for b, out, want in verifies:
        assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)
    eng.close()


def test_engine_fill_full_scale(dev):
    """cfg 2 tx at full size through the engine: 4 rotated 1 M x 1500 B batches
    with garbage checksum fields, filled 3 times each in one run; the fields
    equal classic generate (on zeroed fields), every frame verifies, and the
    out2 values are the ones stored."""
    from seastar_amd import devsynth

    n, R = 1 << 20, 4
    bs = [devsynth.udp_frames(n, 1500, seed=300 + r, device=dev) for r in range(R)]
    gens = [batch.ipv4_frames(b).clone() for b in bs]
    for b in bs:
        f = b.data[: n * 1500].view(n, 1500)
        f[:, 10:12] = 0xA5
        f[:, 26:28] = 0x3C
    outs = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(R)]
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=64, max_in_flight=8)
    stream = torch.cuda.Stream(device=dev)
    preps = [eng.prepare([(bs[r], outs[r], None)], fill_mode=native.FILL_IP | native.FILL_L4) for r in range(R)]
    eng.start(stream)
    last = [eng.submit_prepared(preps[k % R]) for k in range(3 * R)][-1]
    eng.wait(last)
    eng.stop()
    stream.synchronize()
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for b, gen, out in zip(bs, gens, outs):
        f = b.data[: n * 1500].view(n, 1500)
        got = torch.stack([f[:, 10:12].contiguous().view(torch.int16).view(-1),
                           f[:, 26:28].contiguous().view(torch.int16).view(-1)], dim=1)
        assert torch.equal(got, gen)
        assert torch.equal(out.view(n, 2), gen)
        batch.ipv4_frames(b, status=st)
        assert int((st == 3).sum()) == n
    eng.close()


# ---- sharing the device (include/sccsum.h, "Sharing the device") ---------------

def test_second_engine_on_the_device_is_refused(dev):
    """One engine runs per device: while the first run holds device 0, a second
    engine's start returns SCCSUM_EBUSY and changes nothing; the first run's
    results stay exact; after its stop the second engine runs."""
    rng = np.random.default_rng(0xE6)
    b, want, _ = _frames_step(rng, dev, 0)
    o1 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    o2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    e1 = batch.Engine(0, frames=True, ring_slots=8, max_in_flight=2)
    e2 = batch.Engine(0, frames=True, ring_slots=8, max_in_flight=2)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    e1.start(s1)
    with pytest.raises(native.SccsumError) as e:
        e2.start(s2)
    assert e.value.code == native.SCCSUM_EBUSY
    e1.wait(e1.submit([(b, o1, None)]))
    e1.stop()
    s1.synchronize()
    assert np.array_equal(batch.as_u16(o1).reshape(-1, 2), want)
    e2.start(s2)  # the device is free again
    e2.wait(e2.submit([(b, o2, None)]))
    e2.stop()
    s2.synchronize()
    assert np.array_equal(batch.as_u16(o2).reshape(-1, 2), want)
    e1.close()
    e2.close()


def test_launch_from_another_thread_completes_after_stop(dev):
    """Seastar's shared-device model: one shard runs the engine, another shard
    thread (its own sccsum_init, its own stream) launches frames meanwhile.
    The launch queues behind the resident grid and completes after the run's
    stop, with exact results; the engine's own steps are exact too."""
    import threading

    rng = np.random.default_rng(0xE7)
    b, want, _ = _frames_step(rng, dev, 0)
    b2, want2, want2_st = _frames_step(rng, dev, 1)
    o_eng = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    o_thr = torch.full((2 * b2.n,), -1, dtype=torch.int16, device=dev)
    st_thr = torch.full((b2.n,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=8, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    eng.wait(eng.submit([(b, o_eng, None)]))
    errors, launched, finished = [], threading.Event(), threading.Event()

    def shard():
        try:
            native.check(native.load().sccsum_init(0), "sccsum_init")
            s = torch.cuda.Stream(device=dev)
            batch.ipv4_frames(b2, out2=o_thr, status=st_thr, stream=s)
            launched.set()
            s.synchronize()
            finished.set()
        except Exception as ex:  # noqa: BLE001 - reported below
            errors.append(ex)
            launched.set()

    t = threading.Thread(target=shard)
    t.start()
    assert launched.wait(30)
    eng.wait(eng.submit([(b, o_eng, None)]))  # the engine keeps taking steps meanwhile
    eng.stop()
    stream.synchronize()
    t.join(60)
    assert not t.is_alive() and not errors, errors
    assert finished.is_set()
    assert np.array_equal(batch.as_u16(o_eng).reshape(-1, 2), want)
    assert np.array_equal(batch.as_u16(o_thr).reshape(-1, 2), want2)
    assert np.array_equal(st_thr.cpu().numpy(), want2_st)
    eng.close()


def test_engine_create_keeps_the_callers_device(dev):
    """sccsum_engine_create allocates on its device and leaves the calling
    thread's current device as it was (it used to switch it)."""
    import ctypes

    lib = native.load()
    ndev = ctypes.c_int()
    native.check(lib.sccsum_device_count(ctypes.byref(ndev)), "device count")
    target = ndev.value - 1  # another device where there is one
    torch.cuda.set_device(0)
    native.check(lib.sccsum_init(0), "sccsum_init")
    before = torch.cuda.current_device()
    eng = batch.Engine(target, frames=True, ring_slots=4, max_in_flight=1)
    assert torch.cuda.current_device() == before == 0
    eng.close()


def test_engine_low_rate_steps_all_complete(dev):
    """small steps at a steady low rate.  With a 300 ms idle
    limit and one 64-frame step (64 one-frame tiles) every 10 ms, a wave whose
    claim lies ~4 000 tiles ahead waits ~0.6 s for its step — past the limit
    when it was timed per wave.  Timed from the grid's last new step, the run
    never gives up while steps keep coming: every step completes, exact."""
    import time

    lib = native.load()
    buf, off, lens, _ = synth.udp_ipv4_frames(64, 256, seed=5)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    want, _ = oracle.batch_ipv4(buf, off, lens)
    steps = 100
    outs = [torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev) for _ in range(steps)]
    torch.cuda.synchronize()
    native.check(lib.sccsum_set_engine_idle_ms(300), "idle")
    try:
        eng = batch.Engine(0, frames=True, ring_slots=steps + 1, max_in_flight=4)
        stream = torch.cuda.Stream(device=dev)
        eng.start(stream)
        t0 = time.perf_counter()
        ids = []
        for k in range(steps):
            while time.perf_counter() < t0 + 0.01 * k:
                pass
            ids.append(eng.submit([(b, outs[k], None)]))
        for i in ids:
            eng.wait(i)
        eng.stop()  # raises SccsumError(EIDLE) if any wave had given up
        stream.synchronize()
    finally:
        lib.sccsum_set_engine_idle_ms(0)
    for o in outs:
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
    eng.close()


def test_engine_reads_bytes_rewritten_during_the_run(dev):
    """A shard refills its buffers while the run goes on (a NIC's DMA, a host
    copy between steps): a step must read the bytes as they are when it is
    submitted, not lines an earlier step of the same run left in an XCD's L2.
    One small batch (64 x 1500 B) is rewritten by host-to-device copies (copy
    engine, pinned memory) between steps; every step equals the oracle on the
    bytes it was given."""
    rng = np.random.default_rng(0xE9)
    contents = []
    for k in range(8):
        buf, off, lens, _ = synth.udp_ipv4_frames(64, 1500, seed=int(rng.integers(1 << 30)))
        buf = buf.copy()
        for i in range(64):  # random payloads, random checksum fields: each content verifies differently
            o = int(off[i])
            buf[o + 28:o + 1500] = rng.integers(0, 256, 1472, dtype=np.uint8)
            buf[o + 10:o + 12] = rng.integers(0, 256, 2, dtype=np.uint8)
        contents.append((buf, off, lens, oracle.batch_ipv4(buf, off, lens)))
    b = batch.PacketBatch.from_host(contents[0][0], contents[0][1], contents[0][2], device=dev)
    hosts = [torch.from_numpy(np.concatenate([c[0], np.zeros(b.data.numel() - c[0].size, np.uint8)])).pin_memory()
             for c in contents]
    outs = [torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev) for _ in contents]
    sts = [torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev) for _ in contents]
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=32, max_in_flight=2)
    stream, side = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    eng.start(stream)
    for rep in range(2):
        for k in range(len(contents)):
            with torch.cuda.stream(side):
                b.data.copy_(hosts[k], non_blocking=True)
            side.synchronize()
            eng.wait(eng.submit([(b, outs[k], sts[k])]))
    eng.stop()
    stream.synchronize()
    for (buf, off, lens, (want, want_st)), o, st in zip(contents, outs, sts):
        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)
        assert np.array_equal(st.cpu().numpy(), want_st)
    eng.close()


def test_engine_fill_limits_and_empty_batches(dev):
    """A fill takes two consecutive steps of the run, published together once
    the in-flight limit has room for both; a fill step may
    hold empty batches beside real ones; a fill on an engine created without
    SCCSUM_ENGINE_FILL, or without out2, or in a header-only mode, is refused
    (SCCSUM_EINVAL); the step a fill returns is its store step, done once
    the frames hold their values.  (The two-step form: fills are forced past
    the one-pass limit here.)"""
    from test_gpu_parity import _tx_frames

    rng = np.random.default_rng(0xEA)
    buf, off, length = _tx_frames(rng, 700)
    m = native.FILL_IP | native.FILL_L4
    want = oracle.batch_ipv4_fill(buf, off, length, m)
    lib0 = native.load()
    native.check(lib0.sccsum_set_fill_single_max(0), "two passes")  # this test is about the two-step form
    try:
        _fill_limits_two_steps(dev, rng, buf, off, length, m, want)
    finally:
        native.check(lib0.sccsum_set_fill_single_max(native.FILL_SINGLE_MAX), "default")


def _fill_limits_two_steps(dev, rng, buf, off, length, m, want):
    import ctypes

    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    empty = batch.PacketBatch(data=torch.zeros(16, dtype=torch.uint8, device=dev),
                              off=torch.zeros(0, dtype=torch.int64, device=dev),
                              length=torch.zeros(0, dtype=torch.int32, device=dev), bytes_len=0, max_len=0)
    out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    lib = native.load()
    plain = batch.Engine(0, frames=True, ring_slots=4, max_in_flight=2)
    arr = (native.Batch * 1)()
    arr[0] = native.Batch(b.data.data_ptr(), b.bytes_len, b.off.data_ptr(), b.length.data_ptr(), None,
                          out2.data_ptr(), None, b.n)
    step = ctypes.c_uint64()
    stream = torch.cuda.Stream(device=dev)
    plain.start(stream)
    assert lib.sccsum_engine_submit_fill(plain._h, ctypes.cast(arr, ctypes.c_void_p), 1, 0, m, 10**9,
                                         ctypes.byref(step)) == native.SCCSUM_EINVAL  # not a fill engine
    plain.stop()
    stream.synchronize()
    plain.close()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=2, max_in_flight=2)
    eng.start(stream)
    no_out = (native.Batch * 1)()
    no_out[0] = native.Batch(b.data.data_ptr(), b.bytes_len, b.off.data_ptr(), b.length.data_ptr(), None, None,
                             st.data_ptr(), b.n)
    assert lib.sccsum_engine_submit_fill(eng._h, ctypes.cast(no_out, ctypes.c_void_p), 1, 0, m, 10**9,
                                         ctypes.byref(step)) == native.SCCSUM_EINVAL  # no out2
    assert lib.sccsum_engine_submit_fill(eng._h, ctypes.cast(arr, ctypes.c_void_p), 1, 0,
                                         native.FILL_IP | native.FILL_L4_PSEUDO, 10**9,
                                         ctypes.byref(step)) == native.SCCSUM_EINVAL  # header-only mode
    s1 = eng.submit_fill([(empty, torch.empty(2, dtype=torch.int16, device=dev), None), (b, out2, st)], m)
    assert s1 == 1  # the store step (the generate step is step 0)
    # the same fill again (a fill is idempotent): its two steps come after the first fill's, once the
    # in-flight limit (2) has the first fill done — so it never writes the frames under the first one
    s3 = eng.submit_fill([(b, out2, st)], m)
    assert s3 == 3
    eng.wait(s1, timeout_s=0)  # done: the second fill's submit waited for it
    eng.wait(s3)
    eng.stop()
    stream.synchronize()
    got = b.data.cpu().numpy()[: b.bytes_len]
    assert np.array_equal(got, want[0])
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want[1])
    assert np.array_equal(st.cpu().numpy(), want[2])
    eng.close()


@pytest.mark.parametrize("in_flight", [2, 64])
def test_engine_fill_stress_small_steps(dev, in_flight, fill_passes):
    """Many small steps, fills and verifies interleaved, 2 or 64 in flight:
    100 fill steps of 1-3 tiny batches (1-40 of the tx generator's odd frames,
    so every store tile waits on a generate step of a few one-frame tiles)
    and 100 verify steps between them, in one run.  Every filled batch equals
    the oracle's fill, every verify the oracle (a race in the store step's
    dependency would leave fields unwritten or written from stale values)."""
    from test_gpu_parity import _tx_frames

    rng = np.random.default_rng(0xEB + in_flight)
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    fills, verifies = [], []
    for k in range(100):
        items = []
        for q in range(int(rng.integers(1, 4))):
            buf, off, length = _tx_frames(rng, int(rng.integers(1, 41)))
            b = batch.PacketBatch.from_host(buf, off, length, device=dev)
            out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
            st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
            items.append((b, out2, st, oracle.batch_ipv4_fill(buf, off, length, m)))
        fills.append(items)
        buf, off, length = _tx_frames(rng, int(rng.integers(1, 41)))
        vb = batch.PacketBatch.from_host(buf, off, length, device=dev)
        vout = torch.full((2 * vb.n,), -1, dtype=torch.int16, device=dev)
        verifies.append((vb, vout, oracle.batch_ipv4(buf, off, length)[0]))
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=512, max_in_flight=in_flight)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    last = 0
    for items, (vb, vout, _) in zip(fills, verifies):
        last = max(last, eng.submit_fill([(b, o, s) for b, o, s, _ in items], m))
        last = max(last, eng.submit([(vb, vout, None)]))
    eng.wait(last)
    eng.stop()
    stream.synchronize()
    for items in fills:
        for b, out2, st, (want_buf, want_out2, want_st) in items:
            assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want_buf)
            assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2)
            assert np.array_equal(st.cpu().numpy(), want_st)
    for vb, vout, want in verifies:
        assert np.array_equal(batch.as_u16(vout).reshape(-1, 2), want)
    eng.close()


@pytest.mark.parametrize("ring", [4, 16])
def test_engine_fill_across_empty_steps_on_a_small_ring(dev, ring, fill_passes):
    """Fills of tiny batches (their store step, in the two-pass form, waits on
    the generate step) with runs of 0-20 steps without tiles between them, on
    a 4- or 16-slot ring with the in-flight limit at the ring: a store tile's
    dependency and every wave's walk cross slots reused many times over.
    Every filled batch equals the oracle's fill, every verify the oracle."""
    from test_gpu_parity import _tx_frames

    rng = np.random.default_rng(0xE5 + ring)
    m = native.FILL_IP | native.FILL_L4
    empty = batch.PacketBatch(data=torch.zeros(16, dtype=torch.uint8, device=dev),
                              off=torch.zeros(0, dtype=torch.int64, device=dev),
                              length=torch.zeros(0, dtype=torch.int32, device=dev), bytes_len=0, max_len=0)
    empty_st = torch.empty(1, dtype=torch.uint8, device=dev)
    plan = []
    for k in range(150):
        buf, off, length = _tx_frames(rng, int(rng.integers(1, 41)))
        b = batch.PacketBatch.from_host(buf, off, length, device=dev)
        out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
        st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
        gap = int(rng.integers(0, 21)) if rng.random() < 0.6 else 0
        plan.append((gap, b, out2, st, oracle.batch_ipv4_fill(buf, off, length, m)))
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=ring, max_in_flight=ring)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    last = 0
    try:
        for gap, b, out2, st, _ in plan:
            for _ in range(gap):
                last = max(last, eng.submit([(empty, None, empty_st)]))
            last = max(last, eng.submit_fill([(b, out2, st)], m))
        eng.wait(last)
    finally:
        eng.stop()
        stream.synchronize()
    eng.close()
    for k, (_, b, out2, st, (want_buf, want_out2, want_st)) in enumerate(plan):
        assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want_buf), k
        assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want_out2), k
        assert np.array_equal(st.cpu().numpy(), want_st), k


@pytest.mark.parametrize("sync_every", [1, 3, 0])
def test_engine_barrier_period(dev, sync_every):
    """The grid's barrier (a step that waits for the one before it,
    sccsum_set_engine_sync_every; by default every 10 big steps): with a
    barrier on every step, every third step, or none, 60 steps of mixed frame
    batches and fills, 16 in flight, give the oracle's results.  Every step
    waiting on the one before is the dependency path's worst case: each wave
    parks on a step its neighbours have not finished."""
    from test_gpu_parity import _tx_frames

    lib = native.load()
    rng = np.random.default_rng(0xEC + sync_every)
    m = native.FILL_IP | native.FILL_L4
    steps = []
    for k in range(60):
        if k % 4 == 3:
            buf, off, length = _tx_frames(rng, int(rng.integers(1, 300)))
            b = batch.PacketBatch.from_host(buf, off, length, device=dev)
            out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
            steps.append(("fill", b, out2, oracle.batch_ipv4_fill(buf, off, length, m)))
        else:
            b, want, want_st = _frames_step(rng, dev, int(rng.integers(0, 3)))
            out = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
            st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
            steps.append(("frames", b, (out, st), (want, want_st)))
    torch.cuda.synchronize()
    native.check(lib.sccsum_set_engine_sync_every(sync_every), "sync_every")
    try:
        eng = batch.Engine(0, frames=True, fill=True, ring_slots=128, max_in_flight=16)
        stream = torch.cuda.Stream(device=dev)
        eng.start(stream)
        last = 0
        for kind, b, out, _ in steps:
            if kind == "fill":
                last = max(last, eng.submit_fill([(b, out, None)], m))
            else:
                last = max(last, eng.submit([(b, out[0], out[1])]))
        eng.wait(last)
        eng.stop()
        stream.synchronize()
    finally:
        lib.sccsum_set_engine_sync_every(-1)
    for kind, b, out, want in steps:
        if kind == "fill":
            assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want[0])
            assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want[1])
        else:
            assert np.array_equal(batch.as_u16(out[0]).reshape(-1, 2), want[0])
            assert np.array_equal(out[1].cpu().numpy(), want[1])
    eng.close()


def test_engine_barrier_behind_empty_steps(dev):
    """A barrier step right behind a step without tiles (all its batches
    empty) waits for the latest step that has tiles.  An empty step is done
    in host memory only, so a barrier on it held the grid until the
    dependency limit and the grid left with the barrier step's tiles unsummed
    (the 16x fuzz run's case 35).  Barriers on every second step, with every
    third step empty; each step is waited for, so a grid that gave up fails
    here as SCCSUM_EIDLE."""
    lib = native.load()
    rng = np.random.default_rng(0xEB)
    empty = batch.PacketBatch.from_host(np.zeros(1, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                                        device=dev)
    empty_st = torch.zeros(1, dtype=torch.uint8, device=dev)
    steps = []
    for k in range(30):
        if k % 3 == 1:
            steps.append(None)
            continue
        b, want, want_st = _frames_step(rng, dev, int(rng.integers(0, 3)))
        st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
        steps.append((b, st, want_st))
    torch.cuda.synchronize()
    native.check(lib.sccsum_set_engine_sync_every(2), "sync_every")
    eng = batch.Engine(0, frames=True, ring_slots=64, max_in_flight=8)
    try:
        stream = torch.cuda.Stream(device=dev)
        eng.start(stream)
        ids = [eng.submit([(empty, None, empty_st)] if x is None else [(x[0], None, x[1])]) for x in steps]
        for s in ids:
            eng.wait(s, timeout_s=5.0)
        eng.stop()
        stream.synchronize()
    finally:
        lib.sccsum_set_engine_sync_every(-1)
        eng.close()
    for k, x in enumerate(steps):
        if x is not None:
            assert np.array_equal(x[1].cpu().numpy(), x[2]), f"step {k}"



def test_engine_pacing_counts_every_older_step(dev):
    """Steps finish out of order: tiny steps behind a big one (2 M frames,
    ~0.5 ms) finish long before it.  Pacing must still hold every step up to
    max_in_flight before the newest one done when a submit returns — the
    header's "at most max_in_flight submitted and not yet done", which the
    caller relies on to free an older step's buffers, and which keeps a
    step's completion slot (step % 64) from being taken over while the step
    still counts.  A fill publishes two steps at once; pacing that waited on
    only the step max_in_flight before the newest skipped the one before
    that, here the big step."""
    from seastar_amd import devsynth
    from test_gpu_parity import _tx_frames

    lib = native.load()
    rng = np.random.default_rng(0xED)
    big = devsynth.udp_frames(2 << 20, 1500, seed=77, device=dev)
    big_st = torch.empty(big.n, dtype=torch.uint8, device=dev)
    buf, off, length = _tx_frames(rng, 40)
    m = native.FILL_IP | native.FILL_L4
    want = oracle.batch_ipv4_fill(buf, off, length, m)
    fills = []
    for k in range(12):
        b = batch.PacketBatch.from_host(buf, off, length, device=dev)
        fills.append((b, torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)))
    tiny = batch.PacketBatch.from_host(buf, off, length, device=dev)
    tiny_st = torch.empty(tiny.n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=64, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    late = []
    for rep in range(3):
        eng.start(stream)
        eng.submit([(big, None, big_st)])  # step 0
        eng.submit([(tiny, None, tiny_st)])  # step 1
        floor = 0  # every step below it was seen done
        for b, out2 in fills:
            s = eng.submit_fill([(b, out2, None)], m)  # steps s - 1 (generate) and s (store)
            while floor < s and lib.sccsum_engine_wait(eng._h, floor, 0) == native.SCCSUM_OK:
                floor += 1
            if floor < s + 1 - eng.max_in_flight:
                late.append((rep, s, floor))
        eng.wait(s)
        eng.stop()
        stream.synchronize()
    assert not late, f"(run, store step submitted, first step not done): {late[:8]}"
    for b, out2 in fills:
        assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want[0])
        assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want[1])
    eng.close()


def test_engine_slices_of_one_buffer_with_max_len(dev):
    """Steps that are slices of one large buffer (a shard's rx ring: each
    step's off/len/out arrays point into the whole ring's, bytes_len covers
    the ring): with max_len the engine sizes the tiles by max_len (32 frames
    of 1500 B), not by bytes_len / n (a slice of 1/64 of the ring looked like
    96 KB packets: tiles of a frame or two).  Every slice exact against the
    oracle, at max_len 1500 and 0 (unknown)."""
    import ctypes

    lib = native.load()
    n_all, L = 1 << 16, 1500
    buf, off, lens, _ = synth.udp_ipv4_frames(n_all, L, seed=31)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out = torch.full((2 * n_all,), -1, dtype=torch.int16, device=dev)
    st = torch.full((n_all,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=256, max_in_flight=8)
    stream = torch.cuda.Stream(device=dev)
    sizes = [1024, 4096, 16384, 1, 33]
    for max_len in (L, 0):
        eng.start(stream)
        lo, k, last = 0, 0, 0
        while lo < n_all:
            m = min(sizes[k % len(sizes)], n_all - lo)
            arr = (native.Batch * 1)()
            arr[0] = native.Batch(b.data.data_ptr(), b.bytes_len, b.off.data_ptr() + 8 * lo,
                                  b.length.data_ptr() + 4 * lo, None, out.data_ptr() + 4 * lo,
                                  st.data_ptr() + lo, m)
            step = ctypes.c_uint64()
            native.check(lib.sccsum_engine_submit(eng._h, ctypes.cast(arr, ctypes.c_void_p), 1, max_len, 10**10,
                                                  ctypes.byref(step)), "submit")
            last = step.value
            lo, k = lo + m, k + 1
        eng.wait(last)
        eng.stop()
        stream.synchronize()
        assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)
        assert np.array_equal(st.cpu().numpy(), want_st)
        out.fill_(-1)
        st.fill_(0xEE)
        torch.cuda.synchronize()
    eng.close()


@pytest.mark.parametrize("ring,in_flight,steps", [(1024, 32, 262144), (64, 64, 65536), (2, 2, 8192)])
def test_engine_unbounded_run_on_a_small_ring(dev, ring, in_flight, steps):
    """One run of many more steps than its descriptor ring has slots (VERDICT
    r05 #3: 262 144 steps of 32 frames on a 1 024-slot ring, 256 laps; a
    64-slot ring with the in-flight limit at the ring, 1 024 laps; a 2-slot
    ring, every step waiting for the one two before it).  Each step is one
    DPDK-sized burst of 32 frames (src/net/dpdk.cc:2190-2204) from a pool of
    1 024 distinct bursts, its results into its own slice of one output
    array: every step's every frame exact against the oracle.  Tiny steps put
    most waves' claims far past the published tiles, so the walk from a
    wave's cursor to its tile's step crosses slots the ring has reused."""
    import ctypes

    lib = native.load()
    B, pool = 32, 1024
    buf, off, lens, _ = synth.udp_ipv4_frames(B * pool, 600, seed=43)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out = torch.full((steps * B * 2,), -1, dtype=torch.int16, device=dev)
    st = torch.full((steps * B,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=ring, max_in_flight=in_flight)
    stream = torch.cuda.Stream(device=dev)
    arr = (native.Batch * 1)()
    step = ctypes.c_uint64()
    fn, h, ap = lib.sccsum_engine_submit, eng._h, ctypes.cast(arr, ctypes.c_void_p)
    d0, o0, l0 = b.data.data_ptr(), b.off.data_ptr(), b.length.data_ptr()
    out0, st0 = out.data_ptr(), st.data_ptr()
    eng.start(stream)
    try:
        for k in range(steps):
            q = k % pool
            arr[0] = native.Batch(d0, b.bytes_len, o0 + 8 * B * q, l0 + 4 * B * q, None, out0 + 4 * B * k,
                                  st0 + B * k, B)
            rc = fn(h, ap, 1, 600, 10**10, ctypes.byref(step))
            assert rc == native.SCCSUM_OK, (k, rc)
        assert step.value == steps - 1
        eng.wait(steps - 1)
        for k in range(max(0, steps - ring), steps):  # the last lap's done words answer too
            eng.wait(k)  # (steps finish out of order: the last one done does not make the one before it done)
    finally:
        eng.stop()
        stream.synchronize()
    eng.close()
    got = batch.as_u16(out).reshape(steps // pool, pool * B, 2)
    gst = st.cpu().numpy().reshape(steps // pool, pool * B)
    bad = np.nonzero(np.any(got != want[None], axis=(1, 2)) | np.any(gst != want_st[None], axis=1))[0]
    assert bad.size == 0, f"laps of the burst pool with a wrong frame: {bad[:8].tolist()} of {steps // pool}"


def test_engine_eight_producers(dev):
    """eight threads submit random steps into one running
    engine — frames (generate, verify-only), in-place fills and, in a second
    engine run, seeded spans — each thread waiting on some of its own steps;
    every step's results against the oracle.  (The native-thread form of the
    same is tests/cpp/shards_gpu.cc engine, test_cpp_api.py.)"""
    import threading
    from test_gpu_parity import _tx_frames

    threads, per = 8, 30
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO

    def frames_plan(t):
        rng = np.random.default_rng(0x8E0 + t)
        plan = []
        for k in range(per):
            kind = int(rng.integers(0, 3))
            if kind == 2:
                buf, off, length = _tx_frames(rng, int(rng.integers(1, 300)))
                b = batch.PacketBatch.from_host(buf, off, length, device=dev)
                out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
                st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
                plan.append(("fill", b, out2, st, oracle.batch_ipv4_fill(buf, off, length, m)))
            else:
                b, want, want_st = _frames_step(rng, dev, int(rng.integers(0, 3)))
                if kind == 0:
                    plan.append(("gen", b, torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev), None, want))
                else:
                    plan.append(("verify", b, None, torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev), want_st))
        return plan

    def spans_plan(t):
        rng = np.random.default_rng(0x8F0 + t)
        plan = []
        for k in range(per):
            n = int(rng.integers(1, 3000))
            lens = synth.zipf_lengths(n, seed=int(rng.integers(1 << 30)))
            off, total = synth.pack(lens, seed=int(rng.integers(1 << 30)), max_gap=5)
            buf = rng.integers(0, 256, total, dtype=np.uint8)
            seeds = rng.integers(0, 65536, n).astype(np.uint32)
            b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
            plan.append(("spans", b, torch.empty(n, dtype=torch.int16, device=dev),
                         torch.from_numpy(seeds.view(np.int32)).to(dev), oracle.batch_spans(buf, off, lens, seeds)))
        return plan

    def run(eng, plans):
        errors = []

        def producer(t):
            try:
                rng = np.random.default_rng(0x8A0 + t)
                for what, b, out, st, _ in plans[t]:
                    if what == "fill":
                        s = eng.submit_fill([(b, out, st)], m)
                    elif what == "spans":
                        s = eng.submit([(b, out, None, st)])
                    else:
                        s = eng.submit([(b, out, st)])
                    if rng.random() < 0.2:
                        eng.wait(s)
            except Exception as exc:  # noqa: BLE001
                errors.append((t, exc))

        stream = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        eng.start(stream)
        try:
            ts = [threading.Thread(target=producer, args=(t,)) for t in range(threads)]
            for th in ts:
                th.start()
            for th in ts:
                th.join()
        finally:
            eng.finish()
            stream.synchronize()
        eng.close()
        assert not errors, errors[:3]

    plans = [frames_plan(t) for t in range(threads)]
    run(batch.Engine(0, frames=True, fill=True, ring_slots=64, max_in_flight=16), plans)
    for t, plan in enumerate(plans):
        for k, (what, b, out, st, want) in enumerate(plan):
            msg = f"thread {t} step {k} ({what})"
            if what == "fill":
                assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want[0]), msg
                assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want[1]), msg
                assert np.array_equal(st.cpu().numpy(), want[2]), msg
            elif what == "gen":
                assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want), msg
            else:
                assert np.array_equal(st.cpu().numpy(), want), msg
    plans = [spans_plan(t) for t in range(threads)]
    run(batch.Engine(0, frames=False, ring_slots=64, max_in_flight=16), plans)
    for t, plan in enumerate(plans):
        for k, (_, b, out, _, want) in enumerate(plan):
            assert np.array_equal(batch.as_u16(out), want), f"thread {t} span step {k}"


def test_engine_stop_while_producers_submit(dev):
    """The owner stops the run while four threads are still submitting:
    every submit either returns SCCSUM_EINVAL (after the stop) or a step that
    the leaving grid completes — none is lost (include/sccsum.h, Producers).
    Every accepted step's outputs against the oracle; the next run of the same
    engine starts clean."""
    import threading
    import time

    B, per, threads = 64, 1000, 4
    buf, off, lens, _ = synth.udp_ipv4_frames(B * per * threads, 200, seed=59)
    want, _ = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out = torch.full((B * per * threads * 2,), -1, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=16, max_in_flight=8)
    stream = torch.cuda.Stream(device=dev)
    accepted = [[] for _ in range(threads)]
    errors, started = [], threading.Barrier(threads + 1)

    def producer(t):
        started.wait()
        for k in range(per):
            q = t * per + k
            sl = batch.PacketBatch(data=b.data, off=b.off[B * q:B * (q + 1)], length=b.length[B * q:B * (q + 1)],
                                   bytes_len=b.bytes_len, max_len=200)
            try:
                accepted[t].append((q, eng.submit([(sl, out[2 * B * q:2 * B * (q + 1)], None)])))
            except native.SccsumError as exc:
                if exc.code != native.SCCSUM_EINVAL:
                    errors.append((t, k, exc))
                return  # stopped: every later submit would be refused too

    eng.start(stream)
    ts = [threading.Thread(target=producer, args=(t,)) for t in range(threads)]
    for th in ts:
        th.start()
    started.wait()
    time.sleep(0.003)
    eng.stop()
    for th in ts:
        th.join()
    stream.synchronize()
    assert not errors, errors[:3]
    n_acc = sum(len(a) for a in accepted)
    assert 0 < n_acc < per * threads, n_acc  # the stop landed mid-run
    for a in accepted:
        for q, s in a:
            eng.wait(s, timeout_s=0)  # done before the grid left
    got = batch.as_u16(out).reshape(threads * per, B, 2)
    ref = want.reshape(threads * per, B, 2)
    done_q = sorted(q for a in accepted for q, _ in a)
    assert np.array_equal(got[done_q], ref[done_q])
    rest = np.setdiff1d(np.arange(threads * per), done_q)
    assert np.all(batch.as_u16(out).reshape(threads * per, B * 2)[rest] == 0xFFFF)  # refused steps never ran
    # the same engine runs again
    out.fill_(-1)
    eng.start(stream)
    sl = batch.PacketBatch(data=b.data, off=b.off[:B], length=b.length[:B], bytes_len=b.bytes_len, max_len=200)
    eng.wait(eng.submit([(sl, out[:2 * B], None)]))
    eng.finish()
    stream.synchronize()
    eng.close()
    assert np.array_equal(batch.as_u16(out[:2 * B]).reshape(B, 2), ref[0])


def test_engine_producer_limit(dev):
    """opts.producer_in_flight (a per-producer in-flight
    limit): four producer threads share a 64-step engine limit, each held to
    2 of its own steps not yet done.  When a thread's submit of its k-th step
    returns, its (k-2)-th step is done (a wait with no time left answers 0);
    every step's frames equal the oracle's."""
    import threading

    B, per, threads = 32, 300, 4
    buf, off, lens, _ = synth.udp_ipv4_frames(B * per * threads, 300, seed=53)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out = torch.full((B * per * threads * 2,), -1, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=256, max_in_flight=64, producer_in_flight=2)
    with pytest.raises(native.SccsumError):  # above the shared limit
        batch.Engine(0, frames=True, ring_slots=256, max_in_flight=8, producer_in_flight=9)
    stream = torch.cuda.Stream(device=dev)
    errors = []

    def producer(t):
        try:
            mine = []
            for k in range(per):
                q = t * per + k
                sl = batch.PacketBatch(data=b.data, off=b.off[B * q:B * (q + 1)], length=b.length[B * q:B * (q + 1)],
                                       bytes_len=b.bytes_len, max_len=300)
                mine.append(eng.submit([(sl, out[2 * B * q:2 * B * (q + 1)], None)]))
                if k >= 2:
                    eng.wait(mine[k - 2], timeout_s=0)  # SccsumError(EBUSY) if the limit let it run ahead
        except Exception as exc:  # noqa: BLE001
            errors.append((t, exc))

    eng.start(stream)
    try:
        ts = [threading.Thread(target=producer, args=(t,)) for t in range(threads)]
        for th in ts:
            th.start()
        for th in ts:
            th.join()
    finally:
        eng.finish()
        stream.synchronize()
    eng.close()
    assert not errors, errors[:3]
    assert np.array_equal(batch.as_u16(out).reshape(-1, 2), want)


@pytest.mark.parametrize("ring,in_flight", [(2, 2), (4, 4), (64, 8)])
def test_engine_walk_across_empty_steps(dev, ring, in_flight):
    """Bursts of 32 frames with runs of 0-60 empty steps between them (the
    host marks an empty step done at once, so its slot is handed on at once):
    a wave's next tile lies past many steps whose slots the ring has reused,
    often while the poller rewrites them, so the walk decides by the steps'
    seals alone.  Every burst's every frame exact against
    the oracle; the run's last steps answer their waits."""
    import ctypes

    lib = native.load()
    B, bursts = 32, 3000
    rng = np.random.default_rng(0x5EA1 + ring)
    buf, off, lens, _ = synth.udp_ipv4_frames(B * bursts, 400, seed=47)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    b = batch.PacketBatch.from_host(buf, off, lens, device=dev)
    out = torch.full((bursts * B * 2,), -1, dtype=torch.int16, device=dev)
    st = torch.full((bursts * B,), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, ring_slots=ring, max_in_flight=in_flight)
    stream = torch.cuda.Stream(device=dev)
    arr = (native.Batch * 1)()
    step = ctypes.c_uint64()
    fn, h, ap = lib.sccsum_engine_submit, eng._h, ctypes.cast(arr, ctypes.c_void_p)
    d0, o0, l0 = b.data.data_ptr(), b.off.data_ptr(), b.length.data_ptr()
    out0, st0 = out.data_ptr(), st.data_ptr()
    gaps = rng.integers(0, 61, bursts) * (rng.random(bursts) < 0.5)
    eng.start(stream)
    n_steps = 0
    try:
        for k in range(bursts):
            for _ in range(int(gaps[k])):  # empty steps: no tiles, done once the grid has copied them
                arr[0] = native.Batch(d0, 0, o0, l0, None, out0, st0, 0)
                assert fn(h, ap, 1, 400, 10**10, ctypes.byref(step)) == native.SCCSUM_OK
                n_steps += 1
            arr[0] = native.Batch(d0, b.bytes_len, o0 + 8 * B * k, l0 + 4 * B * k, None, out0 + 4 * B * k,
                                  st0 + B * k, B)
            rc = fn(h, ap, 1, 400, 10**10, ctypes.byref(step))
            assert rc == native.SCCSUM_OK, (k, rc)
            n_steps += 1
        assert step.value == n_steps - 1
        eng.wait(n_steps - 1)
        for k in range(max(0, n_steps - ring), n_steps):
            eng.wait(k)  # (steps finish out of order)
    finally:
        eng.stop()
        stream.synchronize()
    eng.close()
    got = batch.as_u16(out).reshape(bursts, B, 2)
    gst = st.cpu().numpy().reshape(bursts, B)
    bad = np.nonzero(np.any(got != want.reshape(bursts, B, 2), axis=(1, 2)) |
                     np.any(gst != want_st.reshape(bursts, B), axis=1))[0]
    assert bad.size == 0, f"bursts with a wrong frame: {bad[:8].tolist()} of {bursts} ({n_steps} steps)"


def test_engine_dependency_give_up_is_reported(dev):
    """The dependency limit is a create parameter (sccsum_engine_opts.dep_ms,
    VERDICT r05 #3).  A spans engine with a 1 ms limit and a barrier on every
    step (sccsum_set_engine_sync_every(1)): step 0 is one 48 MiB span (one
    wave sums a span past the fast path's 128 KiB exactly, tens of ms), so
    step 1's waves give up waiting for it.  wait, stop and destroy each report
    it (SCCSUM_EFAULT), step 0 itself still completes exact, and the device is
    free for the next engine."""
    lib = native.load()
    rng = np.random.default_rng(0xF0)
    L = 48 << 20
    big_buf = rng.integers(0, 256, L, dtype=np.uint8)
    big = batch.PacketBatch.from_host(big_buf, np.zeros(1, np.uint64), np.array([L], np.uint32), device=dev)
    big_want = oracle.batch_spans(big_buf, np.zeros(1, np.uint64), np.array([L], np.uint32))
    small_buf = rng.integers(0, 256, 64 * 100, dtype=np.uint8)
    small = batch.PacketBatch.from_host(small_buf, np.arange(64, dtype=np.uint64) * 100, np.full(64, 100, np.uint32),
                                        device=dev)
    o_big = torch.full((1,), -1, dtype=torch.int16, device=dev)
    o_small = torch.full((64,), -1, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    native.check(lib.sccsum_set_engine_sync_every(1), "a barrier on every step")
    stream = torch.cuda.Stream(device=dev)
    try:
        eng = batch.Engine(0, frames=False, ring_slots=8, max_in_flight=4, dep_ms=1)
        eng.start(stream)
        s0 = eng.submit([(big, o_big, None)])
        s1 = eng.submit([(small, o_small, None)])
        with pytest.raises(native.SccsumError) as e:
            eng.wait(s1)
        assert e.value.code == native.SCCSUM_EFAULT
        with pytest.raises(native.SccsumError) as e:
            eng.stop()
        assert e.value.code == native.SCCSUM_EFAULT
        stream.synchronize()
        with pytest.raises(native.SccsumError) as e:
            eng.close()
        assert e.value.code == native.SCCSUM_EFAULT
        assert s0 == 0
    finally:
        lib.sccsum_set_engine_sync_every(-1)
    assert np.array_equal(batch.as_u16(o_big), big_want)  # the step that was waited on finished
    # the device is free: a new engine runs, exact
    b, want, _ = _frames_step(rng, dev, 0)
    o = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    eng2 = batch.Engine(0, frames=True, ring_slots=4, max_in_flight=2)
    eng2.start(stream)
    eng2.wait(eng2.submit([(b, o, None)]))
    eng2.finish()
    stream.synchronize()
    eng2.close()
    assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want)


def test_engine_fill_single_pass_takes_one_step(dev):
    """A fill of at most sccsum_set_fill_single_max frames (524 288 by default)
    is ONE engine step whose tiles store the fields themselves: it returns
    that step (the one after the verify step before it), and leaves the
    frames exactly as the oracle's writers do."""
    from test_gpu_parity import _tx_frames

    rng = np.random.default_rng(0xEC)
    buf, off, length = _tx_frames(rng, 700)
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    want = oracle.batch_ipv4_fill(buf, off, length, m)
    b = batch.PacketBatch.from_host(buf, off, length, device=dev)
    out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
    st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
    vb, vwant, _ = _frames_step(rng, dev, 1)
    vout = torch.full((2 * vb.n,), -1, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=2, max_in_flight=2)
    stream = torch.cuda.Stream(device=dev)
    eng.start(stream)
    try:
        assert eng.submit([(vb, vout, None)]) == 0
        s1 = eng.submit_fill([(b, out2, st)], m)
        assert s1 == 1  # one step
        eng.wait(s1)
    finally:
        eng.stop()
        stream.synchronize()
    assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], want[0])
    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), want[1])
    assert np.array_equal(st.cpu().numpy(), want[2])
    assert np.array_equal(batch.as_u16(vout).reshape(-1, 2), vwant)
    eng.close()

