"""Seeded differential fuzzing of the batch entry points against the oracle.

Each case draws
- a random layout: packed, gapped, 64-byte aligned, scattered with overlaps, or
  packed and then shuffled (offsets out of order);
- random lengths: 0-3 bytes, short, Zipf MTUs, jumbo, and spans past the fast
  path's exact 128 KiB limit (phase D's exact redo);
- random IPv4 headers: options, other versions, total lengths that disagree
  with the frame, fragments, TCP / UDP / ICMP / other protocols, fields right
  or wrong;
- random diagnostic knobs: kernel family and form, tile packets, tile bytes,
  run alignment, short chunks, tail split, dynamic tiles, grid cap, and
  fills in one pass or two.

Then it compares every output bit with the oracle (oracle/sccsum_oracle.c).
The knobs never change results (include/sccsum_diag.h), so one oracle answer
checks every setting.  A few entries per case lie outside the byte buffer;
they must come back 0 with SCCSUM_ST_RANGE, and the oracle, which has no
range checks, is asked only about the others.  Seeds are fixed, so a failure
names its case and reproduces.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from seastar_amd import batch, native, synth

pytestmark = pytest.mark.gpu

VARIANTS = [0, 1, 2, 14, 15, 16]
# SCCSUM_FUZZ_SCALE=k runs k times as many seeded cases per test (a deeper one-off run; the
# default suite runs 1x)
SCALE = max(1, int(os.environ.get("SCCSUM_FUZZ_SCALE", "1")))


def _knobs(rng, lib, fill=False):
    """Random knobs for this thread's later launches; returns them for the failure message."""
    k = {
        "variant": 0 if fill else int(rng.choice(VARIANTS)),
        "tile_packets": int(rng.choice([64, 64, 1, 2, 7, 16, 32, 33, 63])),
        "tile_bytes": int(rng.choice([49152, 0, 2048, 262144])),
        "run_align": int(rng.choice([8, 4, 1])),
        "short_chunks": int(rng.integers(0, 2)),
        "tail": (int(rng.choice([1, 2, 4, 8])), int(rng.integers(0, 65))),
        "dynamic": int(rng.integers(0, 2)),
        "blocks_per_cu": int(rng.choice([8, 1, 2, 3])),
        "fill_single_max": int(rng.choice([native.FILL_SINGLE_MAX, 0])),  # fills in one pass, or generate + store
    }
    native.check(lib.sccsum_set_kernel_variant(k["variant"]), "variant")
    native.check(lib.sccsum_set_tile_packets(k["tile_packets"]), "tile_packets")
    native.check(lib.sccsum_set_tile_bytes(k["tile_bytes"]), "tile_bytes")
    native.check(lib.sccsum_set_run_align(k["run_align"]), "run_align")
    native.check(lib.sccsum_set_short_chunks(k["short_chunks"]), "short_chunks")
    native.check(lib.sccsum_set_tail_split(*k["tail"]), "tail_split")
    native.check(lib.sccsum_set_dynamic_tiles(k["dynamic"]), "dynamic")
    native.check(lib.sccsum_set_blocks_per_cu(k["blocks_per_cu"]), "blocks_per_cu")
    native.check(lib.sccsum_set_fill_single_max(k["fill_single_max"]), "fill_single_max")
    return k


@pytest.fixture(autouse=True)
def _default_knobs(dev):
    yield
    lib = native.load()
    lib.sccsum_set_kernel_variant(0)
    lib.sccsum_set_tile_packets(64)
    lib.sccsum_set_tile_bytes(49152)
    lib.sccsum_set_run_align(8)
    lib.sccsum_set_short_chunks(1)
    lib.sccsum_set_tail_split(1, 4)
    lib.sccsum_set_dynamic_tiles(1)
    lib.sccsum_set_blocks_per_cu(8)
    lib.sccsum_set_fill_single_max(native.FILL_SINGLE_MAX)
    lib.sccsum_set_engine_sync_every(-1)


def _engine_sync(case, lib, knobs):
    """A random barrier period for an engine case (-1 auto, 0 never, k every k-th
    step), from a generator of its own so the case's other draws stay as they were."""
    k = int(np.random.default_rng(9000 + case).choice([-1, -1, 0, 1, 2, 3, 10]))
    native.check(lib.sccsum_set_engine_sync_every(k), "sync_every")
    knobs["sync_every"] = k


def _lengths(rng, n, huge=True, lo=0):
    """A mixture: tiny, short, Zipf MTUs, jumbo, and (huge) past 128 KiB."""
    kind = rng.random(n)
    L = synth.zipf_lengths(n, int(rng.integers(1, 2**31))).astype(np.int64)
    L = np.where(kind < 0.08, rng.integers(0, 4, n), L)
    L = np.where((kind >= 0.08) & (kind < 0.25), rng.integers(4, 64, n), L)
    L = np.where((kind >= 0.85) & (kind < 0.97), rng.integers(9001, 20000, n), L)
    if huge:
        big = rng.choice([65535, 65536, 131071, 131072, 131073, 200001], n)
        L = np.where(kind >= 0.995, big, L)
    return np.maximum(L, lo).astype(np.uint32)


def _layout(rng, L, kind=None, disjoint=False):
    """Offsets for lengths L and the buffer size.  Kinds: packed, gapped,
    aligned (64 B), shuffled (packed, then offsets permuted), scattered
    (uniform positions, overlaps allowed; not with disjoint)."""
    kinds = ["packed", "gapped", "aligned", "shuffled"] + ([] if disjoint else ["scattered"])
    kind = kind or str(rng.choice(kinds))
    n = L.size
    if kind == "scattered":
        total = int(L.sum()) // 2 + int(L.max(initial=0)) + 64
        off = (rng.random(n) * (total - L.astype(np.int64) + 1)).astype(np.uint64)
        return off, total, kind
    align = 64 if kind == "aligned" else 1
    gap = 40 if kind == "gapped" else 0
    off, total = synth.pack(L, align=align, seed=int(rng.integers(1, 2**31)), max_gap=gap)
    # ("shuffled": the caller permutes offsets and lengths together, _shuffle_pairs)
    return off, int(total) + int(rng.integers(0, 48)), kind


def _shuffle_pairs(rng, off, L):
    p = rng.permutation(off.size)
    return off[p].copy(), L[p].copy()


def _range_bad(rng, off, L, total, frac=0.02):
    """Push a few entries out of [0, total): returns the mask of them."""
    n = off.size
    bad = rng.random(n) < frac
    idx = np.nonzero(bad)[0]
    for i in idx:
        if rng.random() < 0.5:
            off[i] = total + int(rng.integers(0, 5000))  # starts past the end
        else:
            off[i] = int(rng.integers(0, total + 1))
            L[i] = np.uint32(min(total - int(off[i]) + 1 + int(rng.integers(0, 3000)), 2**32 - 1))
    return bad


def _ipv4_headers(rng, buf, off, L):
    """Random IPv4 headers written into the frames' own bytes (never past a frame)."""
    n = off.size
    fw = synth.frag_words(rng, n, frac=0.15)
    for i in range(n):
        o, ln = int(off[i]), int(L[i])
        if ln == 0:
            continue
        h = rng.integers(0, 256, 40, dtype=np.uint8)
        ver = 4 if rng.random() < 0.95 else int(rng.integers(0, 16))
        ihl = 5 if rng.random() < 0.75 else int(rng.integers(0, 16))
        h[0] = (ver << 4) | ihl
        r = rng.random()
        if r < 0.75:
            tot = ln
        elif r < 0.85:
            tot = max(ln - int(rng.integers(1, 21)), 0)
        elif r < 0.95:
            tot = ln + int(rng.integers(1, 101))
        else:
            tot = int(rng.integers(0, 65536))
        h[2], h[3] = (tot >> 8) & 0xFF, tot & 0xFF
        h[6], h[7] = (int(fw[i]) >> 8) & 0xFF, int(fw[i]) & 0xFF
        h[9] = int(rng.choice([17, 17, 6, 6, 1, 47, int(rng.integers(0, 256))]))
        l4 = 4 * ihl
        if h[9] == 1 and l4 < 40 and rng.random() < 0.7:
            h[l4] = 8  # echo request
        k = min(ln, 40)
        buf[o:o + k] = h[:k]


def _make_some_valid(rng, buf, off, L, frac=0.5):
    """For disjoint in-range frames: give about `frac` of them the checksums
    the oracle's fill would write (so the verify-OK paths run too)."""
    if off.size == 0:
        return
    filled, _, _ = oracle.batch_ipv4_fill(buf, off, L, native.FILL_IP | native.FILL_L4)
    pick = np.nonzero(rng.random(off.size) < frac)[0]
    for i in pick:
        o, ln = int(off[i]), int(L[i])
        buf[o:o + min(ln, 128)] = filled[o:o + min(ln, 128)]


def _fill_diff(gbuf, wbuf, buf, off, L, k=6):
    """The first differing bytes of a fill, by frame: (frame offset, length,
    byte 0, total length, frag word, proto, byte's offset in the frame, got,
    oracle, original)."""
    diff = np.nonzero(gbuf != wbuf)[0]
    rows = []
    for d in diff[:k]:
        hit = np.nonzero((off <= d) & (d < off + L))[0]
        i = int(hit[0]) if hit.size else -1
        o = int(off[i]) if i >= 0 else -1
        h = buf[o:o + 10] if i >= 0 else np.zeros(10, np.uint8)
        rows.append((o, int(L[i]) if i >= 0 else -1, hex(int(h[0])), (int(h[2]) << 8) | int(h[3]),
                     hex((int(h[6]) << 8) | int(h[7])), int(h[9]), int(d) - o, int(gbuf[d]), int(wbuf[d]), int(buf[d])))
    return f"{diff.size} bytes differ; first (off, len, b0, totlen, frag, proto, at, got, want, orig): {rows}"


def _case_msg(case, kind, knobs, n):
    return f"case {case}: layout {kind}, n {n}, knobs {knobs}"


@pytest.mark.parametrize("case", range(16 * SCALE))
def test_fuzz_spans(dev, case):
    rng = np.random.default_rng(1000 + case)
    lib = native.load()
    n = int(rng.choice([0, 1, 63, 64, 65, 700, 3000]))
    L = _lengths(rng, n, huge=case % 4 == 0)
    off, total, kind = _layout(rng, L)
    if kind == "shuffled":
        off, L = _shuffle_pairs(rng, off, L)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    if case % 3 == 1:
        buf[: total // 3] = 0  # runs of zeros: sums that fold to 0 / 0xFFFF
    bad = _range_bad(rng, off, L, total)
    seeds = None if case % 2 else rng.integers(0, 65536, size=n).astype(np.uint32)
    knobs = _knobs(rng, lib)
    b = batch.PacketBatch.from_host(buf[:total] if total else buf[:0], off, L, device=dev)
    st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    sd = None if seeds is None else torch.from_numpy(seeds.view(np.int32)).to(dev)
    got = batch.as_u16(batch.spans(b, seeds=sd, status=st))
    torch.cuda.synchronize()
    gst = st[:n].cpu().numpy()
    msg = _case_msg(case, kind, knobs, n)
    ok = ~bad
    want = oracle.batch_spans(buf, off[ok], L[ok], None if seeds is None else seeds[ok])
    assert np.array_equal(got[ok], want), msg
    assert np.array_equal(gst[ok], (want == 0).astype(np.uint8)), msg
    assert np.all(got[bad] == 0) and np.all(gst[bad] == native.ST_RANGE), msg


@pytest.mark.parametrize("case", range(16 * SCALE))
def test_fuzz_frames(dev, case):
    rng = np.random.default_rng(2000 + case)
    lib = native.load()
    n = int(rng.choice([1, 64, 65, 500, 2500]))
    L = _lengths(rng, n, huge=case % 5 == 0)
    off, total, kind = _layout(rng, L)
    if kind == "shuffled":
        off, L = _shuffle_pairs(rng, off, L)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    _ipv4_headers(rng, buf, off, L)
    if kind != "scattered":
        _make_some_valid(rng, buf, off, L)
    bad = _range_bad(rng, off, L, total)
    knobs = _knobs(rng, lib)
    b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    got = batch.as_u16(batch.ipv4_frames(b, status=st)).reshape(n, 2)
    st2 = torch.empty(n, dtype=torch.uint8, device=dev)
    batch.verify_frames(b, st2)  # the verify-only form: status alone
    torch.cuda.synchronize()
    gst, gst2 = st.cpu().numpy(), st2.cpu().numpy()
    msg = _case_msg(case, kind, knobs, n)
    ok = ~bad
    w2, wst = oracle.batch_ipv4(buf, off[ok], L[ok])
    mism = np.nonzero(np.any(got[ok] != w2, axis=1) | (gst[ok] != wst))[0]
    assert mism.size == 0, f"{msg}: first mismatches {[(int(off[ok][i]), int(L[ok][i])) for i in mism[:6]]}"
    assert np.array_equal(gst2, gst), msg
    assert np.all(got[bad] == 0) and np.all(gst[bad] == native.ST_RANGE), msg


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_multi(dev, case):
    """1..16 batches in one launch, spans or frames, each its own layout."""
    _fuzz_multi(dev, case, np.random.default_rng(3000 + case), default_form=False)


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_multi_small_default_form(dev, case):
    """Small multi launches (at most 65 536 packets) with the default kernel
    choice: the multi-batch row kernel (one launch over every batch)."""
    _fuzz_multi(dev, case, np.random.default_rng(3500 + case), default_form=True)


def _fuzz_multi(dev, case, rng, default_form):
    lib = native.load()
    frames = case % 2 == 0
    nb = int(rng.integers(1, native.MAX_BATCHES + 1))
    items, wants = [], []
    for _ in range(nb):
        n = int(rng.choice([0, 1, 40, 300, 1200] if not default_form else [0, 1, 7, 64, 65, 300, 4000]))
        # (default form: huge frames reach the several-batch row kernel's exact redo)
        L = _lengths(rng, n, huge=case % 4 == 0)
        off, total, kind = _layout(rng, L)
        if kind == "shuffled":
            off, L = _shuffle_pairs(rng, off, L)
        buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
        if frames:
            _ipv4_headers(rng, buf, off, L)
        bad = _range_bad(rng, off, L, total)
        ok = ~bad
        if frames:
            w2, wst = oracle.batch_ipv4(buf, off[ok], L[ok])
            want = (np.zeros((n, 2), np.uint16), np.full(n, native.ST_RANGE, np.uint8))
            want[0][ok], want[1][ok] = w2, wst
        else:
            seeds = rng.integers(0, 65536, size=n).astype(np.uint32)
            w = np.zeros(n, np.uint16)
            w[ok] = oracle.batch_spans(buf, off[ok], L[ok], seeds[ok])
            want = (w, seeds, bad)
        b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
        if default_form and case % 8 == 0:
            b.max_len = min(b.max_len, 1500)  # a hint only (include/sccsum.h): understated, still exact
        st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        out = torch.empty(max((2 if frames else 1) * n, 2), dtype=torch.int16, device=dev)
        if frames:
            items.append((b, out, st))
        else:
            items.append((b, out, st, torch.from_numpy(want[1].view(np.int32)).to(dev)))
        wants.append(want)
    knobs = _knobs(rng, lib)
    if default_form:
        native.check(lib.sccsum_set_kernel_variant(0), "variant")
        knobs["variant"] = 0
    if frames:
        batch.ipv4_frames_multi(items)
    else:
        batch.spans_multi(items)
    torch.cuda.synchronize()
    for j, (it, want) in enumerate(zip(items, wants)):
        n = it[0].n
        msg = f"case {case} batch {j}/{nb}: n {n}, knobs {knobs}"
        st = it[2][:n].cpu().numpy()
        if frames:
            got = batch.as_u16(it[1][: 2 * n]).reshape(n, 2)
            assert np.array_equal(got, want[0]) and np.array_equal(st, want[1]), msg
        else:
            got = batch.as_u16(it[1][:n])
            assert np.array_equal(got, want[0]), msg
            wst = np.where(want[2], native.ST_RANGE, (want[0] == 0).astype(np.uint8))
            assert np.array_equal(st, wst), msg


FILL_MODES = [
    native.FILL_IP | native.FILL_L4,
    native.FILL_L4,
    native.FILL_IP,
    native.FILL_IP | native.FILL_L4_PSEUDO,
    native.FILL_L4_PSEUDO | native.FILL_TSO,
    native.FILL_ICMP_ECHO,
    native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO,
    native.FILL_IP | native.FILL_ICMP_ECHO,
]


@pytest.mark.parametrize("case", range(16 * SCALE))
def test_fuzz_fill(dev, case):
    """In-place generate over disjoint frames (any order): the whole buffer,
    the values and the status must be the oracle's."""
    rng = np.random.default_rng(4000 + case)
    lib = native.load()
    n = int(rng.choice([1, 64, 65, 400, 2000]))
    L = _lengths(rng, n, huge=case % 8 == 0)
    off, total, kind = _layout(rng, L, disjoint=True)
    if kind == "shuffled":
        off, L = _shuffle_pairs(rng, off, L)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    _ipv4_headers(rng, buf, off, L)
    bad = _range_bad(rng, off, L, total, frac=0.01)
    mode = FILL_MODES[case % len(FILL_MODES)]
    knobs = _knobs(rng, lib, fill=True)
    b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
    if case % 8 == 0:
        # max_len is a hint (include/sccsum.h): understated below frames over 128 KiB, a small
        # fill still takes the row kernel, whose exact redo must read those headers from the
        # frames themselves
        b.max_len = int(rng.choice([64, 1500, 9000, 131072]))
        knobs["max_len"] = b.max_len
    out2 = torch.empty(2 * n, dtype=torch.int16, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    batch.ipv4_fill(b, mode, out2=out2, status=st)
    torch.cuda.synchronize()
    msg = _case_msg(case, kind, knobs, n) + f", mode {mode:#x}"
    ok = ~bad
    wbuf, w2, wst = oracle.batch_ipv4_fill(buf, off[ok], L[ok], mode)
    gbuf = b.data[:total].cpu().numpy()
    assert np.array_equal(gbuf, wbuf[:total]), f"{msg}: {_fill_diff(gbuf, wbuf[:total], buf, off, L)}"
    gst = st.cpu().numpy()
    assert np.array_equal(gst[ok], wst), msg
    got2 = batch.as_u16(out2).reshape(n, 2)
    assert np.array_equal(got2[ok], w2), msg  # the values stored, 0 where nothing was (include/sccsum.h)
    assert np.all(gst[bad] == native.ST_RANGE), msg


@pytest.mark.parametrize("case", range(4 * SCALE))
def test_fuzz_engine_steps(dev, case):
    """One engine run: random steps of 1..4 frame batches, and (fill engine)
    in-place fills between them, every step's results the oracle's."""
    rng = np.random.default_rng(5000 + case)
    lib = native.load()
    fill = case % 2 == 1
    knobs = _knobs(rng, lib, fill=True)
    _engine_sync(case, lib, knobs)
    # every step's batches are built before the run: while the grid runs, a
    # device-wide synchronize (or any kernel) would wait for its stop
    plan = []
    for _ in range(int(rng.integers(10, 40))):
        if fill and rng.random() < 0.3:
            n = int(rng.choice([1, 64, 700]))
            L = _lengths(rng, n, huge=False, lo=20)
            off, total, kind = _layout(rng, L, disjoint=True)
            buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
            _ipv4_headers(rng, buf, off, L)
            b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
            out2 = torch.empty(2 * n, dtype=torch.int16, device=dev)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            mode = int(rng.choice([native.FILL_IP | native.FILL_L4, native.FILL_L4,
                                   native.FILL_IP | native.FILL_ICMP_ECHO]))
            plan.append(("fill", (b, out2, st, buf, off, L, total, mode)))
            continue
        items, wants = [], []
        for _ in range(int(rng.integers(1, native.ENGINE_MAX_BATCHES + 1))):
            n = int(rng.choice([0, 1, 64, 65, 500, 3000]))
            L = _lengths(rng, n, huge=False)
            off, total, kind = _layout(rng, L)
            if kind == "shuffled":
                off, L = _shuffle_pairs(rng, off, L)
            buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
            _ipv4_headers(rng, buf, off, L)
            b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
            # a third of the batches verify only (status, no out2: what cfg 3 and the rx half submit)
            out2 = torch.full((max(2 * n, 2),), -1, dtype=torch.int16, device=dev) if rng.random() < 0.67 else None
            st = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)  # 0xEE: never written
            items.append((b, out2, st))
            wants.append(oracle.batch_ipv4(buf, off, L))
        plan.append(("sum", (items, wants)))
    # a random descriptor ring, often far smaller than the run (slots reused many times, round 6)
    ring = int(np.random.default_rng(7000 + case).choice([2, 4, 8, 256]))
    knobs["ring"] = ring
    eng = batch.Engine(0, frames=True, ring_slots=ring, max_in_flight=int(rng.choice([2, 8, 64])), fill=fill)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    checks = []
    eng.start(stream)
    try:
        for what, data in plan:
            if what == "fill":
                b, out2, st = data[:3]
                checks.append((what, eng.submit_fill([(b, out2, st)], data[7]), data))
            else:
                checks.append((what, eng.submit(data[0]), data))
        for c in checks:
            eng.wait(c[1])  # a grid that gave up (idle, a dependency) reports it here
    finally:
        eng.stop()
        stream.synchronize()
        eng.close()
    for what, step, data in checks:
        msg = f"case {case} step {step} ({what}), knobs {knobs}"
        if what == "sum":
            for j, (it, (w2, wst)) in enumerate(zip(*data)):
                n = it[0].n
                gst = it[2][:n].cpu().numpy()
                diag = (f"{msg} batch {j}/{len(data[0])}: n {n}, out2 {'yes' if it[1] is not None else 'no'}, "
                        f"{int((gst == 0xEE).sum())} status bytes never written, {int((gst != wst).sum())} differ, "
                        f"first differing {np.nonzero(gst != wst)[0][:6].tolist()}")
                if it[1] is not None:
                    got = batch.as_u16(it[1][: 2 * n]).reshape(n, 2)
                    assert np.array_equal(got, w2), diag
                assert np.array_equal(gst, wst), diag
        else:
            b, out2, st, buf, off, L, total, mode = data
            wbuf, w2, wst = oracle.batch_ipv4_fill(buf, off, L, mode)
            gbuf = b.data[:total].cpu().numpy()
            assert np.array_equal(gbuf, wbuf[:total]), f"{msg}: {_fill_diff(gbuf, wbuf[:total], buf, off, L)}"
            assert np.array_equal(st.cpu().numpy(), wst), msg


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_fragments(dev, case):
    """Packets as random fragment lists (odd lengths carry the byte order
    across fragments, empty fragments, fragments anywhere in the buffer)."""
    rng = np.random.default_rng(6000 + case)
    lib = native.load()
    n = int(rng.choice([1, 64, 500, 1500]))
    counts = rng.integers(0, 9, n)
    counts[rng.random(n) < 0.1] = 1
    nf = int(counts.sum())
    flen = np.where(rng.random(nf) < 0.3, rng.integers(0, 8, nf), rng.integers(0, 4097, nf)).astype(np.uint32)
    foff, total, kind = _layout(rng, flen)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    first = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    seeds = rng.integers(0, 65536, n).astype(np.uint32)
    knobs = _knobs(rng, lib)
    d = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    got = batch.fragments(d, total, torch.from_numpy(foff.view(np.int64)).to(dev),
                          torch.from_numpy(flen.view(np.int32)).to(dev), torch.from_numpy(first.view(np.int32)).to(dev),
                          seeds=torch.from_numpy(seeds.view(np.int32)).to(dev), status=st,
                          max_frag_len=int(flen.max(initial=0)))
    torch.cuda.synchronize()
    want = oracle.batch_fragments(buf, foff, flen, first, seeds)
    msg = _case_msg(case, kind, knobs, n)
    assert np.array_equal(batch.as_u16(got), want), msg
    assert np.array_equal(st.cpu().numpy(), (want == 0).astype(np.uint8)), msg


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_rss(dev, case):
    """Toeplitz RSS alone and fused into the frames pass, random keys of 4-52
    bytes, both hash modes, on the random frames above; the fused pass must
    leave the checksums and status exactly as sccsum_ipv4_frames gives them."""
    rng = np.random.default_rng(7000 + case)
    lib = native.load()
    n = int(rng.choice([1, 64, 65, 700, 2500]))
    L = _lengths(rng, n, huge=False)
    off, total, kind = _layout(rng, L)
    if kind == "shuffled":
        off, L = _shuffle_pairs(rng, off, L)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    _ipv4_headers(rng, buf, off, L)
    bad = _range_bad(rng, off, L, total)
    ok = ~bad
    key = bytes(rng.integers(0, 256, int(rng.choice([4, 5, 13, 16, 40, 52])), dtype=np.uint8))
    mode = int(case % 2)
    knobs = _knobs(rng, lib)
    b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    h = batch.ipv4_rss(b, key=key, mode=mode, status=st)
    fst = torch.empty(n, dtype=torch.uint8, device=dev)
    out2, fh = batch.ipv4_frames_rss(b, key=key, mode=mode, status=fst)
    torch.cuda.synchronize()
    msg = _case_msg(case, kind, knobs, n) + f", key {len(key)} B, mode {mode}"
    want_h, want_st = oracle.batch_ipv4_rss(buf, off[ok], L[ok], key=key, mode=mode)
    gh = h.cpu().numpy().view(np.uint32)
    assert np.array_equal(gh[ok], want_h), msg
    assert np.array_equal(st.cpu().numpy()[ok] & 4, want_st & 4), msg
    assert np.array_equal(fh.cpu().numpy().view(np.uint32)[ok], want_h), msg
    w2, wst = oracle.batch_ipv4(buf, off[ok], L[ok])
    assert np.array_equal(batch.as_u16(out2).reshape(n, 2)[ok], w2), msg
    assert np.array_equal(fst.cpu().numpy()[ok], wst), msg
    assert np.all(fst.cpu().numpy()[bad] == native.ST_RANGE), msg


@pytest.mark.parametrize("case", range(6 * SCALE))
def test_fuzz_desc(dev, case):
    """Frames and spans as fragment descriptors in device memory or the
    stage buffer, cut at random points (inside headers too), fragments in a
    shuffled pool: the same bits as the frames / spans the cuts came from."""
    from test_gpu_desc import _scatter

    rng = np.random.default_rng(8000 + case)
    n = int(rng.choice([1, 300, 1500, 3000]))
    frames = case % 2 == 0
    L = _lengths(rng, n, huge=False, lo=0)
    off, total = synth.pack(L, seed=int(rng.integers(1, 2**31)), max_gap=7)
    buf = rng.integers(0, 256, size=max(int(total), 1), dtype=np.uint8)
    if frames:
        _ipv4_headers(rng, buf, off, L)
    pool_len = int(L.sum()) + 40 * 6 * n + 64
    pool_t = torch.empty(pool_len, dtype=torch.uint8, device=dev)
    desc, first, lay_off, pool, stage = _scatter(rng, buf, off, L, pool_t.data_ptr(), pool_len,
                                                 stage_frac=0.3 if case % 3 == 0 else 0.0)
    pool_t.copy_(torch.from_numpy(pool))
    # no descriptors at all when every packet is empty: the C-ABI then takes a NULL array
    dd = torch.from_numpy(desc.view(np.uint8)).to(dev) if desc.size else None
    df = torch.from_numpy(first).to(dev)
    doff = torch.from_numpy(lay_off.view(np.int64)).to(dev)
    dlen = torch.from_numpy(L.view(np.int32)).to(dev)
    dstage = torch.from_numpy(stage).to(dev)
    st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    ml = int(L.max(initial=0))
    if frames:
        out2 = batch.ipv4_frames_desc(dd, df, doff, dlen, ml, stage=dstage, status=st)
        torch.cuda.synchronize()
        w2, wst = oracle.batch_ipv4(buf, off, L)
        assert np.array_equal(batch.as_u16(out2).reshape(n, 2), w2), f"case {case}"
        assert np.array_equal(st[:n].cpu().numpy(), wst), f"case {case}"
    else:
        seeds = rng.integers(0, 65536, n).astype(np.uint32)
        out = batch.spans_desc(dd, df, doff, dlen, ml, seeds=torch.from_numpy(seeds.view(np.int32)).to(dev),
                               stage=dstage, status=st)
        torch.cuda.synchronize()
        want = oracle.batch_spans(buf, off, L, seeds)
        assert np.array_equal(batch.as_u16(out), want), f"case {case}"
        assert np.array_equal(st[:n].cpu().numpy(), (want == 0).astype(np.uint8)), f"case {case}"


@pytest.mark.parametrize("case", range(6 * SCALE))
def test_fuzz_burst(dev, case):
    """The burst queue with random batch limits, depth and delay, spans or
    frames, copied or zero-copy fragments, every fused form: results in
    submit order, each the oracle's."""
    from seastar_amd import pipeline
    from seastar_amd.burst import BurstQueue
    from test_gpu_burst import _split

    rng = np.random.default_rng(9000 + case)
    lib = native.load()
    frames = case % 2 == 0
    n = int(rng.choice([1, 200, 1500]))
    L = np.minimum(_lengths(rng, n, huge=False), 30000).astype(np.uint32)
    off, total = synth.pack(L, seed=int(rng.integers(1, 2**31)), max_gap=5)
    host = rng.integers(0, 256, size=max(int(total), 1), dtype=np.uint8)
    if frames:
        _ipv4_headers(rng, host, off, L)
    pinned = pipeline.pinned_empty(host.size)
    pinned[:] = host
    seeds = None if frames else rng.integers(0, 65536, n).astype(np.uint32)
    fused = int(rng.integers(0, 3))
    native.check(lib.sccsum_set_burst_fused(fused), "burst_fused")
    q = BurstQueue(native.PIPE_IPV4 if frames else native.PIPE_SPANS,
                   batch_bytes=int(rng.choice([64 << 10, 256 << 10, 4 << 20])) + int(L.max(initial=0)),
                   batch_packets=int(rng.choice([1, 7, 32, 128, 1024])),
                   max_delay_ns=int(rng.choice([0, 50_000, 10**12])), depth=int(rng.choice([1, 2, 4, 8])))
    mapped_frac = float(rng.choice([0.0, 0.5, 1.0]))
    try:
        tickets = []
        for i in range(n):
            mapped = bool(rng.random() < mapped_frac)
            src = pinned if mapped else host
            pkt = src[int(off[i]):int(off[i]) + int(L[i])]
            while (t := q.submit(_split(rng, pkt), 0 if seeds is None else int(seeds[i]), mapped=mapped)) is None:
                q.poll()
            tickets.append(t)
            if rng.random() < 0.1:
                q.poll()
        q.drain()
    finally:
        lib.sccsum_set_burst_fused(2)
    msg = f"case {case}: n {n}, fused {fused}, mapped {mapped_frac}"
    assert tickets == list(range(n)), msg
    if frames:
        w2, wst = oracle.batch_ipv4(host, off, L)
        got = np.stack([q.results[t] for t in tickets]) if n else np.zeros((0, 2), np.uint16)
        st = np.array([q.status[t] for t in tickets], np.uint8)
        assert np.array_equal(got, w2) and np.array_equal(st, wst), msg
    else:
        want = oracle.batch_spans(host, off, L, seeds)
        got = np.array([int(q.results[t]) for t in tickets], np.uint16)
        assert np.array_equal(got, want), msg
    q.close()


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_fuzz_host_pipeline(dev, case):
    """Host batches through the pipeline with random chunk limits and depth,
    every gather form, spans or frames, packed or slot-shaped layouts."""
    from seastar_amd import pipeline

    rng = np.random.default_rng(9500 + case)
    lib = native.load()
    frames = case % 2 == 0
    gather = case % 4
    n = int(rng.choice([1, 300, 2500]))
    if rng.random() < 0.5:  # mbuf-slot-shaped: one pitch, odd start, packets up to the pitch
        pitch = int(rng.choice([640, 2304]))
        L = rng.integers(0, pitch + 1, n).astype(np.uint32)
        off = np.arange(n, dtype=np.uint64) * pitch + int(rng.integers(0, 300))
        total = int(off[-1]) + pitch + 64
    else:
        L = np.minimum(_lengths(rng, n, huge=False), 20000).astype(np.uint32)
        off, total = synth.pack(L, seed=int(rng.integers(1, 2**31)), max_gap=9)
        total = int(total) + 16
    host = rng.integers(0, 256, size=total, dtype=np.uint8)
    if frames:
        _ipv4_headers(rng, host, off, L)
    buf = pipeline.pinned_empty(total)
    buf[:] = host
    knobs = _knobs(rng, lib)
    ml = int(L.max(initial=0))
    pl = pipeline.HostPipeline(0, chunk_bytes=int(rng.choice([2 * ml + 4096, 1 << 20, 64 << 20])),
                               chunk_packets=int(rng.choice([1, 64, 300, 1 << 16])), depth=int(rng.choice([1, 2, 3, 5])))
    try:
        msg = f"case {case}: n {n}, gather {gather}, knobs {knobs}"
        if frames:
            got, st = pl.run(native.PIPE_IPV4, buf, off, L, status=True, gather=gather, max_len=ml)
            w2, wst = oracle.batch_ipv4(host, off, L)
            assert np.array_equal(got, w2) and np.array_equal(st, wst), msg
        else:
            seeds = rng.integers(0, 65536, n).astype(np.uint32)
            got, st = pl.run(native.PIPE_SPANS, buf, off, L, seeds=seeds, status=True, gather=gather, max_len=ml)
            want = oracle.batch_spans(host, off, L, seeds)
            assert np.array_equal(got, want), msg
            assert np.array_equal(st, (want == 0).astype(np.uint8)), msg
    finally:
        pl.close()


@pytest.mark.parametrize("case", range(3 * SCALE))
def test_fuzz_engine_spans(dev, case):
    """A spans engine (SCCSUM_PIPE_SPANS): random steps of 1..4 seeded span
    batches, out-of-range entries included, every result the oracle's."""
    rng = np.random.default_rng(9900 + case)
    lib = native.load()
    knobs = _knobs(rng, lib, fill=True)
    _engine_sync(case + 500, lib, knobs)
    plan = []
    for _ in range(int(rng.integers(5, 30))):
        items, wants = [], []
        for _ in range(int(rng.integers(1, native.ENGINE_MAX_BATCHES + 1))):
            n = int(rng.choice([0, 1, 64, 65, 500, 3000]))
            L = _lengths(rng, n, huge=case == 0)
            off, total, kind = _layout(rng, L)
            if kind == "shuffled":
                off, L = _shuffle_pairs(rng, off, L)
            buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
            bad = _range_bad(rng, off, L, total)
            seeds = rng.integers(0, 65536, size=n).astype(np.uint32)
            w = np.zeros(n, np.uint16)
            w[~bad] = oracle.batch_spans(buf, off[~bad], L[~bad], seeds[~bad])
            b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
            out = torch.empty(max(n, 1), dtype=torch.int16, device=dev)
            st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            items.append((b, out, st, torch.from_numpy(seeds.view(np.int32)).to(dev)))
            wants.append((w, np.where(bad, native.ST_RANGE, (w == 0).astype(np.uint8))))
        plan.append((items, wants))
    ring = int(np.random.default_rng(7500 + case).choice([2, 4, 64]))
    knobs["ring"] = ring
    eng = batch.Engine(0, frames=False, ring_slots=ring, max_in_flight=int(rng.choice([2, 8, 64])))
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    eng.start(stream)
    try:
        steps = [eng.submit(items) for items, _ in plan]
        for s in steps:
            eng.wait(s)
    finally:
        eng.stop()
        stream.synchronize()
        eng.close()
    for step, (items, wants) in zip(steps, plan):
        for j, (it, (w, wst)) in enumerate(zip(items, wants)):
            n = it[0].n
            msg = f"case {case} step {step} batch {j}: n {n}, knobs {knobs}"
            assert np.array_equal(batch.as_u16(it[1][:n]), w), msg
            assert np.array_equal(it[2][:n].cpu().numpy(), wst), msg


@pytest.mark.parametrize("case", range(2 * SCALE))
def test_fuzz_engine_producers(dev, case):
    """Several producer threads into one fill engine at once, each a random
    mix of frame steps (generate, verify-only), in-place fills and runs of
    steps without tiles, on a random small ring with a random shared and
    per-producer in-flight limit: every step's results the oracle's."""
    import threading
    from test_gpu_parity import _tx_frames

    rng = np.random.default_rng(8800 + case)
    threads = int(rng.choice([2, 4, 8]))
    ring = int(rng.choice([2, 4, 16, 64]))
    mif = int(rng.choice([2, 8, 64]))
    plim = int(rng.choice([0, 1, 2])) if mif >= 2 else 0
    m = native.FILL_IP | native.FILL_L4 | native.FILL_ICMP_ECHO
    empty = batch.PacketBatch(data=torch.zeros(16, dtype=torch.uint8, device=dev),
                              off=torch.zeros(0, dtype=torch.int64, device=dev),
                              length=torch.zeros(0, dtype=torch.int32, device=dev), bytes_len=0, max_len=0)
    empty_st = torch.empty(1, dtype=torch.uint8, device=dev)
    plans = []
    for t in range(threads):
        trng = np.random.default_rng(8900 + 16 * case + t)
        plan = []
        for _ in range(int(trng.integers(5, 25))):
            r = trng.random()
            if r < 0.2:
                plan.append(("empty", int(trng.integers(1, 12))))
            elif r < 0.45:
                buf, off, length = _tx_frames(trng, int(trng.integers(1, 200)))
                b = batch.PacketBatch.from_host(buf, off, length, device=dev)
                out2 = torch.full((2 * b.n,), -1, dtype=torch.int16, device=dev)
                st = torch.full((b.n,), 0xEE, dtype=torch.uint8, device=dev)
                plan.append(("fill", b, out2, st, oracle.batch_ipv4_fill(buf, off, length, m)))
            else:
                n = int(trng.choice([1, 64, 700]))
                L = _lengths(trng, n, huge=False)
                off, total, _ = _layout(trng, L)
                buf = trng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
                _ipv4_headers(trng, buf, off, L)
                b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
                out2 = torch.full((2 * n,), -1, dtype=torch.int16, device=dev) if trng.random() < 0.6 else None
                st = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
                plan.append(("sum", b, out2, st, oracle.batch_ipv4(buf, off, L)))
        plans.append(plan)
    eng = batch.Engine(0, frames=True, fill=True, ring_slots=ring, max_in_flight=max(mif, 2),
                       producer_in_flight=min(plim, max(mif, 2)))
    errors = []

    def producer(t):
        try:
            for item in plans[t]:
                if item[0] == "empty":
                    for _ in range(item[1]):
                        eng.submit([(empty, None, empty_st)])
                elif item[0] == "fill":
                    eng.submit_fill([(item[1], item[2], item[3])], m)
                else:
                    eng.submit([(item[1], item[2], item[3])])
        except Exception as exc:  # noqa: BLE001
            errors.append((t, exc))

    stream = torch.cuda.Stream()
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
    knobs = f"threads {threads} ring {ring} in_flight {mif} per-producer {plim}"
    assert not errors, (knobs, errors[:3])
    for t, plan in enumerate(plans):
        for k, item in enumerate(plan):
            msg = f"case {case} thread {t} item {k} ({item[0]}), {knobs}"
            if item[0] == "fill":
                _, b, out2, st, (wbuf, wout2, wst) = item
                assert np.array_equal(b.data.cpu().numpy()[: b.bytes_len], wbuf), msg
                assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), wout2), msg
                assert np.array_equal(st.cpu().numpy(), wst), msg
            elif item[0] == "sum":
                _, b, out2, st, (w2, wst) = item
                if out2 is not None:
                    assert np.array_equal(batch.as_u16(out2).reshape(-1, 2), w2), msg
                assert np.array_equal(st.cpu().numpy(), wst), msg


@pytest.mark.parametrize("case", range(4 * SCALE))
def test_fuzz_large_batches(dev, case):
    """100 k-300 k packets under random knobs: long claim chains per wave,
    the tail split over many tiles, grids capped at 1-3 blocks per CU."""
    rng = np.random.default_rng(9700 + case)
    lib = native.load()
    frames = case % 2 == 1
    n = int(rng.integers(100_000, 300_001))
    L = np.minimum(_lengths(rng, n, huge=False), 4000).astype(np.uint32)
    off, total, kind = _layout(rng, L)
    if kind == "shuffled":
        off, L = _shuffle_pairs(rng, off, L)
    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    if frames:
        _ipv4_headers(rng, buf, off, L)
    bad = _range_bad(rng, off, L, total, frac=0.001)
    ok = ~bad
    knobs = _knobs(rng, lib)
    b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    msg = _case_msg(case, kind, knobs, n)
    if frames:
        got = batch.as_u16(batch.ipv4_frames(b, status=st)).reshape(n, 2)
        torch.cuda.synchronize()
        w2, wst = oracle.batch_ipv4(buf, off[ok], L[ok], nthreads=8)
        gst = st.cpu().numpy()
        assert np.array_equal(got[ok], w2) and np.array_equal(gst[ok], wst), msg
    else:
        seeds = rng.integers(0, 65536, size=n).astype(np.uint32)
        got = batch.as_u16(batch.spans(b, seeds=torch.from_numpy(seeds.view(np.int32)).to(dev), status=st))
        torch.cuda.synchronize()
        want = oracle.batch_spans(buf, off[ok], L[ok], seeds[ok], nthreads=8)
        gst = st.cpu().numpy()
        assert np.array_equal(got[ok], want), msg
        assert np.array_equal(gst[ok], (want == 0).astype(np.uint8)), msg
    assert np.all(gst[bad] == native.ST_RANGE), msg


def test_fuzz_shard_threads(dev):
    """Seastar's model from Python: six shard threads on one GPU, each with its
    own sccsum_init, stream, random knobs (thread-local) and random launches
    (spans, frames, multi, fills, fragment lists) in flight together; every
    result checked against the oracle once the thread's stream is done."""
    import threading

    errors = []

    def shard(t):
        try:
            rng = np.random.default_rng(9800 + t)
            lib = native.load()
            native.check(lib.sccsum_init(0), "sccsum_init")
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            knobs = _knobs(rng, lib)
            checks = []
            with torch.cuda.stream(s):
                for it in range(12):
                    op = str(rng.choice(["spans", "frames", "multi", "fill", "frags"]))
                    n = int(rng.choice([1, 64, 400, 1500]))
                    L = _lengths(rng, n, huge=False, lo=20 if op == "fill" else 0)
                    off, total, kind = _layout(rng, L, disjoint=op == "fill")
                    if kind == "shuffled":
                        off, L = _shuffle_pairs(rng, off, L)
                    buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
                    if op in ("frames", "multi", "fill"):
                        _ipv4_headers(rng, buf, off, L)
                    b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
                    if op == "spans":
                        out = batch.spans(b, stream=s)
                        checks.append((op, out, oracle.batch_spans(buf, off, L)))
                    elif op == "frames":
                        st = torch.empty(n, dtype=torch.uint8, device=dev)
                        out = batch.ipv4_frames(b, status=st, stream=s)
                        checks.append((op, (out, st), oracle.batch_ipv4(buf, off, L)))
                    elif op == "multi":
                        st = torch.empty(n, dtype=torch.uint8, device=dev)
                        outs = batch.ipv4_frames_multi([(b, None, st), (b, None, None)], stream=s)
                        checks.append((op, (outs, st), oracle.batch_ipv4(buf, off, L)))
                    elif op == "fill":
                        mode = native.FILL_IP | native.FILL_L4
                        out2 = torch.empty(2 * n, dtype=torch.int16, device=dev)
                        batch.ipv4_fill(b, mode, out2=out2, stream=s)
                        checks.append((op, (b, total), oracle.batch_ipv4_fill(buf, off, L, mode)[0][:total]))
                    else:
                        first = np.arange(n + 1, dtype=np.uint32)  # one fragment per packet
                        got = batch.fragments(b.data, total, b.off, b.length,
                                              torch.from_numpy(first.view(np.int32)).to(dev), stream=s)
                        checks.append((op, got, oracle.batch_spans(buf, off, L)))
            s.synchronize()
            for k, (op, got, want) in enumerate(checks):
                msg = f"thread {t} launch {k} ({op}), knobs {knobs}"
                if op in ("spans", "frags"):
                    assert np.array_equal(batch.as_u16(got), want), msg
                elif op == "frames":
                    n = got[1].numel()
                    assert np.array_equal(batch.as_u16(got[0]).reshape(n, 2), want[0]), msg
                    assert np.array_equal(got[1].cpu().numpy(), want[1]), msg
                elif op == "multi":
                    outs, st = got
                    for o in outs:
                        assert np.array_equal(batch.as_u16(o).reshape(-1, 2), want[0]), msg
                    assert np.array_equal(st.cpu().numpy(), want[1]), msg
                else:
                    b, total = got
                    assert np.array_equal(b.data[:total].cpu().numpy(), want), msg
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append(f"thread {t}: {e!r}")

    threads = [threading.Thread(target=shard, args=(t,)) for t in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a shard thread hung"
    assert not errors, errors
