"""Synthetic frames are built byte-for-byte like the reference's tx path
(ip.cc:249-269, udp.cc:178-182, tcp_hdr::write) and verify after their
checksums are stored."""
import numpy as np

import oracle
from seastar_amd import synth


def test_udp_frames_layout_and_roundtrip():
    buf, off, lens, meta = synth.udp_ipv4_frames(50, 1500, seed=3)
    f = buf.reshape(50, 1500)
    assert np.all(f[:, 0] == 0x45) and np.all(f[:, 8] == 64) and np.all(f[:, 9] == 17)
    assert np.all((f[:, 2].astype(int) << 8 | f[:, 3]) == 1500)
    assert np.all((f[:, 24].astype(int) << 8 | f[:, 25]) == 1480)
    src = (f[:, 12].astype(np.uint64) << 24) | (f[:, 13].astype(np.uint64) << 16) | \
          (f[:, 14].astype(np.uint64) << 8) | f[:, 15]
    assert np.array_equal(src, meta["src"])
    out, st = oracle.batch_ipv4(buf, off, lens)
    assert np.all(st == 0)  # zero fields -> not verifying, not malformed
    rx = buf.copy()
    synth.store_ipv4_checksums(rx, off, out)
    out2, st2 = oracle.batch_ipv4(rx, off, lens)
    assert np.all(out2 == 0) and np.all(st2 == 3)


def test_tcp_segments_pseudo_seed_verify():
    buf, off, lens, meta = synth.tcp_segments(20, 1000, seed=2, options_len=12)
    seg = buf.reshape(20, 1000)
    assert np.all(seg[:, 12] == ((20 + 12) // 4) << 4)
    seeds = np.array([oracle.pseudo_seed(int(s), int(d), 6, 1000) for s, d in zip(meta["src"], meta["dst"])],
                     np.uint32)
    c = oracle.batch_spans(buf, off, lens, seeds)
    for i in range(20):  # tcp_hdr::write_nbo_checksum copies the 2 bytes verbatim
        seg[i, 16:18] = np.frombuffer(np.uint16(c[i]).tobytes(), np.uint8)
    assert np.all(oracle.batch_spans(buf, off, lens, seeds) == 0)


def test_mixed_frames_and_packing():
    lens = synth.zipf_lengths(2000, seed=4)
    assert lens.min() >= 64 and lens.max() <= 9000
    off, total = synth.pack(lens, align=64)
    assert np.all(off % 64 == 0) and total >= int(lens.sum())
    buf, off, lens, _ = synth.mixed_udp_frames(300, seed=8, max_gap=5)
    assert np.any(off % 2 == 1)
    out, st = oracle.batch_ipv4(buf, off, lens)
    assert np.all((st & 4) == 0)


def test_ipv4_fragment_cuts_like_ipv4_send():
    """synth.ipv4_fragment follows ipv4::send (ip.cc:244-299): pieces of
    mtu - 20 bytes, MF on all but the last, offsets in 8-byte units, one
    header per piece; a datagram that fits goes out whole with frag = 0."""
    import numpy as np

    from seastar_amd import synth

    rng = np.random.default_rng(3)
    for size in (8, 1480, 1481, 2960, 9000, 65515):
        l4 = rng.integers(0, 256, size, dtype=np.uint8)
        frames = synth.ipv4_fragment(l4, 17, 0x0A000001, 0x0A000002, mtu=1500, ident=77)
        assert len(frames) == max(1, -(-size // 1480))
        at = 0
        for k, f in enumerate(frames):
            ip_len = (int(f[2]) << 8) | int(f[3])
            fw = (int(f[6]) << 8) | int(f[7])
            assert ip_len == f.size and f[0] == 0x45 and f[9] == 17 and (int(f[4]) << 8 | int(f[5])) == 77
            if len(frames) == 1:
                assert fw == 0
            else:
                assert (fw & 0x1FFF) * 8 == at and bool(fw & 0x2000) == (k + 1 < len(frames))
            assert np.array_equal(f[20:], l4[at:at + f.size - 20])
            at += f.size - 20
        assert at == size


def test_frag_words_mix():
    import numpy as np

    from seastar_amd import synth

    w = synth.frag_words(np.random.default_rng(5), 20000)
    frag = (w & 0x3FFF) != 0
    assert 0.2 < frag.mean() < 0.4
    mf, off = (w & 0x2000) != 0, (w & 0x1FFF) != 0
    assert np.any(mf & ~off)  # first fragments
    assert np.any(mf & off)   # middle fragments
    assert np.any(~mf & off)  # last fragments
    assert np.any((w & 0x1FFF) * 8 > 62000)                   # offsets near the 65 535-byte limit
    assert np.any(w == 0x4000)                                # DF alone: atomic
