"""Pins the oracle (oracle/sccsum_oracle.c) before it is trusted as checker.

1. Known answers: tests/golden/kat.json — outputs of the compiled reference
   recorded in SURVEY.md §8(c) plus the RFC 1071 / RFC 791 published vectors.
2. An independent formulation: the closed form of the reference's result
   (SURVEY.md finding 4: htons(~fold(S)) with S the integer sum of big-endian
   words, fold(0)=0, fold(S)=1+((S-1) mod 65535)), in pure Python.
3. The stateful semantics of the inline members (ip_checksum.hh:40-69) and of
   fragment walks (ip_checksum.cc:64-68), against a pure-Python model.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def closed_form(data: bytes, seed: int = 0) -> int:
    """uint16 value (little-endian host) the reference returns."""
    if len(data) % 2:
        data = data + b"\0"
    s = seed + sum(int.from_bytes(data[i:i + 2], "big") for i in range(0, len(data), 2))
    f = 0 if s == 0 else 1 + (s - 1) % 65535
    c = ~f & 0xFFFF
    return ((c & 0xFF) << 8) | (c >> 8)


class PyChecksummer:
    """Pure-Python statement of struct checksummer (ip_checksum.hh:35-69)."""

    def __init__(self):
        self.csum = 0
        self.odd = False

    def u8(self, v):
        self.csum += v if self.odd else v << 8
        self.odd = not self.odd

    def u16(self, v):
        if self.odd:
            self.u8(v >> 8)
            self.u8(v & 0xFF)
        else:
            self.csum += v

    def u32(self, v):
        if self.odd:
            self.u16(v & 0xFFFF)
            self.u16(v >> 16)
        else:
            self.csum += v

    def data(self, b: bytes):
        for x in b:
            self.u8(x)

    def get(self):
        s = self.csum
        f = 0 if s == 0 else 1 + (s - 1) % 65535
        c = ~f & 0xFFFF
        return ((c & 0xFF) << 8) | (c >> 8)


def test_kat():
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    for case in kat["ip_checksum"]:
        data = bytes.fromhex(case["hex"])
        want = int.from_bytes(bytes.fromhex(case["result_bytes"]), "little")
        assert oracle.ip_checksum(data) == want, case["name"]
        assert closed_form(data) == want, case["name"]


def test_closed_form_random():
    rng = np.random.default_rng(123)
    for _ in range(3000):
        n = int(rng.integers(0, 300))
        kind = rng.integers(0, 4)
        if kind == 0:
            d = bytes(n)
        elif kind == 1:
            d = b"\xff" * n
        else:
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.ip_checksum(d) == closed_form(d), (n, kind)


def test_closed_form_long():
    rng = np.random.default_rng(7)
    for n in (1500, 9000, 65535, 65536):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.ip_checksum(d) == closed_form(d)


def test_fragments_equal_contiguous():
    """1501 random bytes split 7/1/333/1160 = contiguous;
    plus the packet_test.cc fragment sizes 5/31/65/4096/4096."""
    rng = np.random.default_rng(99)
    for sizes in ([7, 1, 333, 1160], [5, 31, 65, 4096, 4096], [1] * 17, [3, 3, 3, 2, 9]):
        total = sum(sizes)
        d = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
        c = oracle.new()
        pos = 0
        for s in sizes:
            oracle.sum_bytes(c, d[pos:pos + s])
            pos += s
        assert oracle.get(c) == oracle.ip_checksum(d) == closed_form(d)
        # and the fragment-list entry point
        arrs = [np.frombuffer(d[sum(sizes[:i]):sum(sizes[:i + 1])], np.uint8).copy() for i in range(len(sizes))]
        bases = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        szs = (ctypes.c_size_t * len(arrs))(*sizes)
        c2 = oracle.new()
        oracle.lib().oracle_sum_fragments(ctypes.byref(c2), bases, szs, len(arrs))
        assert oracle.get(c2) == oracle.get(c)


def test_inline_members_model():
    rng = np.random.default_rng(5)
    for _ in range(500):
        c = oracle.new()
        m = PyChecksummer()
        for _ in range(int(rng.integers(1, 12))):
            op = int(rng.integers(0, 4))
            if op == 0:
                v = int(rng.integers(0, 256))
                oracle.lib().oracle_sum_u8(ctypes.byref(c), v)
                m.u8(v)
            elif op == 1:
                v = int(rng.integers(0, 65536))
                oracle.lib().oracle_sum_u16(ctypes.byref(c), v)
                m.u16(v)
            elif op == 2:
                v = int(rng.integers(0, 2**32))
                oracle.lib().oracle_sum_u32(ctypes.byref(c), v)
                m.u32(v)
            else:
                d = rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
                oracle.sum_bytes(c, d)
                m.data(d)
            assert bool(c.odd) == m.odd
        assert oracle.get(c) == m.get()


def test_pseudo_header_len_wrap():
    """len 65536 == len 0 (uint16_t parameter, ip.hh:70-75)."""
    a = oracle.pseudo_seed(0xC0A80001, 0x0A000002, 6, 65536)
    b = oracle.pseudo_seed(0xC0A80001, 0x0A000002, 6, 0)
    assert a == b
    m = PyChecksummer()
    for v in (0xC0A80001, 0x0A000002):
        m.u32(v)
    m.u8(0)
    m.u8(6)
    m.u16(1480)
    c = oracle.new()
    oracle.lib().oracle_pseudo_header(ctypes.byref(c), 0xC0A80001, 0x0A000002, 6, 1480)
    assert c.csum == m.csum


@pytest.mark.parametrize("nthreads", [1, 4])
def test_batch_drivers_match_single_calls(nthreads):
    from seastar_amd import synth

    buf, off, lens, meta = synth.udp_ipv4_frames(200, 1500, seed=3)
    out2, st = oracle.batch_ipv4(buf, off, lens, nthreads=nthreads)
    for i in range(0, 200, 17):
        f = buf[int(off[i]):int(off[i]) + 1500].tobytes()
        assert out2[i, 0] == closed_form(f[:20])
        seed = int(meta["src"][i]) + int(meta["dst"][i]) + 17 + 1480
        assert out2[i, 1] == closed_form(f[20:], seed)
    assert np.all(st & 0x4 == 0)
    spans = oracle.batch_spans(buf, off, lens, nthreads=nthreads)
    assert spans[5] == closed_form(buf[int(off[5]):int(off[5]) + 1500].tobytes())


# ---- RSS (Toeplitz) --------------------------------------------------------

RSS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rss.json")))


def test_toeplitz_matches_reference_build():
    """oracle_toeplitz vs the reference's own toeplitz_hash (rss.json, built
    from include/seastar/net/toeplitz.hh; MS RSS suite rows included)."""
    for c in RSS["cases"]:
        data = bytes.fromhex(c["data"]) if c["data"] != "-" else b""
        assert oracle.toeplitz(bytes.fromhex(c["key"]), data) == c["hash"], c


def _fwd_hash(frame: bytes, mode: int) -> bytes | None:
    """forward_hash bytes, restated from the reference code in Python:
    ip.cc:77-92 + udp.cc:153-161 + tcp.hh:852-862 (mode 0), ip.cc:186-197 (mode 1)."""
    if len(frame) < 20:
        return None
    data = frame[12:20]
    proto = frame[9]
    need = {6: 20, 17: 8}.get(proto, 0)
    if mode == 0:
        frag = (frame[6] << 8) | frame[7]
        if need and not (frag & 0x2000) and not (frag & 0x1FFF) and len(frame) >= 20 + need:
            data += frame[20:24]
    else:
        l4_off = 4 * (frame[0] & 0xF)
        ip_len = (frame[2] << 8) | frame[3]
        l4_end = min(ip_len, len(frame))
        if l4_off > l4_end:
            return None
        if need and l4_end - l4_off >= need:
            data += frame[l4_off:l4_off + 4]
    return data


@pytest.mark.parametrize("mode", [0, 1])
def test_rss_forward_hash_construction(mode):
    from seastar_amd import synth

    buf, off, lens = synth.rss_frames(3000, seed=9)
    for key in (oracle.RSS_KEY_40, bytes.fromhex(RSS["cases"][0]["key"]), bytes(range(1, 9))):
        h, st = oracle.batch_ipv4_rss(buf, off, lens, key=key, mode=mode)
        for i in range(off.size):
            fr = bytes(buf[int(off[i]):int(off[i]) + int(lens[i])])
            d = _fwd_hash(fr, mode)
            if d is None:
                assert st[i] == 4 and h[i] == 0
            else:
                assert st[i] == 0 and h[i] == oracle.toeplitz(key, d), (i, len(fr))
    # the batch really exercises the branches
    kinds = {len(_fwd_hash(bytes(buf[int(o):int(o) + int(L)]), mode) or b"") for o, L in zip(off, lens)}
    assert {0, 8, 12} <= kinds


# ---- rx / tx semantics of the frames drivers (ip.cc:114-299, 464-474) -------


def _py_rx(frame: bytes):
    """(out2 pair, status) of one received frame, restated in Python from
    ipv4::handle_received_packet (ip.cc:114-229) and the L4 receivers."""
    if len(frame) < 20:
        return (0, 0), 4
    ipc = closed_form(frame[:20])
    ihl, ip_len, proto = frame[0] & 0xF, (frame[2] << 8) | frame[3], frame[9]
    fragw = (frame[6] << 8) | frame[7]
    l4_end = min(ip_len, len(frame))
    st = 0
    if len(frame) < ip_len or (fragw & 0x1FFF) * 8 + l4_end > 65535 or 4 * ihl > l4_end:
        st |= 4
    if ipc == 0:
        st |= 1
    if fragw & 0x3FFF:  # reassembly first: no L4 on a fragment
        return (ipc, 0), st | 16
    l4 = frame[4 * ihl:l4_end] if 4 * ihl <= l4_end else b""
    seed = 0
    if proto in (6, 17):
        seed = int.from_bytes(frame[12:16], "big") + int.from_bytes(frame[16:20], "big") + proto + (len(l4) & 0xFFFF)
    l4c = closed_form(l4, seed)
    return (ipc, l4c), st | (2 if l4c == 0 else 0)


def test_frames_driver_fragments_and_protocols():
    """oracle_batch_ipv4 on fragments (first / middle / last / past 65 535),
    ICMP and other protocols (no pseudo-header), TCP / UDP, malformed frames:
    each frame against the Python restatement of the rx path."""
    from seastar_amd import synth

    rng = np.random.default_rng(0xF7)
    n = 3000
    lens = rng.integers(0, 2200, n).astype(np.uint32)
    off, total = synth.pack(lens, seed=5, max_gap=3)
    buf = rng.integers(0, 256, size=int(total) + 8, dtype=np.uint8)
    fw = synth.frag_words(rng, n)
    for i in range(n):
        o, L = int(off[i]), int(lens[i])
        if L >= 20:
            ihl = 5 if rng.random() < 0.8 else int(rng.integers(0, 16))
            ip_len = L if rng.random() < 0.8 else int(rng.integers(0, L + 30))
            buf[o] = 0x40 | ihl
            buf[o + 2], buf[o + 3] = ip_len >> 8, ip_len & 0xFF
            buf[o + 6], buf[o + 7] = int(fw[i]) >> 8, int(fw[i]) & 0xFF
            buf[o + 9] = int(rng.choice([6, 17, 1, 47]))
    out2, st = oracle.batch_ipv4(buf, off, lens)
    seen = set()
    for i in range(n):
        fr = bytes(buf[int(off[i]):int(off[i]) + int(lens[i])])
        want, wst = _py_rx(fr)
        assert tuple(out2[i]) == want and st[i] == wst, (i, fr[:20].hex())
        seen.add(wst & 0x1C)
    assert {0, 4, 16, 20} <= seen


def test_fill_driver_icmp_echo_and_fragments():
    """oracle_batch_ipv4_fill: an ICMP echo request becomes the reply
    (icmp::received, ip.cc:464-474: type 0, code 0, checksum over the message
    with the field 0); other ICMP types, fragments and short messages are
    left alone; an all-zero message gets 0xffff; fragments get the IP
    checksum only (ip.cc:256-278)."""
    frames = []
    msgs = [bytes([8, 5, 0xAA, 0xBB]) + bytes(range(40)), bytes([8, 0, 1, 2]) + bytes(60),
            bytes([0, 0, 1, 2]) + bytes(range(12)), bytes([8, 0, 1, 2, 3, 4, 5]), bytes([8, 9, 9, 9]) + b"\x01" * 33]
    for k, m in enumerate(msgs + [msgs[0]]):
        f = bytearray(20) + m
        f[0], f[2], f[3], f[9] = 0x45, len(f) >> 8, len(f) & 0xFF, 1
        if k == len(msgs):  # the same echo request as a first fragment
            f[6] = 0x20
        frames.append(bytes(f))
    lens = np.array([len(f) for f in frames], np.uint32)
    off = np.concatenate([[1], 1 + np.cumsum(lens)[:-1]]).astype(np.uint64)
    buf = np.zeros(int(off[-1] + lens[-1]) + 3, np.uint8)
    for o, f in zip(off, frames):
        buf[int(o):int(o) + len(f)] = np.frombuffer(f, np.uint8)
    got, out2, st = oracle.batch_ipv4_fill(buf, off, lens, 0x11)
    for i, f in enumerate(frames):
        g = bytes(got[int(off[i]):int(off[i]) + len(f)])
        assert g[10:12] == closed_form(f[:10] + b"\0\0" + f[12:20]).to_bytes(2, "little")
        m = f[20:]
        echo = m[0] == 8 and len(m) >= 8 and i != len(msgs)
        if echo:
            r = closed_form(b"\0\0\0\0" + m[4:])
            assert g[20:] == b"\0\0" + r.to_bytes(2, "little") + m[4:] and out2[i, 1] == r and st[i] & 2
        else:
            assert g[20:] == m and not st[i] & 2
    assert out2[1, 1] == 0xFFFF  # all-zero message
    assert st[len(msgs)] & 16


def test_pinned_batch_survives_bad_cpu_lists():
    """oracle_batch_ipv4_cpus never reads past its list or overflows
    cpu_set_t: an empty list, CPU ids past CPU_SETSIZE and
    negative ids still give the single-thread results."""
    from seastar_amd import synth

    buf, off, lens, _ = synth.mixed_udp_frames(3000, seed=9, max_gap=3)
    want, want_st = oracle.batch_ipv4(buf, off, lens)
    for cpus in ([], [5000, 70000], [-1, 0, 1 << 20]):
        got, st = oracle.batch_ipv4(buf, off, lens, cpus=cpus)
        assert np.array_equal(got, want) and np.array_equal(st, want_st), cpus
