"""Where a flat-kernel launch's fixed cost goes: with the
SCCSUM_AB_TIMELINE build (tools/build_ab.sh timeline=SCCSUM_AB_TIMELINE), every
wave stamps the constant clock (100 MHz) at its start, when its first chunk's
data is in registers, and at its failing dequeue, plus its tile count.  For
bench-shaped launches (cfg 2: tx + verify-only rx, 2 x 1 M x 1500 B frames in
one multi launch; and one 1 M-frame batch) this prints the spread of those
times and the per-wave idle time they imply at the launch's two ends:
  ramp  = mean over waves of (first data - earliest start)
  drain = mean over waves of (last end - own end)
both in us; (ramp + drain) x waves / waves is the launch time the stream is
not fully fed.

    SCCSUM_LIB=seastar_amd/lib/ab/libsccsum_timeline.so python tools/dev/timeline_probe.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native  # noqa: E402

TICK_US = 0.01  # 100 MHz


def stats(tl: np.ndarray) -> dict:
    st = tl[:, 0].astype(np.int64)
    live = st > 0
    last = st[live].max()
    w = tl[live & (st > last - 100_000)]  # this launch's waves (started within 1 ms of the last start)
    t0 = w[:, 0].min()
    start = (w[:, 0] - t0) * TICK_US
    first = (np.where(w[:, 1] > 0, w[:, 1], w[:, 2]) - t0) * TICK_US
    end = (w[:, 2] - t0) * TICK_US
    span = end.max()
    pct = lambda a: [round(float(np.percentile(a, q)), 2) for q in (0, 10, 50, 90, 100)]  # noqa: E731
    return {"waves": int(len(w)), "span_us": round(float(span), 2),
            "start_us_p0_10_50_90_100": pct(start), "first_data_us": pct(first), "end_us": pct(end),
            "tiles_per_wave_min_mean_max": [int(w[:, 3].min()), round(float(w[:, 3].mean()), 2), int(w[:, 3].max())],
            "ramp_us_mean": round(float(first.mean()), 2), "drain_us_mean": round(float((span - end).mean()), 2)}


def main():
    lib = native.load()
    fn = lib.sccsum_ab_timeline
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    native.check(lib.sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    n = 1 << 20
    R = 3
    txs = [devsynth.udp_frames(n, 1500, seed=11 + r, device=dev) for r in range(R)]
    rxs = [devsynth.udp_frames(n, 1500, seed=31 + r, device=dev) for r in range(R)]
    o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    s = torch.cuda.current_stream()
    from seastar_amd import synth
    nz = 3_400_000  # cfg 3: Zipf frames packed at odd offsets, one sccsum_ipv4_frames launch (bench.py's single form)
    lens = synth.zipf_lengths(nz, seed=0x5EA57A2C)
    zs = [devsynth.mixed_frames(lens, seed=7 * r + 1, device=dev) for r in range(R)]
    o_z = torch.empty(2 * nz, dtype=torch.int16, device=dev)
    cases = {
        "cfg3_step (3.4 M Zipf frames, one batch)":
            [batch.prepare_call("sccsum_ipv4_frames", z.data, z.bytes_len, z.off, z.length, o_z, None, z.n, z.max_len)
             for z in zs],
        "cfg2_step (tx + verify-only rx, 2 M frames)":
            [batch.prepare_ipv4_frames_multi([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)],
        "one 1 M-frame batch":
            [batch.prepare_ipv4_frames_multi([(txs[r], o_tx, None)]) for r in range(R)],
    }
    host = np.zeros((16384, 4), dtype=np.uint64)
    for name, pre in cases.items():
        for r in range(R):  # warm
            pre[r](s)
        torch.cuda.synchronize()
        rows = []
        for rep in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            pre[rep % R](s)
            e1.record(s)
            torch.cuda.synchronize()
            native.check(fn(host.ctypes.data, host.nbytes), "sccsum_ab_timeline")
            d = stats(host)
            d["event_us"] = round(e0.elapsed_time(e1) * 1e3, 1)
            rows.append(d)
        for d in rows:
            print(json.dumps({"case": name, **d}), flush=True)


if __name__ == "__main__":
    main()
