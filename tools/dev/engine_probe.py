"""Where a resident-engine run's time goes: with the
SCCSUM_AB_TIMELINE build (tools/build_ab.sh timeline=SCCSUM_AB_TIMELINE) every
engine wave counts its waits for an unpublished step (and the time asleep),
its reloads of the published-tiles mirror, its descriptor walks (and their
time), its completion flushes (and their time) and its polls of host memory.  For cfg 2-shaped steps (tx + verify-only
rx, n frames each) this prints, per step size, the step time, the host's time
blocked in submit, and those per-wave figures (us).

    SCCSUM_LIB=seastar_amd/lib/ab/libsccsum_timeline.so python tools/dev/engine_probe.py
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native  # noqa: E402

TICK_US = 0.01  # 100 MHz


def main():
    lib = native.load()
    fn = getattr(lib, "sccsum_ab_engine_stats", None)  # timeline builds only
    if fn is not None:
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    dev = torch.device("cuda:0")
    flights = [int(x) for x in os.environ.get("ENGINE_IN_FLIGHT", "2").split(",")]
    sizes = [int(x) for x in os.environ.get("ENGINE_FRAMES", f"{1 << 18},{1 << 20}").split(",")]
    K = int(os.environ.get("ENGINE_STEPS", "20"))
    for n, in_flight in [(n, f) for n in sizes for f in flights]:
        R = 4
        txs = [devsynth.udp_frames(n, 1500, seed=11 + r, device=dev) for r in range(R)]
        rxs = [devsynth.udp_frames(n, 1500, seed=31 + r, device=dev) for r in range(R)]
        o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
        sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
        eng = batch.Engine(0, frames=True, max_steps=K + 8, max_in_flight=in_flight)
        preps = [eng.prepare([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
        s = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        for rep in range(2):  # the first run warms
            stats = np.zeros((16384, 8), dtype=np.uint64)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            eng.start(s)
            blocked, ret = [], []
            for k in range(K):
                t0 = time.perf_counter()
                eng.submit_prepared(preps[k % R])
                ret.append(time.perf_counter())
                blocked.append(ret[-1] - t0)
            eng.stop()
            e1.record(s)
            torch.cuda.synchronize()
            if fn is not None:
                native.check(fn(stats.ctypes.data, stats.nbytes), "sccsum_ab_engine_stats")
        # submit k returns when step k - in_flight is done: the spacing of the returns is the
        # grid's step time, here in 10 quantiles of the run
        gaps = np.diff(np.array(ret[in_flight:])) * 1e6
        q = [round(float(np.mean(c)), 1) for c in np.array_split(gaps, 10)] if len(gaps) >= 10 else []
        d = {"frames_per_batch": n, "steps": K, "in_flight": in_flight,
             "run_us": round(e0.elapsed_time(e1) * 1e3, 1),
             "us_per_step": round(e0.elapsed_time(e1) * 1e3 / K, 1),
             "host_blocked_us_mean": round(float(np.mean(blocked)) * 1e6, 1),
             "host_blocked_us_max": round(float(np.max(blocked)) * 1e6, 1),
             "step_us_by_tenth_of_run": q,
             "longest_submits_us_at_step": sorted(((round(b * 1e6, 1), k) for k, b in enumerate(blocked)),
                                                  reverse=True)[:5]}
        live = stats[(stats[:, 3] > 0)]
        if fn is not None and len(live):
            w = live.astype(np.float64)
            d.update({
                "waves": int(len(live)),
                "waits_per_wave": round(float(w[:, 0].mean()), 2),
                "asleep_us_per_wave": round(float(w[:, 1].mean()) * TICK_US, 1),
                "asleep_us_max": round(float(w[:, 1].max()) * TICK_US, 1),
                "pub_reloads_per_wave": round(float(w[:, 2].mean()), 2),
                "walks_per_wave": round(float(w[:, 3].mean()), 2),
                "walk_us_per_wave": round(float(w[:, 4].mean()) * TICK_US, 1),
                "flushes_per_wave": round(float(w[:, 5].mean()), 2),
                "flush_us_per_wave": round(float(w[:, 6].mean()) * TICK_US, 1),
                "host_polls_total": int(w[:, 7].sum())})
        print(json.dumps(d), flush=True)
        eng.close()
        del txs, rxs


if __name__ == "__main__":
    main()
