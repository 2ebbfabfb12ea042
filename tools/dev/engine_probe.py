"""Where a resident-engine run's time goes: with the
SCCSUM_AB_TIMELINE build (tools/build_ab.sh timeline=SCCSUM_AB_TIMELINE) every
engine wave counts its waits for an unpublished step (and the time asleep),
its reloads of the published-tiles mirror, its descriptor walks (and their
time), its completion flushes (and their time) and its polls of host memory.  For cfg 2-shaped steps (tx + verify-only
rx, n frames each) this prints, per step size, the step time, the host's time
blocked in submit, and those per-wave figures (us).

    SCCSUM_LIB=seastar_amd/lib/ab/libsccsum_timeline.so python tools/dev/engine_probe.py

ENGINE_MIXED=1: cfg 3's steps instead (one verify-only batch of Zipf frames,
ENGINE_FRAMES frames each).
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


def step_spread(rec, K):
    """Per step of the run: how far apart its 64 dequeue groups and 8 XCDs
    finished, how many later steps had begun on some XCD when it completed,
    and each XCD's lag behind the step's first XCD to finish (us), by tenths."""
    grp = rec[:1024 * 64].reshape(1024, 64)[:K].astype(np.float64)
    xcd = rec[1024 * 64:].reshape(1024, 8, 2)[:K]
    fin = xcd[:, :, 0].astype(np.float64)
    first = (~xcd[:, :, 1]).astype(np.float64)  # stored complemented
    ok = (grp.min(axis=1) > 0) & (fin.min(axis=1) > 0)
    done = grp.max(axis=1)
    ahead = []
    for k in range(K):
        later = first[k + 1:k + 17].min(axis=1) if k + 1 < K else np.array([])
        ahead.append(int((later < done[k]).sum()))
    tenth = lambda a: [round(float(np.mean(c)), 1) for c in np.array_split(np.asarray(a, dtype=np.float64), 10)]
    gs = (grp.max(axis=1) - grp.min(axis=1)) * TICK_US
    xs = (fin.max(axis=1) - fin.min(axis=1)) * TICK_US
    lag = (fin - fin.min(axis=1, keepdims=True)) * TICK_US
    glag = ((grp - grp.min(axis=1, keepdims=True)) * TICK_US)[ok]
    return {"steps_recorded": int(ok.sum()),
            "group_finish_spread_us_by_tenth": tenth(gs[ok]),
            "xcd_finish_spread_us_by_tenth": tenth(xs[ok]),
            "later_steps_begun_at_completion_by_tenth": tenth(np.asarray(ahead)[ok]),
            "step_interval_us_by_tenth": tenth(np.diff(done[ok]) * TICK_US),
            "group_lag_us_last_tenth_by_g_mod_4": [round(float(v), 1) for v in
                glag[-max(1, K // 10):].mean(axis=0).reshape(16, 4).mean(axis=0)],
            "slowest_groups_last_tenth": [int(g) for g in np.argsort(-glag[-max(1, K // 10):].mean(axis=0))[:6]],
            "fastest_groups_last_tenth": [int(g) for g in np.argsort(glag[-max(1, K // 10):].mean(axis=0))[:6]],
            "xcd_lag_us_first_tenth": [round(float(v), 1) for v in lag[ok][:max(1, K // 10)].mean(axis=0)],
            "xcd_lag_us_last_tenth": [round(float(v), 1) for v in lag[ok][-max(1, K // 10):].mean(axis=0)]}


def main():
    lib = native.load()
    fn = getattr(lib, "sccsum_ab_engine_stats", None)  # timeline builds only
    if fn is not None:
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    tl_fn = getattr(lib, "sccsum_ab_timeline", None)  # per-wave start / first data / end / tiles
    if tl_fn is not None:
        tl_fn.restype = ctypes.c_int
        tl_fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    st_fn = getattr(lib, "sccsum_ab_step_times", None)  # per-step group / XCD retire times
    if st_fn is not None:
        st_fn.restype = ctypes.c_int
        st_fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    dev = torch.device("cuda:0")
    flights = [int(x) for x in os.environ.get("ENGINE_IN_FLIGHT", "2").split(",")]
    sizes = [int(x) for x in os.environ.get("ENGINE_FRAMES", f"{1 << 18},{1 << 20}").split(",")]
    K = int(os.environ.get("ENGINE_STEPS", "20"))
    for n, in_flight in [(n, f) for n in sizes for f in flights]:
        R = 4
        o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
        mixed = bool(os.environ.get("ENGINE_MIXED"))  # cfg 3's steps: one verify-only Zipf batch each
        if mixed:
            from seastar_amd import synth
            lens = synth.zipf_lengths(n, seed=1234)
            txs = []
            rxs = [devsynth.mixed_frames(lens, seed=7 * r, device=dev) for r in range(R)]
            for rx in rxs:
                batch.ipv4_fill(rx, native.FILL_IP | native.FILL_L4)
        elif os.environ.get("ENGINE_BENCH_DATA"):  # bench.py's cfg 2 batches: rx = tx with its checksums stored
            txs, rxs = [], []
            for r in range(R):
                txs.append(devsynth.udp_frames(n, 1500, seed=11 + r, device=dev))
                first = batch.ipv4_frames(txs[-1], out2=o_tx)
                rxs.append(devsynth.store_checksums(txs[-1], first))
        else:
            txs = [devsynth.udp_frames(n, 1500, seed=11 + r, device=dev) for r in range(R)]
            rxs = [devsynth.udp_frames(n, 1500, seed=31 + r, device=dev) for r in range(R)]
        sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
        eng = batch.Engine(0, frames=True, max_steps=K + 8, max_in_flight=in_flight)
        preps = [eng.prepare([(rxs[r], None, sts[r])] if mixed else [(txs[r], o_tx, None), (rxs[r], None, sts[r])])
                 for r in range(R)]
        s = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        for rep in range(2):  # the first run warms
            stats = np.zeros((16384, 8), dtype=np.uint64)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            steps_rec = np.zeros(1024 * 64 + 1024 * 16, dtype=np.uint64)
            if st_fn is not None:  # clear the last run's records
                native.check(st_fn(steps_rec.ctypes.data, steps_rec.nbytes), "sccsum_ab_step_times")
            e0.record(s)
            t_start = time.perf_counter()
            eng.start(s)
            start_us = (time.perf_counter() - t_start) * 1e6
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
            if st_fn is not None:
                native.check(st_fn(steps_rec.ctypes.data, steps_rec.nbytes), "sccsum_ab_step_times")
        # submit k returns when step k - in_flight is done: the spacing of the returns is the
        # grid's step time, here in 10 quantiles of the run
        gaps = np.diff(np.array(ret[in_flight:])) * 1e6
        q = [round(float(np.mean(c)), 1) for c in np.array_split(gaps, 10)] if len(gaps) >= 10 else []
        d = {"frames_per_batch": n, "steps": K, "in_flight": in_flight,
             "run_us": round(e0.elapsed_time(e1) * 1e3, 1),
             "us_per_step": round(e0.elapsed_time(e1) * 1e3 / K, 1),
             "host_start_call_us": round(start_us, 1),
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
        if st_fn is not None:
            d.update(step_spread(steps_rec, min(K, 1024)))
        if tl_fn is not None and st_fn is not None:  # where a run's fixed cost goes
            tl = np.zeros((16384, 4), dtype=np.uint64)
            native.check(tl_fn(tl.ctypes.data, tl.nbytes), "sccsum_ab_timeline")
            w = tl[tl[:, 0] > 0].astype(np.float64)
            grp = steps_rec[:1024 * 64].reshape(1024, 64)[:K].astype(np.float64)
            xcd = steps_rec[1024 * 64:].reshape(1024, 8, 2)[:K]
            k_start = w[:, 0].min()
            first_retire0 = (~xcd[0, :, 1]).astype(np.float64).min()
            last_done = grp[K - 1].max()
            fd = w[w[:, 1] > 0, 1]
            d["run_phases_us"] = {
                "waves_started_over": round((w[:, 0].max() - k_start) * TICK_US, 1),
                "kernel_start_to_first_data_median": round((np.median(fd) - k_start) * TICK_US, 1),
                "kernel_start_to_first_data_min": round((fd.min() - k_start) * TICK_US, 1),
                "kernel_start_to_step0_first_retire": round((first_retire0 - k_start) * TICK_US, 1),
                "step0_done": round((grp[0].max() - k_start) * TICK_US, 1),
                "last_step_done": round((last_done - k_start) * TICK_US, 1),
                "last_step_done_to_last_wave_end": round((w[:, 2].max() - last_done) * TICK_US, 1),
                "kernel_span": round((w[:, 2].max() - k_start) * TICK_US, 1),
                "events_minus_kernel_span": round(e0.elapsed_time(e1) * 1e3 - (w[:, 2].max() - k_start) * TICK_US, 1)}
        print(json.dumps(d), flush=True)
        eng.close()
        del txs, rxs


if __name__ == "__main__":
    main()
