"""Where an engine fill's step time goes: a resident
run of K fills (sccsum_engine_submit_fill: a generate step, then a store step
that waits for it) over R rotated 1 M x 1500 B batches.  With the
SCCSUM_AB_TIMELINE build (tools/build_ab.sh timeline=SCCSUM_AB_TIMELINE) the
grid records, per step, each dequeue group's last tile retire and each XCD's
first and last: this prints, per fill, the generate step's span, the wait
between its last generate tile and the first store tile, the store step's span
and how the next fill's generate overlaps it (us, means over the run's second
half).  Without that build it prints the step time only.

    SCCSUM_LIB=seastar_amd/lib/ab/libsccsum_timeline.so python tools/dev/engine_fill_probe.py [K] [R]
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
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    n = 1 << 20
    lib = native.load()
    native.check(lib.sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    bs = [devsynth.udp_frames(n, 1500, seed=500 + r, device=dev) for r in range(R)]
    outs = [torch.empty(2 * n, dtype=torch.int16, device=dev) for _ in range(R)]
    mode = native.FILL_IP | native.FILL_L4
    eng = batch.Engine(0, frames=True, fill=True, max_steps=2 * K + 8, max_in_flight=8)
    preps = [eng.prepare([(bs[r], outs[r], None)], fill_mode=mode) for r in range(R)]
    stream = torch.cuda.Stream(device=dev)
    timeline = hasattr(lib, "sccsum_ab_step_times")
    rec = None
    if timeline:
        rec = np.zeros(1024 * 64 + 1024 * 16, dtype=np.uint64)
        lib.sccsum_ab_step_times(rec.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(rec.nbytes))  # clear
    torch.cuda.synchronize()
    for run in range(2):  # the first run warms up
        t0 = time.perf_counter()
        eng.start(stream)
        for k in range(K):
            eng.submit_prepared(preps[k % R])
        eng.stop()
        stream.synchronize()
        wall = time.perf_counter() - t0
        if timeline and run == 0:  # keep only the second run's record
            lib.sccsum_ab_step_times(rec.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(rec.nbytes))
    out = {"fills": K, "rotated_batches": R, "us_per_fill_wall": round(wall / K * 1e6, 1)}
    if timeline:
        native.check(lib.sccsum_ab_step_times(rec.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(rec.nbytes)),
                     "step times")
        # fill k: its generate step is step 2k, its store step 2k + 1
        S = 2 * K
        grp = rec[:1024 * 64].reshape(1024, 64)[:S].astype(np.float64)
        xcd = rec[1024 * 64:].reshape(1024, 8, 2)[:S]
        first = (~xcd[:, :, 1]).astype(np.float64).min(axis=1)  # earliest tile retire of the step
        last = grp.max(axis=1)  # latest tile retire of the step
        half = range(K // 2, K - 1)
        gen_span = [(last[2 * k] - first[2 * k]) * TICK_US for k in half]
        wait = [(first[2 * k + 1] - last[2 * k]) * TICK_US for k in half]
        store_span = [(last[2 * k + 1] - first[2 * k + 1]) * TICK_US for k in half]
        next_gen_first = [(first[2 * k + 2] - last[2 * k + 1]) * TICK_US for k in half]
        interval = [(last[2 * k + 3] - last[2 * k + 1]) * TICK_US for k in half]
        m = lambda a: round(float(np.mean(a)), 1)
        out.update({"gen_span_us": m(gen_span), "gen_last_to_first_store_us": m(wait),
                    "store_span_us": m(store_span), "next_gen_first_minus_store_last_us": m(next_gen_first),
                    "fill_interval_us": m(interval)})
    eng.close()
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    for b in bs:
        batch.ipv4_frames(b, status=st)
        torch.cuda.synchronize()
        assert int((st != 3).sum()) == 0, "filled frames do not verify"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
