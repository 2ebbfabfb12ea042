"""Where a short engine run's fixed cost goes: bench.py's cfg 2
steps (tx generate + rx verify over 1 M x 1500 B frames, 4 rotations, 8 in
flight) through one engine run of K steps, timed the way bench.py times it
(synchronise, then the host clock), with host timestamps at each phase:
start call, first submit returned, last submit returned, the last step seen
done (sccsum_engine_wait), stop returned, and the device idle again
(torch.cuda.synchronize).  Prints one JSON line per K with the median over
reps of each phase (us) and the per-step time the run would need for no fixed
cost at all (the K=200 run's rate).

    python tools/dev/run_cost_probe.py [K ...]      (default 5 20 200)

RUN_COST_GAP_MS=g: the host sleeps g ms before each run (an idle GPU between
runs, as bench.py's checks between its warm-up and timed runs leave it).
RUN_COST_STOP_FIRST=1: stop right after the last submit, then wait on the
last step (the "last_done" phase is then the stop call, "stop" the wait).
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from seastar_amd import batch, devsynth  # noqa: E402


def main():
    ks = [int(a) for a in sys.argv[1:]] or [5, 20, 200]
    reps = int(os.environ.get("RUN_COST_REPS", "5"))
    gap_s = float(os.environ.get("RUN_COST_GAP_MS", "0")) / 1e3  # host idle before each run (the GPU idles too)
    stop_first = bool(os.environ.get("RUN_COST_STOP_FIRST"))  # stop, then wait (phases last_done / stop swap)
    dev = torch.device("cuda:0")
    n, R = 1 << 20, 4
    o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    txs, rxs = [], []
    for r in range(R):
        txs.append(devsynth.udp_frames(n, 1500, seed=11 + r, device=dev))
        first = batch.ipv4_frames(txs[-1], out2=o_tx)
        rxs.append(devsynth.store_checksums(txs[-1], first))
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    eng = batch.Engine(0, frames=True, ring_slots=1024, max_in_flight=8)
    preps = [eng.prepare([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    for K in ks:
        ph = {k: [] for k in ("start", "first_submit", "last_submit", "last_done", "stop", "synced")}
        walls = []
        for rep in range(reps + 1):  # the first run warms
            torch.cuda.synchronize()
            if gap_s:
                time.sleep(gap_s)
            t0 = time.perf_counter()
            eng.start(s)
            t1 = time.perf_counter()
            eng.submit_prepared(preps[0])
            t2 = time.perf_counter()
            for k in range(1, K):
                eng.submit_prepared(preps[k % R])
            t3 = time.perf_counter()
            if stop_first:  # the grid leaves as soon as its published steps are done
                eng.stop()
                t4 = time.perf_counter()
                eng.wait(eng.last_step)
                t5 = time.perf_counter()
            else:
                eng.wait(eng.last_step)
                t4 = time.perf_counter()
                eng.stop()
                t5 = time.perf_counter()
            torch.cuda.synchronize()
            t6 = time.perf_counter()
            if rep == 0:
                continue
            for name, a, b in (("start", t0, t1), ("first_submit", t1, t2), ("last_submit", t2, t3),
                               ("last_done", t3, t4), ("stop", t4, t5), ("synced", t5, t6)):
                ph[name].append((b - a) * 1e6)
            walls.append((t6 - t0) * 1e6)
        d = {"steps": K, "wall_us": round(statistics.median(walls), 1),
             "wall_us_per_step": round(statistics.median(walls) / K, 2)}
        d.update({f"{k}_us": round(statistics.median(v), 1) for k, v in ph.items()})
        print(json.dumps(d), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
