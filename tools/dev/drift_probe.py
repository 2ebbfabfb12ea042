"""Does a long cfg 2 run slow down as it goes (clock / power), and does the
resident engine drift differently from launches?  Runs 400 cfg 2 steps (tx +
verify-only rx, 1 M x 1500 B frames each, 4 rotated batch pairs) as multi
launches with an event after every 20th launch (the events cost ~5 us each,
once per 20 launches), then as one engine run timed by the host (submit k
returns when step k - in_flight is done), and prints the mean step time of
each 20-step block for both.

    python tools/dev/drift_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, R, K, blk = 1 << 20, 4, int(os.environ.get("DRIFT_STEPS", "400")), 20
    txs = [devsynth.udp_frames(n, 1500, seed=11 + r, device=dev) for r in range(R)]
    rxs = [devsynth.udp_frames(n, 1500, seed=31 + r, device=dev) for r in range(R)]
    o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    s = torch.cuda.Stream(device=dev)
    pre = [batch.prepare_ipv4_frames_multi([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
    for order in ("multi", "engine", "multi", "engine"):
        torch.cuda.synchronize()
        time.sleep(1.0)  # the same idle gap before each run
        if order == "multi":
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(K // blk + 1)]
            ev[0].record(s)
            for k in range(K):
                pre[k % R](s)
                if (k + 1) % blk == 0:
                    ev[(k + 1) // blk].record(s)
            torch.cuda.synchronize()
            per = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3 / blk, 1) for i in range(K // blk)]
        else:
            eng = batch.Engine(0, frames=True, max_steps=K + 4, max_in_flight=8)
            pe = [eng.prepare([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
            ret = []
            eng.start(s)
            for k in range(K):
                eng.submit_prepared(pe[k % R])
                ret.append(time.perf_counter())
            eng.stop()
            torch.cuda.synchronize()
            eng.close()
            g = np.diff(np.array(ret[8:])) * 1e6
            per = [round(float(np.mean(c)), 1) for c in np.array_split(g, len(g) // blk)]
        print(json.dumps({"form": order, "steps": K, "us_per_step_by_block_of_20": per,
                          "first_block": per[0], "last_block": per[-1], "mean": round(float(np.mean(per)), 1)}),
              flush=True)


if __name__ == "__main__":
    main()
