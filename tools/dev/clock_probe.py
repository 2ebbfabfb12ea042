"""Clock and power while cfg 2 runs for ~2 s as multi launches and as one
engine run: the GPU's hwmon (freq1_input = shader clock, power1_average /
power1_input) sampled every 5 ms from a host thread, printed as 100 ms means
beside the step rate of the same 100 ms.  Reads sysfs only (no settings).

    python tools/dev/clock_probe.py
"""
import glob
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth  # noqa: E402


def hwmon_dir():
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    d = glob.glob(f"/sys/bus/pci/devices/{bdf}/hwmon/hwmon*")
    return bdf, (d[0] if d else None)


def read_int(path):
    try:
        with open(path) as f:
            return int(f.read().split()[0])
    except (OSError, ValueError):
        return None


def main():
    bdf, hw = hwmon_dir()
    files = {k: os.path.join(hw, f) for k, f in (("sclk_hz", "freq1_input"), ("mclk_hz", "freq2_input"),
                                                  ("power_uw", "power1_average"), ("power_in_uw", "power1_input"))} if hw else {}
    for t in sorted(glob.glob(os.path.join(hw, "temp*_input"))) if hw else []:  # every readable sensor, by label
        lab = os.path.join(os.path.dirname(t), os.path.basename(t).replace("_input", "_label"))
        try:
            name = open(lab).read().strip()
        except OSError:
            name = os.path.basename(t)
        files[f"temp_{name}_mc"] = t
    print(json.dumps({"bdf": bdf, "hwmon": hw, "readable": {k: read_int(v) for k, v in files.items()}}), flush=True)
    dev = torch.device("cuda:0")
    n, R, K = 1 << 20, 4, 4000
    txs = [devsynth.udp_frames(n, 1500, seed=11 + r, device=dev) for r in range(R)]
    rxs = [devsynth.udp_frames(n, 1500, seed=31 + r, device=dev) for r in range(R)]
    o_tx = torch.empty(2 * n, dtype=torch.int16, device=dev)
    sts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(R)]
    s = torch.cuda.Stream(device=dev)
    pre = [batch.prepare_ipv4_frames_multi([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
    for form in ("multi", "engine"):
        torch.cuda.synchronize()
        time.sleep(2.0)
        samples, stop = [], threading.Event()

        def sampler():
            while not stop.is_set():
                samples.append((time.perf_counter(), {k: read_int(v) for k, v in files.items()}))
                time.sleep(0.005)

        th = threading.Thread(target=sampler, daemon=True)
        th.start()
        marks = []  # (host time, steps done)
        t_start = time.perf_counter()
        if form == "multi":
            ev = []
            for k in range(K):
                pre[k % R](s)
                if (k + 1) % 100 == 0:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(s)
                    ev.append((k + 1, e))
            torch.cuda.synchronize()
            t_end = time.perf_counter()
            # GPU time of each 100-launch block from the events; host times placed back from the run's end
            gpu = [0.0] + [ev[0][1].elapsed_time(e) / 1e3 for _, e in ev[1:]]
            span = gpu[-1]
            marks = [(t_end - (span - g), k1) for g, (k1, _) in zip(gpu, ev)]
        else:
            eng = batch.Engine(0, frames=True, max_steps=K + 4, max_in_flight=8)
            pe = [eng.prepare([(txs[r], o_tx, None), (rxs[r], None, sts[r])]) for r in range(R)]
            eng.start(s)
            for k in range(K):
                eng.submit_prepared(pe[k % R])
                if k >= 8 and (k - 8 + 1) % 100 == 0:
                    marks.append((time.perf_counter(), k - 8 + 1))
            eng.stop()
            torch.cuda.synchronize()
            eng.close()
        torch.cuda.synchronize()
        stop.set()
        th.join()
        t = np.array([m[0] for m in marks])
        k = np.array([m[1] for m in marks])
        rows = []
        for i in range(1, len(t)):
            win = [v for (ts, v) in samples if t[i - 1] <= ts < t[i]]
            row = {"t_ms": round((t[i] - t_start) * 1e3), "us_per_step": round((t[i] - t[i - 1]) / (k[i] - k[i - 1]) * 1e6, 1)}
            for key in files:
                vals = [w[key] for w in win if w[key] is not None]
                if vals:
                    row[key] = round(float(np.mean(vals)) / (1e3 if key.endswith("_mc") else 1e6), 1)
            rows.append(row)
        print(json.dumps({"form": form, "steps": K, "rows_every_100_steps": rows}), flush=True)


if __name__ == "__main__":
    main()
