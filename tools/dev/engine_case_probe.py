"""Replays one seeded engine fuzz case (tests/test_gpu_fuzz.py::test_fuzz_engine_steps) with
knob overrides and reports every step / batch whose results differ from the oracle (dev probe).
usage: python tools/dev/engine_case_probe.py CASE [sync_every] [fill_single_max]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "..", "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import test_gpu_fuzz as F  # noqa: E402
from seastar_amd import batch, native  # noqa: E402

case = int(sys.argv[1])
lib = native.load()
native.check(lib.sccsum_init(0), "init")
torch.cuda.set_device(0)
dev = torch.device("cuda:0")
rng = np.random.default_rng(5000 + case)
fill = case % 2 == 1
knobs = F._knobs(rng, lib, fill=True)
if len(sys.argv) > 2:
    native.check(lib.sccsum_set_engine_sync_every(int(sys.argv[2])), "sync")
if len(sys.argv) > 3:
    native.check(lib.sccsum_set_fill_single_max(int(sys.argv[3])), "single")
plan = []
for _ in range(int(rng.integers(10, 40))):
    if fill and rng.random() < 0.3:
        n = int(rng.choice([1, 64, 700]))
        L = F._lengths(rng, n, huge=False, lo=20)
        off, total, kind = F._layout(rng, L, disjoint=True)
        buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
        F._ipv4_headers(rng, buf, off, L)
        b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
        out2 = torch.empty(2 * n, dtype=torch.int16, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        mode = int(rng.choice([native.FILL_IP | native.FILL_L4, native.FILL_L4, native.FILL_IP | native.FILL_ICMP_ECHO]))
        plan.append(("fill", (b, out2, st, buf, off, L, total, mode)))
        continue
    items, wants = [], []
    for _ in range(int(rng.integers(1, native.ENGINE_MAX_BATCHES + 1))):
        n = int(rng.choice([0, 1, 64, 65, 500, 3000]))
        L = F._lengths(rng, n, huge=False)
        off, total, kind = F._layout(rng, L)
        if kind == "shuffled":
            off, L = F._shuffle_pairs(rng, off, L)
        buf = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
        F._ipv4_headers(rng, buf, off, L)
        b = batch.PacketBatch.from_host(buf[:total], off, L, device=dev)
        out2 = torch.full((max(2 * n, 2),), -1, dtype=torch.int16, device=dev) if rng.random() < 0.67 else None
        st = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)
        items.append((b, out2, st))
        wants.append(oracle.batch_ipv4(buf, off, L))
    plan.append(("sum", (items, wants)))
mif = int(rng.choice([2, 8, 64]))
eng = batch.Engine(0, frames=True, max_steps=256, max_in_flight=mif, fill=fill)
stream = torch.cuda.Stream()
torch.cuda.synchronize()
steps = []
eng.start(stream)
for what, data in plan:
    if what == "fill":
        steps.append(eng.submit_fill([data[:3]], data[7]))
    else:
        steps.append(eng.submit(data[0]))
eng.stop()
stream.synchronize()
print("knobs", knobs, "max_in_flight", mif, "fill", fill, "steps", len(plan), "last step", steps[-1])
for k, ((what, data), s) in enumerate(zip(plan, steps)):
    if what != "sum":
        continue
    for j, (it, (w2, wst)) in enumerate(zip(*data)):
        n = it[0].n
        gst = it[2][:n].cpu().numpy()
        if not np.array_equal(gst, wst):
            print(f"plan {k} step {s} batch {j}/{len(data[0])}: n {n} B? out2 {it[1] is not None}: "
                  f"{int((gst == 0xEE).sum())} never written, {int((gst != wst).sum())} differ")
print("kinds:", [w for w, _ in plan])
print("sizes:", [[it[0].n for it in d[0]] if w == "sum" else d[0].n for w, d in plan])
