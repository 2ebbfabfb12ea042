"""Probe: why is one multi launch over two Zipf batches slower than two
single launches?  Times, on rotated batches: single launches over tx and rx
batches, multi launches over (tx, rx), (rx, rx'), (tx, tx'), and the same for
1500 B frames.  Prints one JSON line per case (median us per launch)."""
from __future__ import annotations

import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import batch, devsynth, native, synth  # noqa: E402


def timeit(fns, rounds=8, reps=4):
    t = []
    k = 0
    for _ in range(rounds):
        fns[k % len(fns)]()
        k += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fns[k % len(fns)]()
            k += 1
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1) / reps * 1e3)
    return round(float(np.median(t)), 1)


def main():
    native.check(native.load().sccsum_init(0), "init")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = int(os.environ.get("N", "3400000"))
    R = 4
    which = sys.argv[1:] or ["zipf", "udp"]
    for kind in which:
        if kind == "zipf":
            la = synth.zipf_lengths(n, seed=11)
            lb = synth.zipf_lengths(n, seed=12)
            A = [devsynth.mixed_frames(la, seed=100 + r, device=dev) for r in range(R)]
            B = [devsynth.mixed_frames(lb, seed=200 + r, device=dev) for r in range(R)]
        else:
            A = [devsynth.udp_frames(1 << 20, 1500, seed=100 + r, device=dev) for r in range(R)]
            B = [devsynth.udp_frames(1 << 20, 1500, seed=200 + r, device=dev) for r in range(R)]
        m = max(A[0].n, B[0].n)
        o1 = torch.empty(2 * m, dtype=torch.int16, device=dev)
        o2 = torch.empty(2 * m, dtype=torch.int16, device=dev)

        def single(bs):
            return [lambda b=b: batch.prepare_call("sccsum_ipv4_frames", b.data, b.bytes_len, b.off, b.length, o1,
                                                   None, b.n, b.max_len)(s) for b in bs]

        sts = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(R)]

        def multi(xs, ys, status=False):
            pre = [batch.prepare_ipv4_frames_multi([(x, o1, None), (y, o2, sts[i] if status else None)])
                   for i, (x, y) in enumerate(zip(xs, ys))]
            return [lambda p=p: p(s) for p in pre]

        res = {
            "single_A": timeit(single(A)),
            "single_B": timeit(single(B)),
            "multi_AB": timeit(multi(A, B)),
            "multi_BA": timeit(multi(B, A)),
            "multi_AA'": timeit(multi(A, A[1:] + A[:1])),
            "multi_BB'": timeit(multi(B, B[1:] + B[:1])),
            "single_A_again": timeit(single(A)),
            "multi_AB_status": timeit(multi(A, B, True)),
        }
        for b in B:  # checksums stored in place, as bench's rx batches
            batch.ipv4_fill(b, native.FILL_IP | native.FILL_L4)
        torch.cuda.synchronize()
        res["multi_AB_status_filled"] = timeit(multi(A, B, True))
        res["single_B_filled"] = timeit(single(B))
        print(json.dumps({"kind": kind, "n": A[0].n, "bytes": A[0].bytes_len, "us": res}), flush=True)
        del A, B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
