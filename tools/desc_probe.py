"""PCIe read rate of the zero-copy paths, kernel alone (no burst queue):
the fragment-list kernel (sccsum_ipv4_frames_desc) and the gather kernel
(sccsum_gather) reading packets from a pinned host pool, against one
contiguous hipMemcpyAsync DMA of the same byte count.  Layouts: packets back
to back ("packed"), or one per 2304-byte mbuf slot at +256 ("slots",
dpdk.cc:139-156), or slots of a small pool reused round robin, or the slots copied to HBM; fixed 1500 B
or random 28..1500 B frames.  Pinned memory is cached by the GPU's L2s, so
every timed run follows a 256 MiB device read that evicts them.

usage: python tools/desc_probe.py [packets] [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seastar_amd import batch, native, pipeline, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = native.load()
    native.check(lib.sccsum_init(0), "sccsum_init")
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream()
    rng = np.random.default_rng(5)
    flush = torch.ones(64 << 20, dtype=torch.float32, device=dev)
    for lens_kind in ("1500", "rand"):
        lens = np.full(n, 1500, np.uint32) if lens_kind == "1500" else rng.integers(28, 1501, n).astype(np.uint32)
        frames = synth.udp_ipv4_frames(min(n, 4096), 1500, seed=9)[0].reshape(-1, 1500)
        for layout in ("packed", "slots", "slots_small_pool", "slots_in_hbm"):
            if layout in ("packed",):
                src_off = np.zeros(n, np.uint64)
                src_off[1:] = np.cumsum(((lens.astype(np.uint64) + 15) // 16) * 16)[:-1]
                pool_len = int(src_off[-1]) + 1600
            elif layout in ("slots", "slots_in_hbm"):
                src_off = np.arange(n, dtype=np.uint64) * 2304 + 256
                pool_len = n * 2304 + 64
            else:  # 2048 slots reused round robin (a 4.7 MB pool)
                src_off = (np.arange(n, dtype=np.uint64) % 2048) * 2304 + 256
                pool_len = 2048 * 2304 + 64
            pool = pipeline.pinned_empty(pool_len)
            for i in range(n):  # valid headers everywhere: the frames kernel reads each whole L4 range
                pool[int(src_off[i]):int(src_off[i]) + int(lens[i])] = frames[i % frames.shape[0], :lens[i]]
            base = pool.ctypes.data
            if layout == "slots_in_hbm":  # the same slots in device memory: the kernels' HBM rate
                dpool = torch.from_numpy(np.asarray(pool)).to(dev)
                base = dpool.data_ptr()
            lay = np.zeros(n, np.uint64)
            lay[1:] = np.cumsum(((lens.astype(np.uint64) + 15) // 16) * 16)[:-1]
            desc = batch.make_desc(base + src_off, lay, lens)
            first = np.arange(n + 1, dtype=np.int32)
            d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
            d_first = torch.from_numpy(first).to(dev)
            d_off = torch.from_numpy(lay.view(np.int64)).to(dev)
            d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
            out = torch.empty(2 * n, dtype=torch.int16, device=dev)
            dst = torch.empty(int(lay[-1]) + 1600, dtype=torch.uint8, device=dev)
            nbytes = int(lens.sum())
            contig = pipeline.pinned_empty(nbytes)
            dcont = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            tsrc = torch.from_numpy(contig)

            def fused():
                batch.ipv4_frames_desc(d_desc, d_first, d_off, d_len, 1500, out2=out, stream=s)

            def gather():
                native.check(lib.sccsum_gather(d_desc.data_ptr(), n, dst.data_ptr(), s.cuda_stream), "gather")

            def dma():
                with torch.cuda.stream(s):
                    dcont.copy_(tsrc, non_blocking=True)

            row = []
            for name, fn in (("fused", fused), ("gather", gather), ("dma", dma)):
                for _ in range(3):
                    fn()
                tot = 0.0
                for _ in range(reps):
                    # evict the L2s between timed runs (pinned memory is cached by the GPU): read 256 MiB
                    with torch.cuda.stream(s):
                        flush.sum()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    fn()
                    e1.record(s)
                    e1.synchronize()
                    tot += e0.elapsed_time(e1) * 1e3
                us = tot / reps
                row.append(f"{name} {nbytes / us / 1e3:6.1f} GB/s ({us:7.1f} us)")
            print(f"{lens_kind:>4} {layout:>16} n={n}: " + "   ".join(row), flush=True)


if __name__ == "__main__":
    main()
