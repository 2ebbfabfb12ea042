"""Probe: the zero-copy gather (sccsum_gather) reading mbuf-shaped frames out
of pinned host memory over PCIe, against the copy engine moving the same
bytes, by host allocation kind.  Prints one line per case.

  python tools/gather_probe.py [frames] [frame_len]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from seastar_amd import native  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")
FLAGS = {"coherent": 0x40000000, "noncoherent": 0x80000000, "default": 0}
SLOT, DATA = 2304, 256


def host_alloc(nbytes, flags):
    p = ctypes.c_void_p()
    rc = HIP.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
    assert rc == 0, rc
    return p.value


def timed(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
    lib = native.load()
    torch.cuda.init()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    total = n * L
    dst = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
    for kind, flags in FLAGS.items():
        pool = host_alloc(n * SLOT, flags)
        ctypes.memset(pool, 0x5A, n * SLOT)
        desc = np.zeros(n, dtype=[("src", "<u8"), ("dst_off", "<u4"), ("len", "<u4")])
        desc["src"] = pool + DATA + np.arange(n, dtype=np.uint64) * SLOT
        desc["dst_off"] = np.arange(n, dtype=np.uint64) * ((L + 15) // 16 * 16)
        desc["len"] = L
        d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
        dst_big = torch.empty(int(desc["dst_off"][-1]) + L + 16, dtype=torch.uint8, device="cuda")

        def gather():
            native.check(lib.sccsum_gather(ctypes.c_void_p(d_desc.data_ptr()), n,
                                           ctypes.c_void_p(dst_big.data_ptr()), stream), "gather")

        def dma():
            rc = HIP.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(pool), ctypes.c_size_t(total),
                                    ctypes.c_int(1), stream)
            assert rc == 0, rc

        tg = timed(gather)
        td = timed(dma)
        print(f"{kind:12s} n={n} L={L}: gather {total / tg / 1e9:6.1f} GB/s ({tg * 1e6:8.1f} us)   "
              f"dma contiguous {total / td / 1e9:6.1f} GB/s", flush=True)
        HIP.hipHostFree(ctypes.c_void_p(pool))


if __name__ == "__main__":
    main()
