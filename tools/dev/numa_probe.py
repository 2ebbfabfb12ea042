"""Where pinned host memory lands: for the calling
thread's memory policy (none / MPOL_BIND to the GPU's node / MPOL_BIND to
another node) and hipHostMalloc flags (Default / NumaUser), allocate 64 MiB,
and report the pages' NUMA nodes (move_pages query), plus the same for a
pageable numpy buffer (first touch).  One JSON line per case.

    python tools/dev/numa_probe.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from seastar_amd import numa  # noqa: E402

MB64 = 64 << 20
NUMA_USER = 0x20000000  # hipHostMallocNumaUser (hip_runtime_api.h)


def main():
    torch.cuda.set_device(0)
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    node = numa.pci_numa_node(bdf)
    nodes = numa.online_nodes()
    other = next((n for n in nodes if n != node), None)
    print(json.dumps({"bdf": bdf, "gpu_node": node, "online_nodes": nodes,
                      "allowed_cpus": numa.format_cpulist(sorted(os.sched_getaffinity(0))),
                      "mems_allowed": open("/proc/self/status").read().split("Mems_allowed_list:")[1].split()[0]}),
          flush=True)
    hip = ctypes.CDLL("libamdhip64.so")
    policies = [("default", None)] + ([("bind_gpu_node", node)] if node >= 0 else []) + \
               ([("bind_other_node", other)] if other is not None else [])
    for pname, pnode in policies:
        try:
            if pnode is None:
                numa.set_mempolicy(0, [])
            else:
                numa.set_mempolicy(numa.MPOL_BIND, [pnode])
        except OSError as e:
            print(json.dumps({"policy": pname, "error": str(e)}), flush=True)
            continue
        for fname, flags in (("hipHostMallocDefault", 0), ("hipHostMallocNumaUser", NUMA_USER)):
            ptr = ctypes.c_void_p()
            rc = hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(MB64), ctypes.c_uint(flags))
            hist = numa.page_nodes(ptr.value, MB64, 256) if rc == 0 else None
            if rc == 0:
                hip.hipHostFree(ptr)
            print(json.dumps({"policy": pname, "alloc": fname, "rc": rc, "pages_by_node": hist}), flush=True)
        t = torch.empty(MB64, dtype=torch.uint8, pin_memory=True)
        print(json.dumps({"policy": pname, "alloc": "torch pin_memory",
                          "pages_by_node": numa.page_nodes(t.data_ptr(), MB64, 256)}), flush=True)
        del t
        a = np.ones(MB64, np.uint8)
        print(json.dumps({"policy": pname, "alloc": "numpy (first touch)",
                          "pages_by_node": numa.page_nodes(a.ctypes.data, MB64, 256)}), flush=True)
    numa.set_mempolicy(0, [])


if __name__ == "__main__":
    main()
