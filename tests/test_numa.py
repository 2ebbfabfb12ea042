"""Rank / shard locality (seastar_amd/numa.py): the PCI bus id -> NUMA node ->
cpulist mapping on a fake sysfs tree, thread affinity and the memory policy
in a child process, and bench.py's ranks bound to their (stand-in) GPUs'
nodes.  Reference: Seastar pins a shard's thread to its core and binds its
memory to the core's node (src/core/reactor.cc:4163, src/core/memory.cc:1898-1951)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from seastar_amd import numa  # noqa: E402

GPU0, GPU1, GPU_NONODE = "0000:05:00.0", "0000:85:00.0", "0000:c1:00.0"


def fake_sysfs(root) -> str:
    """Two nodes: node 0 = CPUs 0-3, node 1 = CPUs 4-7, SMT pairs (0,1) (2,3)
    (4,5) (6,7) on one core each; GPU0 on node 0, GPU1 on node 1, GPU_NONODE
    without a node (-1)."""
    def put(path, text):
        p = os.path.join(root, path)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text + "\n")

    put("devices/system/node/online", "0-1")
    put("devices/system/node/node0/cpulist", "0-3")
    put("devices/system/node/node1/cpulist", "4-7")
    put("devices/system/cpu/online", "0-7")
    for c in range(8):
        put(f"devices/system/cpu/cpu{c}/topology/physical_package_id", str(c // 4))
        put(f"devices/system/cpu/cpu{c}/topology/core_id", str((c % 4) // 2))
        put(f"devices/system/cpu/cpu{c}/cache/index0/level", "1")  # L1, L2 per core; L3 per package
        put(f"devices/system/cpu/cpu{c}/cache/index0/shared_cpu_list", f"{c // 2 * 2}-{c // 2 * 2 + 1}")
        put(f"devices/system/cpu/cpu{c}/cache/index2/level", "2")
        put(f"devices/system/cpu/cpu{c}/cache/index2/shared_cpu_list", f"{c // 2 * 2}-{c // 2 * 2 + 1}")
        put(f"devices/system/cpu/cpu{c}/cache/index3/level", "3")
        put(f"devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", "0-3" if c < 4 else "4-7")
    put(f"bus/pci/devices/{GPU0}/numa_node", "0")
    put(f"bus/pci/devices/{GPU1}/numa_node", "1")
    put(f"bus/pci/devices/{GPU_NONODE}/numa_node", "-1")
    return str(root)


def test_cpulist_round_trip():
    assert numa.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.parse_cpulist(" 5 ") == [5] and numa.parse_cpulist("") == []
    assert numa.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert numa.format_cpulist([]) == ""
    for s in ("0-255", "0,2,4", "1-2,4-5,7"):
        assert numa.format_cpulist(numa.parse_cpulist(s)) == s


def test_bdf_to_node_to_cpus(tmp_path):
    fs = fake_sysfs(tmp_path)
    assert numa.pci_numa_node(GPU0, fs) == 0 and numa.pci_numa_node(GPU1, fs) == 1
    assert numa.pci_numa_node("0000:85:00.0".upper(), fs) == 1  # HIP prints upper-case hex
    assert numa.pci_numa_node("85:00.0", fs) == 1  # no domain
    assert numa.pci_numa_node(GPU_NONODE, fs) == -1 and numa.pci_numa_node("0000:01:00.0", fs) == -1
    assert numa.online_nodes(fs) == [0, 1] and numa.node_cpus(1, fs) == [4, 5, 6, 7]
    assert numa.cpu_node(6, fs) == 1 and numa.cpu_node(9, fs) == -1
    assert numa.physical_cores(range(8), fs) == [0, 2, 4, 6]
    assert numa.physical_cores([1, 3, 5], fs) == [1, 3, 5] and numa.host_physical_cores(fs) == 4
    # L3 domains (CCDs): cores round robin over them, so k pinned threads use min(k, domains) links
    assert numa.l3_domain(2, fs) == "0-3" and numa.l3_domain(9, fs) == "9"
    assert numa.spread_over_l3([0, 2, 4, 6], fs) == [0, 4, 2, 6]
    assert numa.l3_domains([0, 2, 4, 6], fs) == {"0-3": [0, 2], "4-7": [4, 6]} and numa.host_l3_domains(fs) == 2

    p = numa.plan(GPU1, allowed=range(8), sysfs=fs)
    assert p["bound"] and p["numa_node"] == 1 and p["cpus"] == [4, 5, 6, 7]
    p = numa.plan(GPU1, allowed=[0, 1, 5], sysfs=fs)  # a cpuset: only the node's schedulable CPUs
    assert p["cpus"] == [5]
    p = numa.plan(GPU1, allowed=[0, 1], sysfs=fs)  # none of them schedulable: stay, and say why
    assert not p["bound"] and p["cpus"] == [0, 1] and "schedulable" in p["reason"]
    p = numa.plan(GPU_NONODE, allowed=range(8), sysfs=fs)
    assert not p["bound"] and p["numa_node"] == -1 and "no NUMA node" in p["reason"]
    assert not numa.plan(None, allowed=[3], sysfs=fs)["bound"]


CHILD = r"""
import json, os, sys, threading
sys.path.insert(0, sys.argv[1])
from seastar_amd import numa
import numpy as np
helper = threading.Thread(target=lambda: __import__("time").sleep(2)); helper.start()
cpus = sorted(os.sched_getaffinity(0))
node = numa.cpu_node(cpus[0])
p = {"numa_node": node, "cpus": cpus[:1], "bound": True}
done = numa.bind(p, mem="bind")
a = np.ones(1 << 22, np.uint8)  # allocated and touched after the policy
helper_aff = sorted(os.sched_getaffinity(helper.native_id))
print(json.dumps({"done": done, "aff": sorted(os.sched_getaffinity(0)), "helper": helper_aff, "cpu0": cpus[0],
                  "node": node, "policy": numa.get_mempolicy(), "pages": numa.page_nodes(a.ctypes.data, a.nbytes, 64)}))
helper.join()
"""


@pytest.mark.skipif(not os.path.isdir("/sys/devices/system/node/node0"), reason="no NUMA sysfs here")
def test_bind_moves_every_thread_and_sets_the_policy():
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["aff"] == [d["cpu0"]] and d["helper"] == [d["cpu0"]]  # threads created before bind() move too
    assert d["done"]["mempolicy"] == f"MPOL_BIND node {d['node']}"
    assert d["policy"] == [numa.MPOL_BIND, [d["node"]]]
    assert set(map(int, d["pages"])) == {d["node"]}  # the pages landed on the bound node


def _dry(args, extra_env, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def test_bench_ranks_bind_to_their_gpus_nodes(tmp_path):
    """Two dry-run ranks with stand-in GPUs on nodes 0 and 1 of a fake
    sysfs: each rank's threads go to its GPU's node's schedulable CPUs, and
    per_rank reports node, CPUs, affinity and memory policy."""
    fs = fake_sysfs(tmp_path)
    allowed = sorted(os.sched_getaffinity(0))
    r = _dry(["--gpus", "2", "--dry-run"], {"SCCSUM_SYSFS": fs, "SCCSUM_DRY_RUN_BDFS": f"{GPU0},{GPU1}"})
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    pr = d["per_rank"]
    for rank, node, cpus in ((0, 0, [0, 1, 2, 3]), (1, 1, [4, 5, 6, 7])):
        want = sorted(set(cpus) & set(allowed))
        e = pr[rank]
        assert e["numa_node"] == node
        if want:
            assert e["cpus"] == numa.format_cpulist(want) and e["affinity"].endswith(f"on node {node}")
            # node 1 may not exist on this host: the policy is then refused and reported, never fatal
            assert e["mempolicy"] == f"MPOL_BIND node {node}" or e["mempolicy"].startswith("refused")
        else:
            assert e["affinity"] == "unchanged"


def test_bench_refuses_more_ranks_than_devices(tmp_path):
    env = {"SCCSUM_DRY_RUN_NDEV": "2"}
    r = _dry(["--gpus", "3", "--dry-run"], env)
    assert r.returncode != 0 and "--share-devices" in (r.stdout + r.stderr)
    r = _dry(["--gpus", "3", "--dry-run", "--share-devices", "--numa", "off"], env)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert d["n_gpus"] == 3 and all(e["affinity"].startswith("unchanged") for e in d["per_rank"])


@pytest.mark.gpu
def test_device_numa_node_matches_sysfs():
    """sccsum_device_numa_node (the C-ABI's answer for C++ shards) agrees with
    the sysfs node of the PCI address torch reports for the same device."""
    import ctypes

    import torch

    from seastar_amd import native

    lib = native.load()
    p = torch.cuda.get_device_properties(0)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    node = ctypes.c_int(-7)
    native.check(lib.sccsum_device_numa_node(0, ctypes.byref(node)), "sccsum_device_numa_node")
    assert node.value == numa.pci_numa_node(bdf)
    assert lib.sccsum_device_numa_node(0, None) == native.SCCSUM_EINVAL
    assert lib.sccsum_device_numa_node(10_000, ctypes.byref(node)) == native.SCCSUM_ENODEV
    print(f"device 0 {bdf}: NUMA node {node.value}")
