"""NUMA locality of a shard and its GPU.

Seastar pins each shard's reactor thread to one core (smp::pin,
src/core/reactor.cc:4163) and binds the shard's memory to that core's NUMA
node (src/core/memory.cc:1898-1951).  The batch path adds a GPU per shard, so
the locality that matters is the GPU's: a rank (or shard thread) that drives
device d runs on d's node's cores and allocates its host memory — the pinned
mbuf pool of cfg 5, burst staging, the CPU baseline's buffers — on d's node,
so that its DMA does not cross the socket link.

Everything here is sysfs + two syscalls (sched_setaffinity for every thread of
the process, set_mempolicy for the calling thread); nothing touches HIP.  The
sysfs root is a parameter so the mapping is testable on a fake tree
(tests/test_numa.py).
"""
from __future__ import annotations

import ctypes
import os
import platform

SYSFS = "/sys"

MPOL_PREFERRED = 1
MPOL_BIND = 2
_MAXNODE = 1024  # bits in the node masks passed to the kernel
# x86-64 syscall numbers (arch/x86/entry/syscalls/syscall_64.tbl)
_SYS = {"x86_64": {"set_mempolicy": 238, "get_mempolicy": 239, "move_pages": 279}}


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out: list[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.extend(range(int(lo), int(hi) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpulist(cpus) -> str:
    """[0, 1, 2, 3, 8, 10, 11] -> '0-3,8,10-11'."""
    cpus = sorted(set(int(c) for c in cpus))
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(runs)


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def normalize_bdf(bdf: str) -> str:
    """'0000:05:00.0' in sysfs's lower-case form (HIP prints upper case hex)."""
    bdf = bdf.strip().lower()
    if bdf.count(":") == 1:  # bus:dev.fn without the domain
        bdf = "0000:" + bdf
    return bdf


def pci_numa_node(bdf: str, sysfs: str = SYSFS) -> int:
    """The NUMA node sysfs reports for a PCI device, -1 if none (a one-node
    host, or firmware that does not say)."""
    v = _read(os.path.join(sysfs, "bus", "pci", "devices", normalize_bdf(bdf), "numa_node"))
    try:
        return int(v) if v is not None else -1
    except ValueError:
        return -1


def node_cpus(node: int, sysfs: str = SYSFS) -> list[int]:
    v = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    return parse_cpulist(v) if v else []


def online_nodes(sysfs: str = SYSFS) -> list[int]:
    v = _read(os.path.join(sysfs, "devices", "system", "node", "online"))
    return parse_cpulist(v) if v else []


def cpu_node(cpu: int, sysfs: str = SYSFS) -> int:
    for n in online_nodes(sysfs):
        if cpu in node_cpus(n, sysfs):
            return n
    return -1


def physical_cores(cpus, sysfs: str = SYSFS) -> list[int]:
    """One CPU per physical core among `cpus` (the first hardware thread of
    each (package, core) pair, from the topology files), in CPU order.  A CPU
    without topology files counts as its own core."""
    seen, out = set(), []
    for c in sorted(set(cpus)):
        base = os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology")
        pkg, core = _read(os.path.join(base, "physical_package_id")), _read(os.path.join(base, "core_id"))
        key = (pkg, core) if pkg is not None and core is not None else ("cpu", c)
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def l3_domain(cpu: int, sysfs: str = SYSFS) -> str:
    """The CPUs sharing `cpu`'s last-level (L3) cache, as a cpulist string —
    on EPYC one CCD, whose link to memory caps what its cores stream
    together.  A CPU without cache files is its own domain."""
    base = os.path.join(sysfs, "devices", "system", "cpu", f"cpu{cpu}", "cache")
    for idx in range(8):
        lvl = _read(os.path.join(base, f"index{idx}", "level"))
        if lvl == "3":
            shared = _read(os.path.join(base, f"index{idx}", "shared_cpu_list"))
            if shared:
                return format_cpulist(parse_cpulist(shared))
    return str(cpu)


def spread_over_l3(cores, sysfs: str = SYSFS) -> list[int]:
    """`cores` reordered round robin over their L3 domains (first core of
    each domain, then the second of each, ...), so k threads pinned to the
    first k use as many domains — and their memory links — as they can."""
    groups: dict[str, list[int]] = {}
    for c in cores:
        groups.setdefault(l3_domain(c, sysfs), []).append(c)
    out, lists = [], list(groups.values())
    for i in range(max((len(g) for g in lists), default=0)):
        out.extend(g[i] for g in lists if i < len(g))
    return out


def l3_domains(cpus, sysfs: str = SYSFS) -> dict[str, list[int]]:
    groups: dict[str, list[int]] = {}
    for c in sorted(set(cpus)):
        groups.setdefault(l3_domain(c, sysfs), []).append(c)
    return groups


def host_physical_cores(sysfs: str = SYSFS) -> int:
    """Physical cores of the whole host (every online CPU's (package, core))."""
    v = _read(os.path.join(sysfs, "devices", "system", "cpu", "online"))
    return len(physical_cores(parse_cpulist(v), sysfs)) if v else 0


def host_l3_domains(sysfs: str = SYSFS) -> int:
    """L3 domains (CCDs) of the whole host."""
    v = _read(os.path.join(sysfs, "devices", "system", "cpu", "online"))
    return len(l3_domains(parse_cpulist(v), sysfs)) if v else 0


def plan(bdf: str | None, allowed=None, sysfs: str = SYSFS) -> dict:
    """Where a rank driving the PCI device `bdf` should run: its NUMA node and
    the schedulable CPUs on that node.  Falls back to the current CPU set (and
    says why) when the device has no node or none of the node's CPUs is
    schedulable here (a cgroup's cpuset)."""
    allowed = sorted(os.sched_getaffinity(0) if allowed is None else set(allowed))
    node = pci_numa_node(bdf, sysfs) if bdf else -1
    p = {"pci_bus_id": normalize_bdf(bdf) if bdf else None, "numa_node": node, "cpus": allowed, "bound": False,
         "reason": None}
    if node < 0:
        p["reason"] = "the device reports no NUMA node"
        return p
    local = sorted(set(node_cpus(node, sysfs)) & set(allowed))
    if not local:
        p["reason"] = f"none of node {node}'s CPUs is schedulable here"
        return p
    p["cpus"] = local
    p["bound"] = True
    return p


def _libc():
    return ctypes.CDLL(None, use_errno=True)


def _syscall_no(name: str) -> int | None:
    return _SYS.get(platform.machine(), {}).get(name)


def _nodemask(nodes) -> ctypes.Array:
    mask = (ctypes.c_ulong * (_MAXNODE // 64))()
    for n in nodes:
        mask[n // 64] |= 1 << (n % 64)
    return mask


def set_mempolicy(mode: int, nodes) -> None:
    """set_mempolicy(2) for the calling thread (and the threads it creates
    from now on).  Raises OSError on failure (e.g. a node outside the
    cgroup's cpuset.mems)."""
    no = _syscall_no("set_mempolicy")
    if no is None:
        raise OSError(f"set_mempolicy: unsupported architecture {platform.machine()}")
    mask = _nodemask(nodes)
    if _libc().syscall(no, ctypes.c_int(mode), mask, ctypes.c_ulong(_MAXNODE + 1)) != 0:
        e = ctypes.get_errno()
        raise OSError(e, f"set_mempolicy: {os.strerror(e)}")


def get_mempolicy() -> tuple[int, list[int]]:
    """The calling thread's (mode, nodes)."""
    no = _syscall_no("get_mempolicy")
    if no is None:
        raise OSError(f"get_mempolicy: unsupported architecture {platform.machine()}")
    mode = ctypes.c_int(0)
    mask = (ctypes.c_ulong * (_MAXNODE // 64))()
    if _libc().syscall(no, ctypes.byref(mode), mask, ctypes.c_ulong(_MAXNODE + 1), None, ctypes.c_ulong(0)) != 0:
        e = ctypes.get_errno()
        raise OSError(e, f"get_mempolicy: {os.strerror(e)}")
    return mode.value, [i for i in range(_MAXNODE) if mask[i // 64] >> (i % 64) & 1]


def page_nodes(addr: int, nbytes: int, samples: int = 1024) -> dict[int, int]:
    """Where the pages of [addr, addr + nbytes) live: {node: pages} over up to
    `samples` pages spread over the range (move_pages(2) in query mode; a
    negative key is an errno, e.g. -14 for a page not yet touched)."""
    no = _syscall_no("move_pages")
    if no is None or nbytes <= 0:
        return {}
    page = os.sysconf("SC_PAGE_SIZE")
    first, last = addr // page, (addr + nbytes - 1) // page
    total = last - first + 1
    k = min(samples, total)
    idx = sorted({first + (i * total) // k for i in range(k)})
    pages = (ctypes.c_void_p * len(idx))(*[p * page for p in idx])
    status = (ctypes.c_int * len(idx))()
    if _libc().syscall(no, ctypes.c_int(0), ctypes.c_ulong(len(idx)), pages, None, status, ctypes.c_int(0)) != 0:
        return {}
    hist: dict[int, int] = {}
    for s in status:
        hist[int(s)] = hist.get(int(s), 0) + 1
    return hist


def bind(p: dict, mem: str = "bind") -> dict:
    """Apply a plan(): every thread of this process onto p["cpus"]
    (sched_setaffinity per task: HIP's and torch's helper threads too, not
    only the caller), and the calling thread's memory policy onto the node
    (mem = "bind": MPOL_BIND, "preferred": MPOL_PREFERRED, "none": leave it).
    Returns what was done; never raises — a refused step is reported."""
    done = {"numa_node": p["numa_node"], "cpus": format_cpulist(p["cpus"]), "ncpus": len(p["cpus"]),
            "affinity": "unchanged", "mempolicy": "default", "reason": p.get("reason")}
    if not p.get("bound"):
        return done
    cpus = set(p["cpus"])
    moved, failed = 0, 0
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
            moved += 1
        except OSError:  # a thread that exited meanwhile
            failed += 1
    done["affinity"] = f"{moved} threads on node {p['numa_node']}" + (f" ({failed} gone)" if failed else "")
    if mem != "none":
        mode = MPOL_BIND if mem == "bind" else MPOL_PREFERRED
        try:
            set_mempolicy(mode, [p["numa_node"]])
            done["mempolicy"] = f"{'MPOL_BIND' if mode == MPOL_BIND else 'MPOL_PREFERRED'} node {p['numa_node']}"
        except OSError as e:
            done["mempolicy"] = f"refused ({e})"
    return done
