"""bench.py's JSON line carries every field the driver contract names
(metric, value, unit, n_gpus, steps, warmup, ms_per_step, higher_is_better,
scaling, vs_baseline, dtype, data, config), plus `roofline` (bound, achieved,
peak, unit, frac, traffic) and `cpu_baseline` (value, unit, cores, kind,
sample) — checked on the CPU with the bench's own builders, a small frame
sample for the oracle leg and synthetic launch timings."""
import argparse
import importlib.util
import io
import json
import os
import sys
from contextlib import redirect_stdout
from types import SimpleNamespace

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["bench_under_test"] = mod
    spec.loader.exec_module(mod)
    return mod


def test_bench_line_has_the_contract_fields():
    bench = _bench()
    bench._imports()  # bench imports numpy / torch / the package lazily (the launcher parent never does)
    frame = bench.FRAME
    n = 512
    rng = np.random.default_rng(5)
    data = torch.from_numpy(rng.integers(0, 256, size=n * frame, dtype=np.uint8))
    cpu = bench.cpu_baseline(SimpleNamespace(n=n, data=data), 0.2)
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    assert cpu["kind"] in ("port", "reference") and cpu["value"] > 0 and cpu["cores"] >= 1
    # one thread per physical core (pinned), the host's physical cores and the all-cores figure
    assert cpu["physical_cores"]["host"] >= cpu["cores"] and cpu["value_all_cores"] >= cpu["value"] * 0.99
    assert cpu["scaling_GiBps"]["1"] == cpu["value_1core"] and cpu["pinned_cpus"]
    assert cpu["physical_cores"]["l3_domains_host"] >= 1 and "one_l3_domain" in cpu
    args = argparse.Namespace(pmc=None, steps=200, warmup=5)
    alg = 3_176_136_704
    roof = bench.roofline(alg, 460e-6, "udp1500", "csum_flat_kernel<16, true, false, false, false>",
                          {"kernel": "csum_flat_kernel<16, true, false, false, false>", "skip": 9, "count": 200}, args)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == bench.HBM_PEAK_GBPS
    assert abs(roof["frac"] - alg / 460e-6 / 1e9 / bench.HBM_PEAK_GBPS) < 1e-3
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.emit("GiB/s test", 6300.0, "GiB/s", args, 1, 0.092, "u8", {"workload": "cfg2"}, roof, cpu)
    line = json.loads(buf.getvalue().strip())
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 200 and line["scaling"] == "weak"
    assert line["config"]["workload"] == "cfg2" and line["data"] == "synthetic"


def test_e2e_line_names_the_slowest_rank():
    """cfg 5 (--config e2e) at N ranks: per rank H2D / D2H rates and its NUMA
    node; the line carries the sum over ranks and names the slowest rank
    (VERDICT r03 item 7), built here from synthetic per-rank figures."""
    bench = _bench()
    bench._imports()
    h2d, d2h = bench.e2e_pcie_bytes(1 << 20, bench.native.GATHER_STRIDED)
    assert h2d == (1 << 20) * (bench.FRAME + 12) and d2h == (1 << 20) * 4
    assert bench.e2e_pcie_bytes(8, bench.native.GATHER_NONE)[0] == 8 * (2304 + 12)
    ranks = [{"rank": r, "device": r, "pci_bus_id": f"0000:{r:02x}:00.0", "numa_node": r // 4,
              "variants": {"C_strided_dma": {"GiBps_packet_bytes": 48.0 - (r == 5) * 9, "ms_per_batch": 30.0,
                                             "h2d_GBps": 52.5 - (r == 5) * 10, "d2h_GBps": 0.14}}}
             for r in range(8)]
    s = bench.e2e_ranks_summary(ranks, "C_strided_dma")
    assert s["slowest_rank"]["rank"] == 5 and s["slowest_rank"]["numa_node"] == 1
    assert s["slowest_rank"]["pci_bus_id"] == "0000:05:00.0"
    assert abs(s["sum_over_ranks_GiBps"] - (8 * 48 - 9)) < 1e-6 and len(s["per_rank_h2d_GBps"]) == 8
    assert abs(s["sum_h2d_GBps"] - (8 * 52.5 - 10)) < 1e-6
    # the whole line, as test_bench_launcher's GPU test checks the real one
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_bench_launcher import check_e2e_line

    for r in ranks:
        r.update(cpus="0-7", pool_pages_by_node={"1": 512})
        r["variants"]["C_strided_dma"]["GiBps_packet_bytes"] = float(r["variants"]["C_strided_dma"]["GiBps_packet_bytes"])
    check_e2e_line({"n_gpus": 8, "best_variant": "C_strided_dma", "variants": {"C_strided_dma": {}}, "per_rank": ranks,
                    "ranks_summary": s}, 8)


def test_flat_kernel_names_follow_the_library_choice():
    """bench.py names the flat-kernel instantiation rocprofv3 will report,
    which selects the timed dispatches from a trace: U = 16 for launches of
    512 Ki+ packets and 256 MiB+, else U = 8 with a chunk in flight, whose
    late-claim form (PLATE) the library picks for 1 KiB+ packets in 256 MiB+
    (sccsum.hip launch_flat_variant)."""
    bench = _bench()
    mi, kb = 1 << 20, 1 << 10
    assert bench.flat_kernel(True, False, 2 * mi, 2 * mi * 1500) == "csum_flat_kernel<16, true, false, false, false>"
    assert bench.flat_kernel(True, True, mi, mi * 1500) == "csum_flat_kernel<16, true, true, false, false>"
    assert bench.flat_kernel(False, False, 2 * mi, 2 * mi * 65536) == "csum_flat_kernel<16, false, false, false, false>"
    # small launches: 2 x 131 072 x 1500 B (393 MB) late, Zipf and 196 MB batches read back at once
    assert bench.flat_kernel(True, False, 256 * kb, 256 * kb * 1500) == "csum_flat_kernel<8, true, false, true, true>"
    assert bench.flat_kernel(True, False, 128 * kb, 128 * kb * 1500) == "csum_flat_kernel<8, true, false, true, false>"
    assert bench.flat_kernel(True, False, 262144, 262144 * 442) == "csum_flat_kernel<8, true, false, true, false>"
    assert bench.flat_kernel(True, True, 256 * kb, 256 * kb * 1500) == "csum_flat_kernel<8, true, true, true, true>"


def test_layout_traffic_of_aligned_frames():
    """cfg 3 (ii) (--align 64) lines carry roofline.layout_traffic: the gap
    bytes between 64 B-aligned frames, their share of the packet bytes, the
    traffic ratio they add to the algorithmic bytes and frac x ratio, the
    rate per streamed byte (74.9 % at 1.08x traffic is
    the packed layout's rate, not kernel loss)."""
    bench = _bench()
    alg, gap, packets = 1.557e9, 116_000_000, 1_503_052_521
    d = bench.layout_traffic(alg, gap, packets, 0.749)
    assert d["gap_bytes"] == gap and abs(d["gap_per_packet_byte"] - gap / packets) < 1e-5
    assert abs(d["traffic_ratio"] - (alg + gap) / alg) < 1e-5
    assert abs(d["frac_of_streamed_bytes"] - 0.749 * (alg + gap) / alg) < 1e-4
    assert bench.layout_traffic(alg, 0, packets, 0.8)["traffic_ratio"] == 1.0  # packed: no gaps
