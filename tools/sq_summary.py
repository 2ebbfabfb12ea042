"""Per-kernel SQ counter summary of rocprofv3 SQ_* / GRBM_* passes (means over dispatches; round 1-2, the sq_profile.sh runner is in git history)."""
import collections
import csv
import re
import glob
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sccsum" not in r["Kernel_Name"]:
            continue
        m = re.search(r"(csum_\w+<[^>]*>|read_probe_kernel)", r["Kernel_Name"])
        key = (m.group(1) if m else r["Kernel_Name"][:60]) + " grid=" + r.get("Grid_Size", "?")
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c, v in sorted(m.items()):
        print(f"   {c:24s} {v:16.0f}  (n={len(cs[c])})")
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        w = m["SQ_WAVE_CYCLES"]
        print("   shares of wave-cycles: wait(s_waitcnt/barrier) %.2f  issue-stall %.2f  active %.2f" % (
            m.get("SQ_WAIT_ANY", 0) / w, m.get("SQ_WAIT_INST_ANY", 0) / w, m.get("SQ_ACTIVE_INST_ANY", 0) / w))
