"""Per-kernel SQ counter summary from tools/sq_profile.sh output (means over dispatches)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sccsum" not in r["Kernel_Name"]:
            continue
        key = r["Kernel_Name"].split("(")[0].replace("void sccsum::(anonymous namespace)::", "") + " grid=" + r.get("Grid_Size", "?")
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.0f}  (n={len(v)})")
