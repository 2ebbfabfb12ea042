"""Quick look at a rocprofv3 FETCH_SIZE pass: mean MB per dispatch for every
kernel name (x 2048 = KiB x 1024 x 2, the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md).  For the committed per-launch figures use
tools/prof_timed.py, which cuts the timed dispatches.

usage: python tools/pmc_by_name.py DIR   (a rocprofv3 -d output directory)
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
v = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[(r["Kernel_Name"][:110], r["Grid_Size"] if "Grid_Size" in r else "")].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(f"{sum(x) / len(x) * 2048 / 1e6:10.1f} MB  n={len(x):3d}  {k[0]}")
