"""Quick look at a rocprofv3 counter pass: mean MB per dispatch for every
kernel name.  FETCH_SIZE (default): x 2048 = KiB x 1024 x 2, the gfx950
correction of MI355X_MICROARCH.md for wide (16 B / lane) coalesced streaming
reads — narrower loads (a store pass's header bytes) are not doubled by the
hardware, so for those kernels the figure is an upper bound; --write:
WRITE_SIZE, x 1024.  With --trace DIR (a kernel-trace pass of the same
program) the mean duration per kernel name is printed beside it.  For the
committed per-launch figures of bench.py runs use tools/prof_timed.py, which
cuts the timed dispatches.

usage: python tools/pmc_by_name.py DIR [--write] [--trace TRACE_DIR]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
write = "--write" in sys.argv
trace = sys.argv[sys.argv.index("--trace") + 1] if "--trace" in sys.argv else None
scale = 1024 if write else 2048
dur = collections.defaultdict(list)
if trace:
    for f in glob.glob(trace + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"][:110]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
v = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"][:110]].append(float(r["Counter_Value"]))
print("WRITE_SIZE" if write else "FETCH_SIZE (x2 gfx950 correction)")
for k, x in sorted(v.items()):
    t = dur.get(k)
    ts = f"  {sum(t) / len(t):9.1f} us (n={len(t)})" if t else ""
    print(f"{sum(x) / len(x) * scale / 1e6:10.1f} MB  n={len(x):3d}{ts}  {k}")
