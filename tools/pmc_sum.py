"""Sum of every counter over all dispatches, per kernel name, from rocprofv3
--pmc passes (counter_collection.csv under each DIR): the instruction mix and
wait cycles of two bench forms that do the same work (e.g. --launch multi and
--launch engine: the same number of cfg 2 steps, warm-up included) compare
directly.  usage: python tools/pmc_sum.py DIR [DIR ...]
"""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:90]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((d, r.get("Dispatch_Id") or r.get("Correlation_Id")))
for k in sorted(tot):
    n = len(disp[k]) // max(1, len(sys.argv) - 1)
    print(f"{k}  (dispatches per pass: {n})")
    for c, v in sorted(tot[k].items()):
        print(f"    {c:28s} {v:18.0f}")
