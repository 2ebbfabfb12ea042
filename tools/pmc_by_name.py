import csv,glob,sys,collections
d=sys.argv[1]
v=collections.defaultdict(list)
for f in glob.glob(d+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        v[(r["Kernel_Name"][:110], r["Grid_Size"] if "Grid_Size" in r else "")].append(float(r["Counter_Value"]))
for k,x in sorted(v.items()):
    print(f"{sum(x)/len(x)*2048/1e6:10.1f} MB  n={len(x):3d}  {k[0]}")
