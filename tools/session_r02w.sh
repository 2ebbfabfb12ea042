#!/bin/bash
# two streams with split priorities: does the overlap stay at the boundary?
set -o pipefail
mkdir -p gpurun_out/prio
O=gpurun_out/prio
L=$O/ab.log
: > $L
for r in 1 2; do for a in "--streams 1" "--streams 2" "--streams 2 --stream-priority"; do
echo -n "udp1500 $a: " >> $L
timeout -k 10 300 python bench.py $a --steps 20 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $L || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/tr -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --streams 2 --stream-priority --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$O/tr.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 - <<'PY' >> $L
import csv, glob
rows = []
for f in glob.glob("gpurun_out/prio/tr/**/*kernel_trace.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "csum_flat_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows][-10:]
print("last 10 launches: durations us", [round((e - s) / 1e3, 1) for s, e in t])
print("overlap with previous us", [round((a[1] - b[0]) / 1e3, 1) for a, b in zip(t, t[1:])])
print("span per launch us", round((t[-1][1] - t[0][0]) / 1e3 / len(t), 1))
PY
cat $L
