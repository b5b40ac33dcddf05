#!/bin/bash
# WRITE_SIZE of the store shapes in tools/write_probe.hip (one rocprofv3 pass), summarised per kernel.
R=$GRAFT_REPO_ROOT; TAG=${1:-wp}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/bin/write_probe > $O/write_probe.txt 2>&1; echo "plain rc=$?"; cat $O/write_probe.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_w -o run --output-format csv -- $R/tools/bin/write_probe > $O/pmc_w.log 2>&1
echo "pmc rc=$?"
python3 - "$O/pmc_w" <<'PY'
import csv, glob, sys, collections
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(list)
for r in rows:
    if r["Counter_Name"] == "WRITE_SIZE":
        agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:60s} launches {len(v)}  WRITE_SIZE/launch {sum(v)/len(v)/1024/1024:.4f} GiB (of 2 GiB)")
PY
