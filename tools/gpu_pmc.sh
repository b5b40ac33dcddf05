#!/bin/bash
# PMC passes for one field kernel (one counter group per rocprofv3 run, each under its own time limit):
# HBM bytes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM/rocprofv3 recipe), MFMA busy cycles + clock,
# wave-state split.   usage: tools/gpu_pmc.sh <tag> <kernel-regex> [bench precision]
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
KRE=${2:-field_w16}
PREC=${3:-f32}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
IFS='|' read -ra PASS_LIST <<< "$PASSES"
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex $KRE -d $O/$tag -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --precision $PREC > $O/pmc_$tag.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$tag.log; exit $rc; }
done
find $O -name "*counter_collection.csv"
python $R/tools/pmc_summary.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
