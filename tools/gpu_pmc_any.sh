#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over any timing tool, for the kernels matching
# a regex, summarised by pmc_kernels.py.
#   tools/gpu_pmc_any.sh <tag> <kernel-regex> <tool.py> [tool args...]
R=$GRAFT_REPO_ROOT
TAG=$1; RX=$2; TOOL=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"}
IFS='|' read -ra PASS_LIST <<< "$PASSES"
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "$RX" -d $O/pmc_$tag -o run --output-format csv -- python $R/tools/$TOOL "$@" > $O/pmc_$tag.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$tag.log; exit $rc; }
done
python $R/tools/pmc_kernels.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
