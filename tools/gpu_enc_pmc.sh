#!/bin/bash
# PMC passes over the C3 training iteration restricted to the encoding dW kernel:
# MFMA busy, instruction mix, wait states, LDS.   tools/gpu_enc_pmc.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-encpmc}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS|SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE|FETCH_SIZE"}
IFS='|' read -ra PASS_LIST <<< "$PASSES"
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "${PMC_REGEX:-gemm_tn_enc}" -d $O/pmc_$tag -o run --output-format csv -- python $R/tools/train_timing.py --iters 2 > $O/pmc_$tag.log 2>&1
  rc=$?; echo "$c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_$tag.log; exit $rc; fi
done
python $R/tools/pmc_kernels.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
