#!/bin/bash
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex field_x3 -d $R/gpurun_out/pmc2/p$i -o run --output-format csv -- python $R/tools/field_timing.py --iters 3 > $R/gpurun_out/pmc2/p$i.log 2>&1
  rc=$?; echo "$c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc2/p$i.log; exit $rc; fi
done
