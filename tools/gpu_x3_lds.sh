#!/bin/bash
# LDS-pressure and issue-mix PMC of the two 3xbf16 field kernels: per format, one pass of LDS
# counters and one of MFMA busy + clock over the C2-sized field launch (tools/field_timing.py).
#   tools/gpu_x3_lds.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-x3lds}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in ${X3_FORMATS:-bf16x3 bf16x3_w16 f32_w16}; do
  for c in "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY"; do
    tag=$(echo $c | cut -d' ' -f1-2 | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "field_" -d $O/${p}_$tag -o run --output-format csv -- python $R/tools/field_timing.py --precision $p --iters 5 > $O/${p}_$tag.log 2>&1
    rc=$?; echo "$p $tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/${p}_$tag.log; exit $rc; }
  done
  python $R/tools/pmc_kernels.py $O/${p}_SQ_INSTS_LDS_SQ_LDS_IDX_ACTIVE > $O/$p.txt
  python $R/tools/pmc_kernels.py $O/${p}_SQ_VALU_MFMA_BUSY_CYCLES_GRBM_GUI_ACTIVE >> $O/$p.txt
  python $R/tools/pmc_kernels.py $O/${p}_SQ_INSTS_VALU_SQ_ACTIVE_INST_VALU >> $O/$p.txt
  echo "== $p"; cat $O/$p.txt
done
