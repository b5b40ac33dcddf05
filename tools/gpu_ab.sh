#!/bin/bash
# A/B of library variants (tools/build_variants.sh) on the training kernels: HIP-event timing of
# the field variants, then per variant one FETCH_SIZE and one MFMA-busy PMC pass.
#   VARIANTS="base PLANE_WB" tools/gpu_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export VT_RAYS=${VT_RAYS:-6144} VT_ONLY=${VT_ONLY:-fwd_masks,fwd_train,bwd_train}
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so VT_ITERS=20 timeout -k 10 120 python $R/tools/variant_timing.py f32 \
      | sed "s/^{/{\"lib\": \"$v\", \"round\": $round, /" >> $O/ab.jsonl 2>> $O/ab.err || { echo "fail $v"; tail -3 $O/ab.err; exit 1; }
  done
done
cat $O/ab.jsonl
export VT_ITERS=3
for v in ${VARIANTS:-base}; do
  for c in "FETCH_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    tag=$(echo $c | tr ' ' '_')
    CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "field_w16" -d $O/pmc_${v}_$tag -o run --output-format csv -- python $R/tools/variant_timing.py f32 > $O/pmc_${v}_$tag.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_${v}_$tag.log; exit $rc; }
  done
  python $R/tools/pmc_kernels.py $O/pmc_${v}_FETCH_SIZE > $O/pmc_${v}.txt
  python $R/tools/pmc_kernels.py $O/pmc_${v}_SQ_VALU_MFMA_BUSY_CYCLES_GRBM_GUI_ACTIVE >> $O/pmc_${v}.txt
  echo "== $v"; grep -E "^w16|FETCH|mfma_busy|clock" $O/pmc_${v}.txt
done
