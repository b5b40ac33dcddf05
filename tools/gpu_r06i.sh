#!/bin/bash
# round-6 PMC of the paired training kernels (C3 iteration: both fields' dX launch, the batched dW launch with
# the XENC role, layer_xyz1's shared launch, the reduction) and the C5 eval kernels: one pass per counter group.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06i}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE"
IFS='|' read -ra PASS_LIST <<< "$PASSES"
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "field_w16|gemm_tn|reduce_jobs" -d $O/train/pmc_$tag -o run --output-format csv -- python $R/tools/train_timing.py --shape c3 --iters 2 > $O/train_$tag.log 2>&1
  rc=$?; echo "train $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_$tag.log; exit $rc; }
done
python $R/tools/pmc_kernels.py $O/train > $O/pmc_train_summary.txt && cat $O/pmc_train_summary.txt
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  C5_PRECISIONS=f32 C5_GRAPH=0 C5_ITERS=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "field_w16|ray_grad" -d $O/c5/pmc_$tag -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5_$tag.log 2>&1
  rc=$?; echo "c5 $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5_$tag.log; exit $rc; }
done
python $R/tools/pmc_kernels.py $O/c5 > $O/pmc_c5_summary.txt && cat $O/pmc_c5_summary.txt
exit 0
