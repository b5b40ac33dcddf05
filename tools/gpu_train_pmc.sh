#!/bin/bash
# Training-kernel profile: kernel stats of the field variants, then one PMC pass per
# counter group over the training forward + fused training backward (each pass under its own limit).
#   tools/gpu_train_pmc.sh <tag> [precision]      (VT_ONLY / VT_RAYS pass through to variant_timing.py)
R=$GRAFT_REPO_ROOT
TAG=${1:-tpmc}
PREC=${2:-f32}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "$LIST_COUNTERS" ] && { timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"; }
export VT_RAYS=${VT_RAYS:-6144} VT_ITERS=${VT_ITERS:-6}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python $R/tools/variant_timing.py $PREC > $O/variants.jsonl 2> $O/variants.err
rc=$?; echo "stats rc=$rc"; cat $O/variants.jsonl; [ $rc -ne 0 ] && { tail -5 $O/variants.err; exit $rc; }
python $R/tools/kstats.py $O/stats/run_kernel_stats.csv > $O/kstats.txt; head -20 $O/kstats.txt
export VT_ONLY=${VT_ONLY:-fwd_train,bwd_train} VT_ITERS=3
PASSES=${PMC_PASSES:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
IFS='|' read -ra PASS_LIST <<< "$PASSES"
for c in "${PASS_LIST[@]}"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "${PMC_REGEX:-field_w16|field_x3|gemm_tn|reduce_jobs}" -d $O/pmc_$tag -o run --output-format csv -- python $R/tools/variant_timing.py $PREC > $O/pmc_$tag.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$tag.log; exit $rc; }
done
python $R/tools/pmc_kernels.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
