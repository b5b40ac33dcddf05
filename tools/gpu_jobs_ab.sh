#!/bin/bash
# A/B of the batched whole-tile dW launch (CN_TN_JOBS=1, default) against one launch per GEMM
# (CN_TN_JOBS=0): the training tests, the C3 iteration timing of both (two rounds), then the
# batched iteration under rocprofv3 kernel stats.   tools/gpu_jobs_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-jobs}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20; [ $rc -ne 1 ] && exit $rc; }
# variants: "0" (one launch per GEMM), "1" (the batch, default costs), "lib:X" (variant build X), or a CN_TN_COST string
for round in 1 2; do
  for v in ${JOBS_VARIANTS:-0 1}; do
    case $v in 0|1) ENVV="CN_TN_JOBS=$v";; lib:*) ENVV="CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_${v#lib:}.so";; *) ENVV="CN_TN_COST=$v";; esac
    env $ENVV timeout -k 10 200 python tools/train_timing.py --precision ${PREC:-f32} --iters ${TRAIN_ITERS:-10} > "$O/train_${v#lib:}.r$round.json" 2> "$O/train_${v#lib:}.err"
    rc=$?; echo "$ENVV round $round rc=$rc $(cut -c1-60 "$O/train_${v#lib:}.r$round.json")"; [ $rc -ne 0 ] && { tail -5 "$O/train_${v#lib:}.err"; exit $rc; }
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision ${PREC:-f32} --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_prof.err; exit $rc; }
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -25 $O/kstats.txt
