#!/bin/bash
# layer_xyz1 dW kernels A/B: the barrier-free per-wave-ring kernel (default) against the 16-row shared
# stage kernel (CN_XENC_V1=1): training tests, C3 iterations alternating, kernel stats of each.
R=$GRAFT_REPO_ROOT; TAG=${1:-xab}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py -m gpu -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  for v in v2 v1; do
    if [ $v = v1 ]; then ENVV="CN_XENC_V1=1"; else ENVV="CN_XENC_V1=0"; fi
    env $ENVV timeout -k 10 200 python tools/train_timing.py --iters 10 > $O/train_$v.r$round.json 2> $O/train_$v.err
    rc=$?; echo "$v round $round rc=$rc $(cut -c1-70 $O/train_$v.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/train_$v.err; exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
for v in v2 v1; do
  if [ $v = v1 ]; then export CN_XENC_V1=1; else export CN_XENC_V1=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python $R/tools/train_timing.py --iters 6 > $O/prof_$v.json 2> $O/prof_$v.err
  rc=$?; echo "prof $v rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/prof_$v.err; exit $rc; fi
  python $R/tools/kstats.py $O/prof_$v/run_kernel_stats.csv > $O/kstats_$v.txt; grep -E "xenc|reduce_jobs|dir_enc" $O/kstats_$v.txt
done
