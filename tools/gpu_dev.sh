#!/bin/bash
# Kernel-development call: the GPU tests (optionally -k), field-variant timing, then the full bench
# (headline + extras incl. train_c3) with rocprofv3 kernel stats.   tools/gpu_dev.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-dev}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
# test failures (rc 1) still let the timing run; anything else (a crash, a time limit) ends the call
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20; [ $rc -ne 1 ] && exit $rc; }
VT_RAYS=6144 VT_ITERS=${VT_ITERS:-20} timeout -k 10 200 python tools/variant_timing.py f32 > $O/variants.jsonl 2> $O/variants.err
rc=$?; echo "variants rc=$rc"; cat $O/variants.jsonl; [ $rc -ne 0 ] && { tail -5 $O/variants.err; exit $rc; }
[ -n "$NO_BENCH" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-3000; [ $rc -ne 0 ] && exit $rc
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -30 $O/kstats.txt
