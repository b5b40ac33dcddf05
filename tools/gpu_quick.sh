#!/bin/bash
# Kernel-development call: GPU tests (optionally a -k filter), then the bench with C5 and rocprof stats.
R=$GRAFT_REPO_ROOT
TAG=${1:-quick}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-2500; [ $rc -ne 0 ] && exit $rc
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -25 $O/kstats.txt
