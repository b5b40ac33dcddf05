#!/bin/bash
# One GPU call: the -m gpu suite (all failures reported), then the bench (optional args).
R=$GRAFT_REPO_ROOT
TAG=${1:-tb}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -30
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 $O/bench.log; exit $rc
