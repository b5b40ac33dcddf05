#!/bin/bash
# One GPU call: full -m gpu suite, bench line, rocprofv3 kernel stats.  Output under gpurun_out/$TAG.
R=$GRAFT_REPO_ROOT
TAG=${1:-r01c}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --hierarchical > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 $O/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof.log; exit $rc; }
find $O -name "*stats*.csv"
