#!/bin/bash
# One GPU call: full -m gpu suite (no -x: all failures reported), bench line, rocprofv3 kernel stats.
# Output under gpurun_out/$TAG.  Stops at the first step that faults / aborts / times out.
R=$GRAFT_REPO_ROOT
TAG=${1:-r02a}
STEPS=${2:-all}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [[ $STEPS == all || $STEPS == *test* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -40
  [ $rc -gt 1 ] && exit $rc
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 3000 $O/bench.log; [ $rc -ne 0 ] && exit $rc
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --eval-iters 3 --train-iters 1 > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof.log; exit $rc; }
  find $O -name "*stats*.csv"
fi
exit 0
