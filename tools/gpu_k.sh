#!/bin/bash
# Kernel-development call: selected GPU tests (-k filter), optional bench args after the filter.
R=$GRAFT_REPO_ROOT
TAG=$1; K=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf -k "$K" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest.log | tail -30
[ $rc -gt 1 ] && exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 600 python "$@" > $O/run.log 2>&1
  rc=$?; echo "run rc=$rc"; tail -c 3000 $O/run.log; exit $rc
fi
exit 0
