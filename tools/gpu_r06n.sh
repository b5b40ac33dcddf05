#!/bin/bash
# the final tree's whole GPU suite and smoke()
R=$GRAFT_REPO_ROOT; TAG=${1:-r06n}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc2=$?; echo "smoke rc=$rc2"; tail -2 $O/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
