#!/bin/bash
# Selected GPU tests:  PYTEST_K=<expr> tools/gpu_pytest.sh <tag> [test paths...]
R=$GRAFT_REPO_ROOT; TAG=${1:-pt}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 ${PT_TIMEOUT:-600} python -u -m pytest ${@:-tests} -m gpu -v -rA --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -3; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; exit $rc
