#!/bin/bash
# the multi-rank and RCCL tests with file:// / in-memory rendezvous (no TCP port race)
R=$GRAFT_REPO_ROOT; TAG=${1:-r06m}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_multirank.py tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1
rc=$?; echo "dist tests rc=$rc"; tail -3 $O/pytest_dist.log; grep -E "^(FAILED|ERROR)" $O/pytest_dist.log | head; exit $rc
