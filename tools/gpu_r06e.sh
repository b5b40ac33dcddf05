#!/bin/bash
# round-6 evidence call (pairing): the new at-size parity tests (reference runnable shapes), then the whole GPU suite
# with the parity margins, then the default bench line.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06e}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
rm -f $O/parity_margins.jsonl
CN_MARGINS=$O/parity_margins_new.jsonl timeout -k 10 300 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_pose_data.py tests/test_gpu_grad.py -k "pair or shape_chunk or chairs or time_optimize" \
  > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 $O/pytest_new.log; [ $rc -gt 1 ] && exit $rc
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
timeout -k 10 120 tools/bin/read_probe > $O/read_probe.jsonl 2>&1; echo "read probe rc=$?"; cat $O/read_probe.jsonl
exit 0
