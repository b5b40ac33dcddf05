#!/bin/bash
# round-6 first call: the new at-size parity tests (reference runnable shapes), then the whole GPU suite
# with the parity margins, then the default bench line.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06a}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
rm -f $O/parity_margins.jsonl
CN_MARGINS=$O/parity_margins_new.jsonl timeout -k 10 300 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py::test_train_shape_chunk_at_size tests/test_gpu_pose_data.py::test_eval_c5_chairs_fused_at_size \
  tests/test_gpu_grad.py::test_field_backward_train_generated_encodings > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 $O/pytest_new.log; [ $rc -gt 1 ] && exit $rc
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
exit 0
