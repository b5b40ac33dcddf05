#!/bin/bash
# the pose backward on a side stream beside the code backward (CN_POSE_SIDE): eval tests, then the C5
# iteration with and without it (two rounds) and one traced iteration with it.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06o}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_pose_data.py tests/test_gpu_configs.py tests/test_gpu_drivers.py > $O/pytest_eval.log 2>&1
rc=$?; echo "eval tests rc=$rc"; tail -3 $O/pytest_eval.log; grep -E "^(FAILED|ERROR)" $O/pytest_eval.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_multirank.py -k "eval or shard" > $O/pytest_mr.log 2>&1
rc=$?; echo "multirank eval rc=$rc"; tail -2 $O/pytest_mr.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for side in 1 0; do
    CN_POSE_SIDE=$side C5_PRECISIONS=f32 C5_GRAPH="0 1" C5_ITERS=60 timeout -k 10 200 python tools/c5_timeline.py > $O/c5.json 2> $O/c5.err; rc=$?
    [ $rc -ne 0 ] && { tail -3 $O/c5.err; exit $rc; }
    python3 -c "import json; [print(json.dumps(dict(json.loads(l), round=$round, side=$side))) for l in open('$O/c5.json')]" | tee -a $O/side_ab.jsonl
  done
done
cd /tmp && export TMPDIR=/tmp
C5_PRECISIONS=f32 C5_GRAPH=0 C5_ITERS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5_traced.json 2> $O/c5_traced.err
rc=$?; echo "c5 trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5_traced.err; exit $rc; }
python $R/tools/launch_seq.py $O/c5/run_kernel_trace.csv --per-iter 2 --iter 20 > $O/seq_c5.txt; tail -1 $O/seq_c5.txt
exit 0
