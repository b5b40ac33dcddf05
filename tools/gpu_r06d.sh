#!/bin/bash
# round-6: the paired eval backward -- its tests and the eval / training tests around it, then the C5 and
# chairs eval iterations' launch sequences and timings.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06d}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_grad.py tests/test_gpu_pose_data.py tests/test_gpu_train.py -k "pair or eval or graph or time_optimize or shape_chunk or in_place" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -gt 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
C5_PRECISIONS=f32 C5_ITERS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5.json 2> $O/c5.err
rc=$?; echo "c5 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
python $R/tools/launch_seq.py $O/c5/run_kernel_trace.csv --per-iter 2 --iter 10 > $O/seq_c5.txt; tail -1 $O/seq_c5.txt
cd $R
timeout -k 10 200 python tools/c5_timeline.py > $O/c5_time.json 2> $O/c5_time.err; rc=$?; echo "c5 time rc=$rc"; cat $O/c5_time.json
exit 0
