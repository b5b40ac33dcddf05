#!/bin/bash
# round-6: the paired training backward -- its tests, then the training iterations' launch sequences.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06c}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py -k "pair or shape_chunk or c3_chunk or minibatch or iteration" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -gt 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for sh in c3 3080; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/train_$sh -o run --output-format csv -- python $R/tools/train_timing.py --shape $sh --iters 6 > $O/train_$sh.json 2> $O/train_$sh.err
  rc=$?; echo "train $sh rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_$sh.err; exit $rc; }
  python $R/tools/launch_seq.py $O/train_$sh/run_kernel_trace.csv > $O/seq_train_$sh.txt; tail -1 $O/seq_train_$sh.txt
done
cd $R
for sh in c3 cars_code 3080; do
  timeout -k 10 200 python tools/train_timing.py --shape $sh --iters 12 > $O/time_$sh.json 2> $O/time_$sh.err; rc=$?
  echo "time $sh rc=$rc $(cut -c1-120 $O/time_$sh.json)"; [ $rc -ne 0 ] && { tail -3 $O/time_$sh.err; exit $rc; }
done
exit 0
