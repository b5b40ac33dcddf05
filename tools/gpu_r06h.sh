#!/bin/bash
# round-6 evidence (g_code rows in the fp32 eval backward's tail, final sum in the ray launch): the fused
# backward / eval tests first, then the whole GPU suite with margins, the C5 launch sequence, the bench line.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06h}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
rm -f $O/parity_margins.jsonl
timeout -k 10 300 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_grad.py tests/test_gpu_pose_data.py -k "fused or pair or chairs or eval or dir1_fold" > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 $O/pytest_new.log; [ $rc -ne 0 ] && exit $rc
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
C5_PRECISIONS=f32 C5_ITERS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5.json 2> $O/c5.err
rc=$?; echo "c5 trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
python $R/tools/launch_seq.py $O/c5/run_kernel_trace.csv --per-iter 2 --iter 10 > $O/seq_c5.txt; tail -1 $O/seq_c5.txt
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); print('c5', d['eval_c5']['f32']['ms_per_iter'], 'chairs', d['eval_c5_chairs']['ms_per_iter'], 'c3', d['train_c3']['ms_per_iter'], '3080', d['train_3080']['ms_per_iter'])"
exit 0
