#!/bin/bash
# round-6: layer_xyz1's dW as a job of the batched dW launch (CN_XENC_ROLE=1) -- its tests, then the
# training iterations A/B against the separate launch, with a sweep of the job's slot cost.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06f}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
CN_XENC_ROLE=1 timeout -k 10 400 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py tests/test_gpu_grad.py -k "pair or shape_chunk or c3_chunk or nogeo or encoding_plane or generated" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
for v in "0 -" "1 1,1.03,1.05,1,0.16,0.25" "1 1,1.03,1.05,1,0.16,0.3" "1 1,1.03,1.05,1,0.16,0.4"; do
  set -- $v
  for sh in c3 3080; do
    if [ "$2" = "-" ]; then env CN_XENC_ROLE=$1 timeout -k 10 120 python tools/train_timing.py --shape $sh --iters 10 > $O/t.json 2> $O/t.err; rc=$?
    else env CN_XENC_ROLE=$1 CN_TN_COST=$2 timeout -k 10 120 python tools/train_timing.py --shape $sh --iters 10 > $O/t.json 2> $O/t.err; rc=$?; fi
    [ $rc -ne 0 ] && { tail -3 $O/t.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/t.json')); print(json.dumps({'round': $round, 'role': '$1', 'cost': '$2', 'shape': '$sh', 'ms': d['ms_per_iter']}))" | tee -a $O/ab.jsonl
  done
done
done
cd /tmp && export TMPDIR=/tmp
CN_XENC_ROLE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/train_c3 -o run --output-format csv -- python $R/tools/train_timing.py --shape c3 --iters 6 > $O/train_c3.json 2> $O/train_c3.err
rc=$?; echo "kstats rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_c3.err; exit $rc; }
python $R/tools/launch_seq.py $O/train_c3/run_kernel_trace.csv > $O/seq_train_c3.txt; tail -1 $O/seq_train_c3.txt
exit 0
