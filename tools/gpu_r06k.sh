#!/bin/bash
# round-6 A/B: the batched dW launch's plain / SIG jobs in 16-row stages on 4 slots (default), 8 / 7
# (CN_TW_ROWS): bitwise test first, then C3 / 3080 iteration times (two rounds), then per-form kernel stats.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06k}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -v -rf --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_train.py -k "stage_forms or paired_fields" > $O/pytest_forms.log 2>&1
rc=$?; echo "form tests rc=$rc"; tail -3 $O/pytest_forms.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for rows in 16 8; do
    for sh in c3 3080; do
      CN_TW_ROWS=$rows timeout -k 10 120 python tools/train_timing.py --shape $sh --iters 10 > $O/t.json 2> $O/t.err; rc=$?
      [ $rc -ne 0 ] && { tail -3 $O/t.err; exit $rc; }
      python3 -c "import json; d=json.load(open('$O/t.json')); print(json.dumps({'round': $round, 'rows': $rows, 'shape': '$sh', 'ms': d['ms_per_iter']}))" | tee -a $O/forms.jsonl
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for rows in 16 8; do
  CN_TW_ROWS=$rows timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/k$rows -o run --output-format csv -- python $R/tools/train_timing.py --shape c3 --iters 4 > $O/k$rows.json 2> $O/k$rows.err
  rc=$?; echo "kstats $rows rc=$rc"; [ $rc -ne 0 ] && { tail -3 $O/k$rows.err; exit $rc; }
  python $R/tools/kstats.py $O/k$rows/run_kernel_stats.csv > $O/kstats_$rows.txt; grep -E "jobs_kernel|field_w16" $O/kstats_$rows.txt
done
exit 0
