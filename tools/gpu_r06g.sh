#!/bin/bash
# round-6 evidence: the GPU suite (XENC role default) with margins, the XENC slot-cost sweep, the bench line.
R=$GRAFT_REPO_ROOT; TAG=${1:-r06g}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
rm -f $O/parity_margins.jsonl
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
for c in 0.28 0.3 0.33 0.36; do
  for sh in c3 3080; do
    CN_TN_COST=1,1.03,1.05,1,0.16,$c timeout -k 10 120 python tools/train_timing.py --shape $sh --iters 10 > $O/t.json 2> $O/t.err; rc=$?
    [ $rc -ne 0 ] && { tail -3 $O/t.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/t.json')); print(json.dumps({'round': $round, 'cost': $c, 'shape': '$sh', 'ms': d['ms_per_iter']}))" | tee -a $O/cost.jsonl
  done
done
done
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
exit 0
