#!/bin/bash
# round 4: dW-kernel tests, the C3 A/B over library variants, the whole-tile dW timing (tree vs head), headline bench
R=$GRAFT_REPO_ROOT; TAG=${1:-r04g}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^(FAILED|ERROR)" $O/pytest.log | head; [ $rc -gt 1 ] && exit $rc
VARIANTS="${VARIANTS:-head lazy linesonly nv steppat}" bash tools/gpu_train_ab.sh $TAG/ab || exit $?
for v in tree head; do
  if [ $v = tree ]; then E=""; else E="CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so"; fi
  env $E timeout -k 10 120 python tools/tn_timing.py --tag $v >> $O/tn.jsonl 2>> $O/tn.err || { echo "tn $v failed"; tail -3 $O/tn.err; exit 1; }
done
cat $O/tn.jsonl
timeout -k 10 300 python -u bench.py --no-cpu-baseline --train-iters 0 --eval-iters 0 > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-500 $O/bench.json
