#!/bin/bash
# round 5 (a): the no-geometry training backward -- its bitwise test and the training tests, then the
# C3 iteration A/B against the geometry schedule (CN_BWD_NOGEO=0), then the default's kernel stats.
R=$GRAFT_REPO_ROOT; TAG=${1:-r05a}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py -m gpu -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  for v in geo nogeo; do
    if [ $v = geo ]; then ENVV="CN_BWD_NOGEO=0"; else ENVV="CN_BWD_NOGEO=1"; fi
    env $ENVV timeout -k 10 200 python tools/train_timing.py --precision ${PREC:-f32} --iters 10 > $O/train_$v.r$round.json 2> $O/train_$v.err
    rc=$?; echo "$v round $round rc=$rc $(cut -c1-90 $O/train_$v.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/train_$v.err; exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision ${PREC:-f32} --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/train_prof.err; exit $rc; fi
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -14 $O/kstats.txt
