#!/bin/bash
# round 5 (c): selected GPU tests, then the fp32 C3 iteration (2 timing runs) and its kernel stats.
R=$GRAFT_REPO_ROOT; TAG=${1:-r05c}; shift; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  timeout -k 10 200 python tools/train_timing.py --precision ${PREC:-f32} --iters 10 > $O/train.r$round.json 2> $O/train.err
  rc=$?; echo "round $round rc=$rc $(cut -c1-90 $O/train.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/train.err; exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision ${PREC:-f32} --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/train_prof.err; exit $rc; fi
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -8 $O/kstats.txt
