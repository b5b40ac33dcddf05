#!/bin/bash
# round 5 (i): the tail work -- sample_pdf (wave scan + bitonic), code backward (64 slices, in-place
# code-table rows), batched reduce -- its tests, then the C3 iteration timing and its kernel stats.
R=$GRAFT_REPO_ROOT; TAG=${1:-r05i}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  timeout -k 10 200 python tools/train_timing.py --precision ${PREC:-f32} --iters 10 > $O/train.r$round.json 2> $O/train.err
  rc=$?; echo "round $round rc=$rc $(cut -c1-90 $O/train.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/train.err; exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision ${PREC:-f32} --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/train_prof.err; exit $rc; fi
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -24 $O/kstats.txt
export C5_PRECISIONS=${C5_PRECISIONS:-f32}
cd $R && timeout -k 10 200 python tools/c5_timeline.py > $O/c5.jsonl 2> $O/c5.err; rc=$?; echo "c5 rc=$rc"; cat $O/c5.jsonl; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
cd /tmp && C5_ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5prof -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5_prof.jsonl 2> $O/c5_prof.err
rc=$?; echo "c5 prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5_prof.err; exit $rc; }
python $R/tools/kstats.py $O/c5prof/run_kernel_stats.csv > $O/c5_kstats.txt; head -30 $O/c5_kstats.txt
