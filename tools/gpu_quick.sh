#!/bin/bash
# Quick development call: selected GPU tests (PYTEST_K), the C3 training iteration (two runs, then
# under rocprofv3 kernel stats), and the volume_render timing at S = 64 and S = 192.
#   PYTEST_K=... tools/gpu_quick.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-quick}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20; [ $rc -ne 1 ] && exit $rc; }
for k in 1 2; do
  timeout -k 10 200 python tools/train_timing.py --precision f32 --iters 10 > $O/train.$k.json 2> $O/train.err
  rc=$?; echo "train $k rc=$rc $(cut -c1-60 $O/train.$k.json)"; [ $rc -ne 0 ] && { tail -5 $O/train.err; exit $rc; }
done
for s in 64 192; do
  timeout -k 10 120 python tools/volume_timing.py --samples $s > $O/volume_$s.json 2> $O/volume.err
  rc=$?; echo "volume S=$s rc=$rc $(cat $O/volume_$s.json)"; [ $rc -ne 0 ] && { tail -5 $O/volume.err; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision f32 --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_prof.err; exit $rc; }
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -8 $O/kstats.txt
