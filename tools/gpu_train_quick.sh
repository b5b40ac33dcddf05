#!/bin/bash
# Training-step development call: the GPU tests (optionally -k), then the C3 training iteration
# alone (tools/train_timing.py) under rocprofv3 kernel stats, then the C2 volume_render timing.
#   PYTEST_K=... tools/gpu_train_quick.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-tq}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -20; [ $rc -ne 1 ] && exit $rc; }
fi
cd /tmp && export TMPDIR=/tmp
for p in ${TRAIN_PRECISIONS:-f32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/train_$p -o run --output-format csv -- python $R/tools/train_timing.py --precision $p --iters ${TRAIN_ITERS:-8} > $O/train_$p.json 2> $O/train_$p.err
  rc=$?; echo "train $p rc=$rc"; tail -1 $O/train_$p.json | cut -c1-400; [ $rc -ne 0 ] && { tail -5 $O/train_$p.err; exit $rc; }
  python $R/tools/kstats.py $O/train_$p/run_kernel_stats.csv > $O/train_${p}_kstats.txt; head -25 $O/train_${p}_kstats.txt
done
for v in ${EXTRA_LIBS}; do   # variant builds (tools/build_variants.sh) of the f32 iteration
  CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/train_f32_$v -o run --output-format csv -- python $R/tools/train_timing.py --precision f32 --iters ${TRAIN_ITERS:-8} > $O/train_f32_$v.json 2> $O/train_f32_$v.err
  rc=$?; echo "train f32 $v rc=$rc"; tail -1 $O/train_f32_$v.json | cut -c1-300; [ $rc -ne 0 ] && { tail -5 $O/train_f32_$v.err; exit $rc; }
  python $R/tools/kstats.py $O/train_f32_$v/run_kernel_stats.csv > $O/train_f32_${v}_kstats.txt; head -12 $O/train_f32_${v}_kstats.txt
done
timeout -k 10 120 python $R/tools/volume_timing.py > $O/volume.json 2> $O/volume.err
rc=$?; echo "volume rc=$rc"; cat $O/volume.json; [ $rc -ne 0 ] && { tail -5 $O/volume.err; exit $rc; }
exit 0
