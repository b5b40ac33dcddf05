#!/bin/bash
# x3 v4 kernel: parity (x3 field tests first), then timing + ablations.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_x4.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -15 gpurun_out/pytest_x4.log; [ $rc -gt 1 ] && exit $rc
rm -f gpurun_out/ablate.jsonl
for v in base NO_DMA NO_MFMA; do
  CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/ablate/lib_$v.so timeout -k 10 200 python tools/field_timing.py --tag $v >> gpurun_out/ablate.jsonl 2>gpurun_out/ablate_$v.err || { echo "fail $v"; tail -3 gpurun_out/ablate_$v.err; exit 1; }
done
cat gpurun_out/ablate.jsonl
