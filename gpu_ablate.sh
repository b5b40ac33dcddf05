#!/bin/bash
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for v in base NO_DMA NO_MFMA; do
  CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/ablate/lib_$v.so timeout -k 10 200 python tools/field_timing.py --tag $v >> gpurun_out/ablate.jsonl 2>gpurun_out/ablate_$v.err || { echo "fail $v"; tail -3 gpurun_out/ablate_$v.err; exit 1; }
done
cat gpurun_out/ablate.jsonl
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
