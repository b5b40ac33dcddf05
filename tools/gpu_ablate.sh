#!/bin/bash
# Kernel-development call: GPU parity of the field/code paths, then field-kernel timing sweeps and ablations.
R=$GRAFT_REPO_ROOT
TAG=${1:-abl}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
[ -z "$SKIP_TESTS" ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc; }
for v in ${VARIANTS:-base NO_DMA NO_MFMA}; do
  CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/ablate/lib_$v.so timeout -k 10 200 python tools/field_timing.py --tag $v ${RAYS:---rays 512 1024 4096 16384} >> $O/ablate.jsonl 2>$O/ablate_$v.err || { echo "fail $v"; tail -3 $O/ablate_$v.err; exit 1; }
done
cat $O/ablate.jsonl
