#!/bin/bash
# A/B of the whole-tile dW GEMM across library variants (tools/build_variants.sh), two rounds.
#   VARIANTS="base TN_NOFLUSH ..." tools/gpu_tn_ab.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-tnab}
O=$R/gpurun_out/$TAG
mkdir -p $O
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so timeout -k 10 120 python $R/tools/tn_timing.py >> $O/tn.jsonl 2>> $O/tn.err || { echo "fail $v"; tail -3 $O/tn.err; exit 1; }
  done
done
cat $O/tn.jsonl
