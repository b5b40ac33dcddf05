#!/bin/bash
# Whole-tile dW GEMM: HIP-event timing (tree library) and the TN_WAITPROF probe (barrier / DMA clocks).
R=$GRAFT_REPO_ROOT; TAG=${1:-tnp}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 120 python tools/tn_timing.py > $O/tn_timing.json 2> $O/tn.err; rc=$?; echo "tn rc=$rc $(cat $O/tn_timing.json)"; [ $rc -ne 0 ] && { tail -3 $O/tn.err; exit $rc; }
CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_TN_WAITPROF.so timeout -k 10 120 python tools/tnprof.py > $O/tnprof.json 2> $O/tnprof.err; rc=$?; echo "tnprof rc=$rc $(cat $O/tnprof.json)"; exit $rc
