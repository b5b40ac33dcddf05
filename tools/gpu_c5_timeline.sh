#!/bin/bash
# C5 eager vs graph: plain timing, then kernel + HIP-runtime trace and the GPU idle analysis.
R=$GRAFT_REPO_ROOT; TAG=${1:-c5t}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 200 python tools/c5_timeline.py > $O/c5.jsonl 2> $O/c5.err; rc=$?; echo "plain rc=$rc"; cat $O/c5.jsonl; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
C5_ITERS=20 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/trace -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5_traced.jsonl 2> $O/c5_traced.err
rc=$?; echo "trace rc=$rc"; cat $O/c5_traced.jsonl; [ $rc -ne 0 ] && { tail -5 $O/c5_traced.err; exit $rc; }
python $R/tools/trace_gaps.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) > $O/gaps.txt; cat $O/gaps.txt
