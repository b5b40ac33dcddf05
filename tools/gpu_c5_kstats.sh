#!/bin/bash
# C5 eval iteration (eager, fp32 unless C5_PRECISIONS): timing, then rocprofv3 kernel stats of the same.
R=$GRAFT_REPO_ROOT; TAG=${1:-c5k}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
export C5_PRECISIONS=${C5_PRECISIONS:-f32}
timeout -k 10 200 python tools/c5_timeline.py > $O/c5.jsonl 2> $O/c5.err; rc=$?; echo "plain rc=$rc"; cat $O/c5.jsonl; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
C5_ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5_prof.jsonl 2> $O/c5_prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5_prof.err; exit $rc; }
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; cat $O/kstats.txt
