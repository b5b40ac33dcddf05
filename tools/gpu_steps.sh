#!/bin/bash
# rocprofv3 kernel stats of the C5 eval step (f32, bf16x3) and the C3 training iteration.
R=$GRAFT_REPO_ROOT
TAG=${1:-steps}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JOBS=${JOBS:-"eval_f32_20 eval_bf16x3_20 train_f32_3"}
for jt in $JOBS; do
  job=$(echo $jt | tr "_" " ")
  t=$(echo $job | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$t -o run --output-format csv -- python $R/tools/step_prof.py $job > $O/$t.log 2>&1
  rc=$?; echo "$job rc=$rc"; tail -1 $O/$t.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
  python $R/tools/kstats.py $O/$t/run_kernel_stats.csv > $O/$t.kstats.txt; head -14 $O/$t.kstats.txt
done
exit 0
