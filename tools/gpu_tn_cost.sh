#!/bin/bash
# Slot-cost sweep of the batched dW launch (CN_TN_COST="dir2,dir1,out,xyz2,rgb"): the jobs kernel's
# time per call under rocprofv3 kernel stats for each cost vector, alternating, ROUNDS rounds.
#   COSTS="1,1.03,1.05,1,0.16 ..." tools/gpu_tn_cost.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-tncost}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do
  for c in ${COSTS:-1,1.03,1.05,1,0.16}; do
    d=$O/r${round}_$(echo $c | tr ',' '_')
    CN_TN_COST=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python $R/tools/train_timing.py --iters 6 > $d.json 2> $d.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$c rc=$rc"; tail -5 $d.err; exit $rc; fi
    echo "$c r$round $(cut -c1-40 $d.json) $(grep -h gemm_tn256_jobs $d/run_kernel_stats.csv | awk -F, '{print $4/1000 " us"}')"
  done
done
