#!/bin/bash
# C3 training-iteration A/B: the tree's library against library variants (code-nerf_amd/codenerf/lib/variants/
# lib_<v>.so, CODENERF_ALLOW_STALE=1), alternating, ROUNDS rounds; then the tree's iteration under kernel stats.
#   VARIANTS="head" ROUNDS=2 tools/gpu_train_ab.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-tab}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in tree ${VARIANTS:-head}; do
    if [ $v = tree ]; then ENVV=""; else ENVV="CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so"; fi
    env $ENVV timeout -k 10 200 python tools/train_timing.py --precision ${PREC:-f32} --iters ${TRAIN_ITERS:-10} > $O/train_$v.r$round.json 2> $O/train_$v.err
    rc=$?; echo "$v round $round rc=$rc $(cut -c1-70 $O/train_$v.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/train_$v.err; exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/train_timing.py --precision ${PREC:-f32} --iters 8 > $O/train_prof.json 2> $O/train_prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/train_prof.err; exit $rc; fi
python $R/tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -12 $O/kstats.txt
