#!/bin/bash
# volume_render / sample_uniform A/B: tools/volume_timing.py on the tree's library and on variants
# (code-nerf_amd/codenerf/lib/variants/lib_<v>.so), alternating, ROUNDS rounds.   VARIANTS="a b" tools/gpu_vol_ab.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-vab}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in tree ${VARIANTS:-head}; do
    if [ $v = tree ]; then ENVV=""; else ENVV="CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so"; fi
    env $ENVV timeout -k 10 120 python tools/volume_timing.py --iters 50 > $O/vol_$v.r$round.json 2> $O/vol_$v.err
    rc=$?; echo "$v r$round rc=$rc $(cat $O/vol_$v.r$round.json)"; if [ $rc -ne 0 ]; then tail -5 $O/vol_$v.err; exit $rc; fi
  done
done
