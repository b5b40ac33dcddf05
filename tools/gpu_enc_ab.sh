#!/bin/bash
# Encoding-dW A/B: library variants (tools/build_variants.sh) alternating, each under rocprofv3 kernel
# stats of the C3 training iteration (tools/train_timing.py); prints the gemm_tn_enc average per run.
#   VARIANTS="DCN_ENC_INTERLEAVE" tools/gpu_enc_ab.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-encab}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ -n "$PYTEST_K" ]; then
  for v in $(echo ${VARIANTS} | tr ' ' '\n' | grep -v -x -e nodir -e noxenc); do
    CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_train.py -m gpu -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider -k "$PYTEST_K" > $O/pytest_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc $(tail -1 $O/pytest_$v.log)"; [ $rc -gt 1 ] && exit $rc
  done
fi
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for v in tree ${VARIANTS}; do
    if [ $v = tree ]; then ENVV=""; elif [ $v = nodir ]; then ENVV="CN_DIR_IN_ENC=0"; elif [ $v = noxenc ]; then ENVV="CN_XENC_PLANE=0"; else ENVV="CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so"; fi
    env $ENVV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$round -o run --output-format csv -- python $R/tools/train_timing.py --precision f32 --iters 6 > $O/t_${v}_$round.json 2> $O/t_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/t_${v}_$round.err; exit $rc; }
    python $R/tools/kstats.py $O/p_${v}_$round/run_kernel_stats.csv > $O/k_${v}_$round.txt
    echo "$v r$round $(grep -o '"ms_per_iter": [0-9.]*' $O/t_${v}_$round.json) | $(grep -E 'gemm_tn_enc|gemm_tn_xenc|dir_enc_dw|field_w16_kernel<1, true, true>' $O/k_${v}_$round.txt | awk '{print $(NF-1)}' | tr '\n' ' ')"
  done
done
