#!/bin/bash
# Kernel stats of the C3 training iteration for the tree's library and library variants
# (code-nerf_amd/codenerf/lib/variants/lib_<v>.so), ROUNDS rounds; prints the kernels matching KRE.
#   VARIANTS="a b" KRE="gemm_tn_enc|jobs" tools/gpu_variant_kstats.sh <tag>
R=$GRAFT_REPO_ROOT; TAG=${1:-vks}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in tree ${VARIANTS:-}; do
    if [ $v = tree ]; then ENVV=""; else ENVV="CODENERF_ALLOW_STALE=1 CODENERF_LIB=$R/code-nerf_amd/codenerf/lib/variants/lib_$v.so"; fi
    d=$O/r${round}_$v
    env $ENVV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python $R/tools/train_timing.py --iters 6 > $d.json 2> $d.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 $d.err; exit $rc; fi
    echo "$v r$round $(cut -c1-30 $d.json)"
    python3 -c "import csv,re,sys; [print('   %-60s %10.1f us' % (r['Name'][:60], float(r['AverageNs']) / 1e3)) for r in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[2], r['Name'])]" $d/run_kernel_stats.csv "${KRE:-gemm_tn_enc}"
  done
done
