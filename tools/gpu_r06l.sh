#!/bin/bash
# round-6 final evidence: the GPU suite with margins, smoke(), the default bench line, the headline under
# rocprofv3 kernel stats, and the headline kernel's PMC passes (HBM bytes, MFMA busy).
R=$GRAFT_REPO_ROOT; TAG=${1:-r06l}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
rm -f $O/parity_margins.jsonl
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kstats -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-extras > $O/kstats_bench.json 2> $O/kstats_bench.err
rc=$?; echo "kstats rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/kstats_bench.err; exit $rc; }
python $R/tools/kstats.py $O/kstats/run_kernel_stats.csv > $O/headline_kstats.txt; head -6 $O/headline_kstats.txt
cd $R && PMC_PASSES="FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/gpu_pmc.sh $TAG/pmc field_w16 f32
