#!/bin/bash
# Bench (bf16x3 default + f32 side number), kernel-trace stats, PMC traffic / MFMA-busy passes for field_x3.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r01b
mkdir -p $O
cd $R
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --hierarchical > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $O/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof.log; exit $rc; }
for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex field_x3 -d $O/pmc/$tag -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-compare > $O/pmc_$tag.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/pmc_$tag.log; exit $rc; }
done
find $O -name "*.csv" | head -20
