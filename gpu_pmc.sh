#!/bin/bash
# PMC passes for the field kernel (one counter group per pass, as MI355X_MICROARCH.md prescribes).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex field_kernel -d $R/gpurun_out/pmc/$tag -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc/$tag.log 2>&1
  rc=$?
  echo "$c rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc/$tag.log; exit $rc; fi
done
