#!/bin/bash
# First GPU pass: parity tests, bench, kernel-trace profile.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --hierarchical > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
ls -R $R/gpurun_out/prof1 | head -20
