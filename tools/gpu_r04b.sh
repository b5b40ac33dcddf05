#!/bin/bash
# gloo device-tensor probe, then the whole GPU suite with the parity margins recorded.
R=$GRAFT_REPO_ROOT; TAG=${1:-r04b}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 120 python tools/gloo_probe.py > $O/gloo_probe.jsonl 2> $O/gloo_probe.err; echo "probe rc=$?"; cat $O/gloo_probe.jsonl
rm -f $O/parity_margins.jsonl
CN_MARGINS=$O/parity_margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "^(FAILED|ERROR)" $O/pytest_gpu.log | head -30; exit $rc
