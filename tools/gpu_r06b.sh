#!/bin/bash
# round-6 launch-sequence profile: kernel traces of the C3, cars-code and 3080 training iterations and
# of the C5 eval iteration (tools/launch_seq.py splits one steady iteration), plus the aten ops the
# C5 / C3 iterations run (tools/iter_ops.py).
R=$GRAFT_REPO_ROOT; TAG=${1:-r06b}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
MODE=c5 timeout -k 10 120 python tools/iter_ops.py > $O/ops_c5.json 2> $O/ops_c5.err; echo "ops c5 rc=$?"
cd /tmp && export TMPDIR=/tmp
for sh in c3 3080; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/train_$sh -o run --output-format csv -- python $R/tools/train_timing.py --shape $sh --iters 6 > $O/train_$sh.json 2> $O/train_$sh.err
  rc=$?; echo "train $sh rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/train_$sh.err; exit $rc; }
  python $R/tools/launch_seq.py $O/train_$sh/run_kernel_trace.csv > $O/seq_train_$sh.txt; tail -1 $O/seq_train_$sh.txt
done
C5_PRECISIONS=f32 C5_ITERS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c5 -o run --output-format csv -- python $R/tools/c5_timeline.py > $O/c5.json 2> $O/c5.err
rc=$?; echo "c5 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/c5.err; exit $rc; }
python $R/tools/launch_seq.py $O/c5/run_kernel_trace.csv --per-iter 2 --iter 10 > $O/seq_c5.txt; tail -1 $O/seq_c5.txt
exit 0
