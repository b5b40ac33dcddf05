"""C3 small-launch tail per training iteration from a rocprofv3 kernel trace of tools/train_timing.py:
the kernels between the first training-forward launch of iteration 2 and that of the last iteration
(whole iterations, past the warm-up and before bench's stand-alone AdamW timing), except the training
forward / fused backward / batched dW / encoding dW / reduce launches.
    python tools/tail_stats.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

BIG = ("field_w16_kernel", "field_w16_bwd_kernel", "field_x3_kernel", "field_x3_bwd_kernel", "gemm_tn256_jobs_kernel",
       "gemm_tn_enc_kernel", "gemm_tn_xenc_kernel", "reduce_jobs_kernel")
FWD_PER_ITER = 8          # 4 chunks x (coarse + fine)


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    fwd = [i for i, r in enumerate(rows) if "field_w16_kernel<" in r["Kernel_Name"] or "field_x3_kernel<" in r["Kernel_Name"]]
    n_it = len(fwd) // FWD_PER_ITER
    lo, hi = fwd[FWD_PER_ITER], fwd[FWD_PER_ITER * (n_it - 1)]
    iters = n_it - 2
    per = defaultdict(lambda: [0.0, 0])
    for r in rows[lo:hi]:
        name = r["Kernel_Name"]
        if any(b in name for b in BIG):
            continue
        p = per[name[:70]]
        p[0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        p[1] += 1
    tot = sum(v[0] for v in per.values())
    n = sum(v[1] for v in per.values())
    print(f"{iters} iterations: tail {tot / iters / 1e3:.3f} ms / iteration, {n / iters:.1f} launches")
    for name, (us, c) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"  {us / iters:7.1f} us  {c / iters:5.1f}x  {name}")


if __name__ == "__main__":
    main()
