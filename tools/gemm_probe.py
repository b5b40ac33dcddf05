"""dW = dPre^T X shapes of the training step: cn_gemm_tn vs the vendor GEMM (torch.mm -> hipBLASLt /
rocBLAS) on MI355X, fp32.  Prints TFLOP/s per shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))

import torch  # noqa: E402


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    from codenerf import ops
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    for M in (262144, 524288):
        for n, k in ((256, 256), (256, 63), (3, 256), (256, 27)):
            a = torch.randn(M, n, device=dev)
            b = torch.randn(M, k, device=dev)
            fl = 2.0 * M * n * k
            ref = torch.mm(a.double().t(), b.double()).float()
            line = [f"M={M} N={n} K={k}:"]
            for prec in ("f32", "bf16x3"):
                for det in (False, True):
                    c = torch.zeros(n, k, device=dev)
                    t = bench(lambda: ops.gemm_tn(a, b, c, precision=prec, deterministic=det))
                    c.zero_()
                    ops.gemm_tn(a, b, c, precision=prec, deterministic=det)
                    err = ((c - ref).abs().max() / ref.abs().max()).item()
                    gbs = 4.0 * M * (n + k) / t / 1e6
                    line.append(f"{prec}{'/det' if det else ''} {t * 1e3:7.1f} us {fl / t / 1e9:6.1f} TF {gbs:6.0f} GB/s "
                                f"(err {err:.1e})")
            t_mm = bench(lambda: torch.mm(a.t(), b))
            line.append(f"torch.mm {t_mm * 1e3:7.1f} us")
            print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
