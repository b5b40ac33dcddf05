"""Achievable HBM streaming rates on this box (calibration for the HBM-bound dW kernels):
torch reductions / copies over 2 GiB buffers, timed with HIP events."""
import torch


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    n = 512 * 1024 * 1024  # 2 GiB of fp32
    x = torch.randn(n, device="cuda")
    y = torch.empty_like(x)
    t = bench(lambda: x.sum())
    print(f"read  (sum)   {4 * n / t / 1e12:.2f} TB/s")
    t = bench(lambda: y.copy_(x))
    print(f"copy          {8 * n / t / 1e12:.2f} TB/s (read + write)")
    t = bench(lambda: y.fill_(1.0))
    print(f"write (fill)  {4 * n / t / 1e12:.2f} TB/s")
    a = x.view(-1, 256)
    t = bench(lambda: a.sum(0))
    print(f"column sum (M x 256) {4 * n / t / 1e12:.2f} TB/s")


if __name__ == "__main__":
    main()
