"""HIP-event timing of the C2 volume_render launch (262,144 rays x 64 samples) in isolation, with and
without the weights output, and of the C2 sample_uniform launch (z only, as the bench; perturbed;
with points).
    python tools/volume_timing.py [--rays 262144] [--samples 64] [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import torch  # noqa: E402


def timed(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    return ms[len(ms) // 2] * 1e3, ms[0] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=262144)
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from codenerf import ops
    dev = torch.device("cuda", 0)
    n, s = args.rays, args.samples
    g = torch.Generator(device="cpu").manual_seed(0)
    raw = torch.randn(n, s, 4, generator=g).to(dev)
    z = (0.8 + torch.rand(n, s, generator=g).sort(-1).values).to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    nbytes = lambda w: n * (12 + 20 * s + 20 + (4 * s if w else 0))
    for _ in range(3):
        ops.volume_render(raw, z, rd)
    torch.cuda.synchronize()
    out = {"rays": n, "samples": s}
    for w in (True, False):
        med, best = timed(lambda: ops.volume_render(raw, z, rd, want_weights=w), args.iters)
        out["weights" if w else "no_weights"] = {"median_us": med, "min_us": best, "TBps": nbytes(w) / (med * 1e-6) / 1e12}
    from codenerf.nerf import PointSampler
    ps = PointSampler(s, s, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    ro = torch.randn(n, 3, generator=g).to(dev)
    t_rand = torch.rand(n, s, generator=g).to(dev)
    for name, t, pts in (("uniform_z", None, False), ("uniform_z_perturbed", t_rand, False), ("uniform_pts", None, True)):
        med, best = timed(lambda: ops.sample_uniform(ro, rd, ps.z_vals, ps.lower, ps.upper, t, want_pts=pts), args.iters)
        b = n * (24 if pts else 0) + n * s * (4 + (4 if t is not None else 0) + (12 if pts else 0))
        out[name] = {"median_us": med, "min_us": best, "TBps": b / (med * 1e-6) / 1e12}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
