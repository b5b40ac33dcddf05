"""Time the C2 field-kernel launch (1,048,576 samples) of the library at $CODENERF_LIB.

Kernel-development harness (variant builds etc.); prints one JSON line.
    CODENERF_LIB=... python tools/field_timing.py [--precision bf16x3] [--iters 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rays", type=int, nargs="+", default=[16384], help="ray counts (x64 samples) to time")
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("CODENERF_LIB", "default")))
    args = ap.parse_args()
    from codenerf import ops, synthetic
    from codenerf.models import CodeNeRFModel
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    m.precision = args.precision
    for n in args.rays:
        run(args, m, n, dev)


def run(args, m, n, dev):
    from codenerf import ops, synthetic
    s = 64
    g = torch.Generator(device="cpu").manual_seed(0)
    ro = (torch.rand(n, 3, generator=g) * 0.2).to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    z = (0.8 + torch.rand(n, s, generator=g).sort(-1).values).to(dev)
    cb = m.code_bias(synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev))
    fx = [2.0 ** k for k in range(10)]
    fd = [2.0 ** k for k in range(4)]
    packed = m.packed()
    for _ in range(3):
        ops.radiance_field(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision=args.precision)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    for a, b in ev:
        a.record()
        raw = ops.radiance_field(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision=args.precision)
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    flop = n * s * 572416
    print(json.dumps({"tag": args.tag, "rays": n, "precision": args.precision, "median_ms": ms[len(ms) // 2], "min_ms": ms[0],
                      "tflops": flop / (ms[len(ms) // 2] * 1e-3) / 1e12, "raw_checksum": float(raw.double().sum())}))


if __name__ == "__main__":
    main()
