"""HIP-event timing of one whole-tile dW GEMM (gemm_tn256_kernel + its fixed-order reduction, the
deterministic cn_gemm_tn_ws path) at the C3 chunk size, for the library at $CODENERF_LIB (a variant
builds).   CODENERF_LIB=... python tools/tn_timing.py [--m 393216] [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=393216)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("CODENERF_LIB", "default")))
    args = ap.parse_args()
    from codenerf import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(args.m, 256, generator=g).to(dev)
    b = torch.relu(torch.randn(args.m, 256, generator=g)).to(dev)
    c = torch.zeros(256, 256, device=dev)
    ops.gemm_tn(a, b, c, deterministic=True)  # one call from zero: a digest to compare kernel variants bitwise
    import hashlib
    digest = hashlib.sha256(c.cpu().numpy().tobytes()).hexdigest()[:16]
    for _ in range(3):
        ops.gemm_tn(a, b, c, deterministic=True)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    for e0, e1 in ev:
        e0.record()
        ops.gemm_tn(a, b, c, deterministic=True)
        e1.record()
    torch.cuda.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    flop = 2.0 * args.m * 256 * 256
    print(json.dumps({"tag": args.tag, "m": args.m, "digest": digest, "wide": os.environ.get("CN_TN_WIDE", "0"), "median_us": ms[len(ms) // 2] * 1e3, "min_us": ms[0] * 1e3,
                      "tflops": flop / (ms[len(ms) // 2] * 1e-3) / 1e12}))


if __name__ == "__main__":
    main()
