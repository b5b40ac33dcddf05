"""Time only bench.py's C3 training iteration (train_bench) -- for rocprofv3 kernel stats of the
training step alone.   python tools/train_timing.py [--precision f32] [--iters 8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--shape", default="c3", help="bench.TRAIN_SHAPES key: c3, cars_code, 3080")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from codenerf import synthetic
    k = synthetic.srn_intrinsics(bench.H, bench.FOCAL)
    r = bench.train_bench(dev, k, args.iters, 1, args.precision, shape=args.shape)
    print(json.dumps({kk: v for kk, v in r.items() if kk != "note"}))


if __name__ == "__main__":
    main()
