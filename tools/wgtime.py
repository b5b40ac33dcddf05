"""Per-workgroup start / end of the training forward field_w16_kernel<.., true, true> (library built with
-DCN_PROBE_WGTIME, tools/build_variants.sh WGTIME): how evenly the persistent grid's static tile
round-robin finishes.   CODENERF_LIB=.../lib_WGTIME.so python tools/wgtime.py [--rays 4096 8192 6144]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, nargs="+", default=[4096, 8192, 6144])
    ap.add_argument("--infer", action="store_true", help="the inference kernel (C2: 262144 rays = one bench step)")
    args = ap.parse_args()
    from codenerf import ops, synthetic
    from codenerf.models import CodeNeRFModel
    fn = ops._lib_ready().cn_debug_wgtime
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    params = [p.detach() for p in m.param_list()]
    packed = ops.mlp_pack(params, "f32_w16")
    cb = ops.code_bias(params, synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev))
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    for n in args.rays:
        s = 64
        g = torch.Generator().manual_seed(0)
        ro = (torch.rand(n, 3, generator=g) * 0.2).to(dev)
        rd = torch.randn(n, 3, generator=g).to(dev)
        z = (0.8 + torch.rand(n, s, generator=g).sort(-1).values).to(dev)
        for _ in range(3):
            if args.infer:
                ops.radiance_field(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision="f32")
            else:
                ops.radiance_field_train_w16(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision="f32")
        torch.cuda.synchronize()
        buf = np.zeros((2048, 2), dtype=np.int64)
        assert fn(buf.ctypes.data, 2048) == 0
        t = buf[:256].astype(np.float64) / 100.0    # 100 MHz -> us
        t0 = t[:, 0].min()
        start, end = t[:, 0] - t0, t[:, 1] - t0
        xcd = np.arange(256) % 8
        print(json.dumps({"rays": n, "samples": n * s, "tiles_per_wg": n * s / 128 / 256,
                          "start_us_max": float(start.max()), "end_us": [float(end.min()), float(np.median(end)),
                                                                          float(end.max())],
                          "end_by_xcd_us": [float(end[xcd == k].mean()) for k in range(8)],
                          "span_last_10pct_us": float(end.max() - np.percentile(end, 10))}))


if __name__ == "__main__":
    main()
