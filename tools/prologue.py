"""Share of the fp32 field kernels' tile loop spent in the tile prologue (sample inputs, code row,
encodings: from a tile's start to its first chunk), training forward and training backward at the
C3 chunk-field size.  Library built with -DCN_PROBE_PROLOGUE (tools/build_variants.sh PROLOGUE):
    CODENERF_LIB=.../lib_PROLOGUE.so python tools/prologue.py [--rays 6144] [--samples 64]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def read(fn, nb):
    buf = np.zeros((nb, 8, 3), dtype=np.int64)
    assert fn(buf.ctypes.data, nb) == 0
    pro, loop, nt = buf[..., 0].astype(np.float64), buf[..., 1].astype(np.float64), buf[..., 2]
    return {"prologue_frac": float(pro.sum() / loop.sum()), "clk_per_tile": float(loop.sum() / nt.sum()),
            "prologue_clk_per_tile": float(pro.sum() / nt.sum()), "tiles": int(nt[:, 0].sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=6144)
    ap.add_argument("--samples", type=int, default=64)
    args = ap.parse_args()
    from codenerf import ops, synthetic
    from codenerf.models import CodeNeRFModel
    fn = ops._lib_ready().cn_debug_prologue
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    params = [p.detach() for p in m.param_list()]
    packed, packed_t = ops.mlp_pack(params, "f32_w16"), ops.mlp_pack(params, "f32_w16_t")
    cb = ops.code_bias(params, synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev))
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    n, s = args.rays, args.samples
    g = torch.Generator().manual_seed(0)
    ro = (torch.rand(n, 3, generator=g) * 0.2).to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    z = (0.8 + torch.rand(n, s, generator=g).sort(-1).values).to(dev)
    nb = min(256, (n * s + 127) // 128)
    out = {"rays": n, "samples": s}
    for _ in range(3):
        ops.radiance_field(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision="f32_w16")
    torch.cuda.synchronize()
    out["forward_inference"] = read(fn, nb)
    for _ in range(3):
        raw, saved, masks = ops.radiance_field_train_w16(packed, cb, rd, s, 4096, fx, fd, ro=ro, z=z, precision="f32")
    torch.cuda.synchronize()
    out["forward_train"] = read(fn, nb)
    gout = torch.randn(n, s, 4, generator=g).to(dev)
    pg = [torch.zeros_like(p) for p in params]
    for _ in range(2):
        ops.field_backward_train(packed_t, params, masks, saved, None, gout, n, s, 4096, 1, fx, fd, rd=rd,
                                 param_grads=pg, precision="f32", ro=ro, z=z)
        torch.cuda.synchronize()
        out["backward_train_then_dw"] = read(fn, nb)   # the last fp32 field launch: the fused backward
    print(json.dumps(out))


if __name__ == "__main__":
    main()
