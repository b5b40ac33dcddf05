"""Per-kernel timing of the fused field kernels at the C3 fine-pass size (4096 rays x 192 samples):
forward (masks, + activation planes) and backward (eval, + training planes) in both precisions.

    python tools/bwd_probe.py [n_rays] [n_samples]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))

import torch  # noqa: E402


def bench(fn, reps=5):
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    from codenerf import ops, synthetic
    from codenerf.models import CodeNeRFModel
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    params = [p.detach() for p in m.param_list()]
    g = torch.Generator().manual_seed(0)
    ro = (torch.randn(n, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(n, s, generator=g), dim=-1).values.to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    gout = torch.randn(n, s, 4, generator=g).to(dev)
    fx = [2.0 ** k for k in range(10)]
    fd = [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    x_enc = ops.encode_inputs(rd, s, n, fx, fd, ro=ro, z=z)
    M = n * s
    for prec, pk, pkt in (("f32", "f32_w16", "f32_w16_t"), ("bf16x3", "bf16x3", "bf16x3_t")):
        packed, packed_t = ops.mlp_pack(params, pk), ops.mlp_pack(params, pkt)
        t_fwd = bench(lambda: ops.radiance_field_masks(packed, cb, rd, s, n, fx, fd, ro=ro, z=z, precision=prec))
        t_fwd_tr = bench(lambda: ops.radiance_field_train_w16(packed, cb, rd, s, n, fx, fd, ro=ro, z=z, precision=prec))
        raw, saved, masks = ops.radiance_field_train_w16(packed, cb, rd, s, n, fx, fd, ro=ro, z=z, precision=prec)
        t_bwd = bench(lambda: ops.field_backward_x3(packed_t, masks, gout, n, s, n, 1, fx, fd, rd=rd, ro=ro, z=z,
                                                    want_ro=True, want_rd=True, precision=prec))
        pg = [torch.zeros_like(p) for p in params]
        t_bwd_tr = bench(lambda: ops.field_backward_train(packed_t, params, masks, saved, x_enc, gout, n, s, n, 1, fx,
                                                          fd, rd=rd, ro=ro, z=z, param_grads=pg, want_ro=True,
                                                          want_rd=True, precision=prec))
        print(f"{prec}: M={M}  fwd(masks) {t_fwd:.3f} ms  fwd(train) {t_fwd_tr:.3f} ms  bwd(eval) {t_bwd:.3f} ms  "
              f"bwd(train, incl. dW) {t_bwd_tr:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
