"""Field-kernel variants at one size (kernel-development harness): the inference forward, the
mask-writing forward (eval step), the training forward (masks + activation planes) and the two
fused backwards, fp32 w16 or 3xbf16, timed with HIP events.  Prints one JSON line per variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import torch  # noqa: E402


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    return ms[len(ms) // 2]


def main(precision="f32", n=int(os.environ.get("VT_RAYS", 8192)), s=64):
    only = set(filter(None, os.environ.get("VT_ONLY", "").split(",")))
    iters = int(os.environ.get("VT_ITERS", 10))
    from codenerf import ops, synthetic
    from codenerf.models import CodeNeRFModel
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    params = [p.detach() for p in m.param_list()]
    g = torch.Generator(device="cpu").manual_seed(0)
    ro = (torch.rand(n, 3, generator=g) * 0.2).to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    z = (0.8 + torch.rand(n, s, generator=g).sort(-1).values).to(dev)
    cb = ops.code_bias(params, synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev))
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    x3 = precision == "bf16x3"
    pk = ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16")
    pkt = ops.mlp_pack(params, "bf16x3_t" if x3 else "f32_w16_t")
    flop = n * s * 572416
    out = {}
    want = lambda k: not only or k in only
    if want("fwd"):
        out["fwd"] = timed(lambda: ops.radiance_field(pk, cb, rd, s, n, fx, fd, ro=ro, z=z,
                                                  precision="bf16x3" if x3 else "f32_w16"), iters)
    raw, masks = ops.radiance_field_masks(pk, cb, rd, s, n, fx, fd, ro=ro, z=z, precision=precision)
    if want("fwd_masks"):
        out["fwd_masks"] = timed(lambda: ops.radiance_field_masks(pk, cb, rd, s, n, fx, fd, ro=ro, z=z,
                                                                  precision=precision), iters)
    if want("fwd_train"):
        out["fwd_train"] = timed(lambda: ops.radiance_field_train_w16(pk, cb, rd, s, n, fx, fd, ro=ro, z=z,
                                                                      precision=precision), iters)
    d_raw = torch.randn(n, s, 4, generator=g).to(dev) * 1e-3
    if want("bwd_eval"):
        out["bwd_eval"] = timed(lambda: ops.field_backward_x3(pkt, masks, d_raw, n, s, n, 1, fx, fd, rd=rd, ro=ro, z=z,
                                                          want_ro=True, want_rd=True, precision=precision), iters)
    _, saved, tmasks = ops.radiance_field_train_w16(pk, cb, rd, s, n, fx, fd, ro=ro, z=z, precision=precision)
    pg = [torch.zeros_like(p) for p in params]
    if want("bwd_train"):
        out["bwd_train"] = timed(lambda: ops.field_backward_train(pkt, params, tmasks, saved, None, d_raw, n, s, n, 1,
                                                              fx, fd, rd=rd, ro=ro, z=z, param_grads=pg,
                                                              want_ro=True, want_rd=True, precision=precision), iters)
    for k, v in out.items():
        print(json.dumps({"precision": precision, "variant": k, "samples": n * s, "ms": v,
                          "tflops_fp32_equiv": flop / (v * 1e-3) / 1e12}))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["f32"]))
