"""GraphedEvalStep vs eager eval_step_loss, gradient by gradient over several replays (debug tool)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(precision="f32"):
    import codenerf
    from codenerf import synthetic
    from codenerf.evaluate import GraphedEvalStep, eval_step_loss
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler
    from codenerf.optim import AdamW
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    g = {k: torch.from_numpy(v).to(dev) for k, v in np.load(os.path.join(ROOT, "tests/golden/eval_c5.npz")).items()}
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    models = {}
    for k, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        m = m.to(dev).train()
        m.requires_grad_(False)
        m.precision = precision
        models[k] = m
    names = ("theta", "phi", "rho", "z_s", "z_t")

    def leaves():
        return [g[k].clone().requires_grad_(True) for k in names]
    n = 4
    eager = []
    np.random.seed(17)
    for _ in range(n):
        lv = leaves()
        loss, _ = eval_step_loss(*lv, g["target"], (rs, ps), emb, models, 1e-5, t_rand=g["t_rand"], u=g["u"])
        loss.backward()
        eager.append((loss.item(), [t.grad.clone() for t in lv]))
    lv = leaves()
    th, ph, rh, zs, zt = lv
    opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(17)
    step = GraphedEvalStep(th, ph, rh, zs, zt, g["target"], (rs, ps), emb, models, opt, 1e-5, t_rand=g["t_rand"],
                           u=g["u"])
    for i in range(n):
        loss, _ = step.step()
        torch.cuda.synchronize()
        print(f"replay {i}: loss {loss.item():.8f} eager {eager[i][0]:.8f}")
        for name, t, ref in zip(names, lv, eager[i][1]):
            d = (t.grad - ref).abs()
            print(f"   {name:6s} max|d| {d.max().item():.3e} scale {ref.abs().max().item():.3e} "
                  f"n_bad {(d > 1e-5 * ref.abs().max()).sum().item()} grad_ptr_is_flat "
                  f"{t.grad.data_ptr() == opt._view('grad', t).data_ptr()}")
            if i > 0:
                acc = (t.grad - ref - eager[i - 1][1][names.index(name)]).abs().max().item()
                first = (t.grad - eager[0][1][names.index(name)]).abs().max().item()
                print(f"          vs eager[i]+eager[i-1] {acc:.3e}   vs eager[0] {first:.3e}  |graph| "
                      f"{t.grad.norm().item():.3e} |eager| {ref.norm().item():.3e} "
                      f"cos {torch.nn.functional.cosine_similarity(t.grad.reshape(1, -1), ref.reshape(1, -1)).item():.4f}")


def _main_entry():
    if len(sys.argv) > 2:
        return
    main(*(sys.argv[1:2] or ["f32"]))


def field_only(precision="f32"):
    """Bisect: one RadianceField forward + backward into (z_s, z_t, ro, rd) captured vs eager."""
    import codenerf
    from codenerf import synthetic
    from codenerf.autograd import radiance_field_autograd
    from codenerf.models import CodeNeRFModel
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    m.requires_grad_(False)
    m.precision = precision
    n, s = 2048, 64
    gen = torch.Generator().manual_seed(0)
    ro0 = (torch.rand(n, 3, generator=gen) * 0.2).to(dev)
    rd0 = torch.randn(n, 3, generator=gen).to(dev)
    z = (0.8 + torch.rand(n, s, generator=gen).sort(-1).values).to(dev)
    w = torch.randn(n, s, 4, generator=gen).to(dev)
    zs0 = (torch.randn(1, 256, generator=gen) * 0.3).to(dev)
    zt0 = (torch.randn(1, 256, generator=gen) * 0.3).to(dev)
    fx = [2.0 ** k for k in range(10)]
    fd = [2.0 ** k for k in range(4)]
    scale = torch.zeros(1, device=dev)

    def run(zs, zt, ro, rd):
        raw = radiance_field_autograd(m, rd, zs.expand(n, -1), zt.expand(n, -1), n, fx, fd, ro=ro, z=z)
        loss = ((raw * w).sum(-1) * (1 + scale)).sum()
        loss.backward()
        return loss

    from codenerf import ops
    seen = {}
    orig_bwd, orig_cb = ops.field_backward_x3, ops.code_bias

    def bwd(*a, **k):
        r = orig_bwd(*a, **k)
        seen["g_code"] = r["g_code"]
        seen["d_rd"] = r["d_rd"]
        return r

    def cbf(*a, **k):
        r = orig_cb(*a, **k)
        seen["cb"] = r
        return r
    orig_cbb = ops.code_bias_backward

    def cbb(*a, **k):
        r = orig_cbb(*a, **k)
        seen["dz_s"], seen["dz_t"] = r
        return r
    ops.field_backward_x3, ops.code_bias, ops.code_bias_backward = bwd, cbf, cbb
    lv = [t.clone().requires_grad_(True) for t in (zs0, zt0, ro0, rd0)]
    run(*lv)
    ref = [t.grad.clone() for t in lv]
    ref_seen = {k: v.clone() for k, v in seen.items()}
    lv2 = [t.clone().requires_grad_(True) for t in (zs0, zt0, ro0, rd0)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run(*lv2)
    torch.cuda.current_stream().wait_stream(side)
    for t in lv2:
        t.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        run(*lv2)
    for i in range(3):
        for t in lv2:
            t.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        print("   ", {k: "%.2e" % ((seen[k] - v).abs().max().item() / max(v.abs().max().item(), 1e-30))
                     for k, v in ref_seen.items()})
        print("field_only replay", i, ["%.2e" % ((a.grad - b).abs().max().item() / b.abs().max().item())
                                       for a, b in zip(lv2, ref)])


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "field":
    field_only(sys.argv[1])


if __name__ == "__main__":
    _main_entry()
