"""Kernel-development check: fused 3xbf16 eval backward vs the CPU oracle, per-sample error profile."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "code-nerf_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def main():
    import oracle.codenerf_oracle as o
    from codenerf import nerf, synthetic
    from codenerf.autograd import sample_points_autograd
    from test_gpu_grad import _oracle_field, embedders, model, oracle_params
    dev = torch.device("cuda", 0)
    r, s, chunk = 37, 16, 13
    for prec in ("bf16x3", "f32"):
        m = model(dev, 0)
        p = {k: v.detach() for k, v in oracle_params(m).items()}
        m.precision = prec
        m.requires_grad_(False)
        g = torch.Generator().manual_seed(r * s + 7)
        ro = torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])
        rd = torch.randn(r, 3, generator=g)
        z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values
        zs, zt = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
        gout = torch.randn(r, s, 4, generator=g)
        for which in range(5):
            go = gout.clone()
            if which < 4:
                mask = torch.zeros(4)
                mask[which] = 1.0
                go = go * mask
            pts_c = (ro[:, None, :] + rd[:, None, :] * z[..., None]).requires_grad_(True)
            zs_c, zt_c = zs.clone().requires_grad_(True), zt.clone().requires_grad_(True)
            raw_c = _oracle_field(o, p, rd, pts_c, zs_c.expand(r, -1), zt_c.expand(r, -1), chunk)
            (raw_c * go).sum().backward()
            pts_g = (ro[:, None, :] + rd[:, None, :] * z[..., None]).to(dev).requires_grad_(True)
            zs_g, zt_g = zs.to(dev).requires_grad_(True), zt.to(dev).requires_grad_(True)
            raw_g = nerf._field(m, embedders(dev), rd.to(dev), zs_g.expand(r, -1), zt_g.expand(r, -1), chunk,
                                pts=pts_g)
            (raw_g * go.to(dev)).sum().backward()
            e = (pts_g.grad.cpu() - pts_c.grad).abs()
            sc = pts_c.grad.abs().max().item()
            per = e.reshape(-1, 3).max(-1).values
            top = torch.topk(per, 5)
            ez = (zs_g.grad.cpu() - zs_c.grad).abs().max().item() / zs_c.grad.abs().max().item()
            et = (zt_g.grad.cpu() - zt_c.grad).abs().max().item() / (zt_c.grad.abs().max().item() + 1e-30)
            print(f"{prec} gout-col {which}: d pts max rel {e.max().item() / sc:.2e} (scale {sc:.2e}); "
                  f"median {per.median().item() / sc:.2e}; top samples {top.indices.tolist()} "
                  f"{[round(v / sc, 5) for v in top.values.tolist()]}; dzs rel {ez:.2e} dzt rel {et:.2e}")


if __name__ == "__main__":
    main()
