"""torch.library operators (namespace ``codenerf``).

CPU: every op is registered with its schema, fake (meta) shapes are right, and
a CPU tensor is refused (no CPU kernel exists -- there is no fallback).
GPU: the ops agree with the module path (which the parity tests pin to the
reference) and their registered backwards give the same gradients.
"""
import numpy as np
import pytest
import torch

OPS = ["ray_bundle", "ray_bundle_backward", "sample_uniform", "sample_pdf", "posenc", "posenc_backward",
       "volume_render", "volume_render_backward", "codenerf_mlp", "codenerf_mlp_train", "codenerf_mlp_backward",
       "render_rays"]


def test_ops_registered():
    import codenerf.torch_ops  # noqa: F401
    for name in OPS:
        assert hasattr(torch.ops.codenerf, name), name


def test_fake_shapes():
    import codenerf.torch_ops  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        c = torch.ops.codenerf
        raw, z, rd = (torch.empty(10, 7, 4, device="cuda"), torch.empty(10, 7, device="cuda"),
                      torch.empty(10, 3, device="cuda"))
        assert [tuple(t.shape) for t in c.volume_render(raw, z, rd)] == [(10, 3), (10,), (10,), (10, 7), (10,)]
        x = torch.empty(33, 3, device="cuda")
        assert tuple(c.posenc(x, [1.0, 2.0], True).shape) == (33, 15)
        pts, zz = c.sample_pdf(rd, rd, torch.empty(10, 5, device="cuda"), z, 9)
        assert tuple(pts.shape) == (10, 16, 3) and tuple(zz.shape) == (10, 16)
        params = [torch.empty(4, device="cuda")] * 18
        out = c.render_rays(rd, rd, torch.empty(10, 256, device="cuda"), torch.empty(10, 256, device="cuda"),
                            params, params, 0.8, 1.8, 64, 0, "lindepth", False, 10, 4, True, True, 10)
        assert tuple(out[0].shape) == (10, 3) and tuple(out[4].shape) == (10, 64)


def test_cpu_tensors_are_refused():
    import codenerf.torch_ops  # noqa: F401
    with pytest.raises(NotImplementedError):
        torch.ops.codenerf.posenc(torch.zeros(3, 3), [1.0], True)


# ---------------------------------------------------------------- GPU


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import codenerf
    import codenerf.torch_ops  # noqa: F401
    codenerf.load_library()
    return torch.device("cuda", 0)


def _params(dev, seed):
    from codenerf import synthetic
    return [t.to(dev) for t in synthetic.codenerf_params(seed).values()]


@pytest.mark.gpu
def test_volume_render_op_grad(dev):
    from codenerf.nerf import volume_render
    g = torch.Generator().manual_seed(0)
    raw = (torch.randn(40, 12, 4, generator=g) + 1).to(dev)
    z = torch.sort(0.8 + torch.rand(40, 12, generator=g), -1).values.to(dev)
    rd = torch.randn(40, 3, generator=g).to(dev)
    a, b = raw.clone().requires_grad_(True), raw.clone().requires_grad_(True)
    outs_a = torch.ops.codenerf.volume_render(a, z, rd)
    outs_b = volume_render(b, z, rd)
    for x, y in zip(outs_a, outs_b):
        assert torch.equal(x, y)
    (outs_a[0].sum() + outs_a[4].sum()).backward()
    (outs_b[0].sum() + outs_b[4].sum()).backward()
    assert torch.equal(a.grad, b.grad)


@pytest.mark.gpu
def test_mlp_ops(dev):
    from codenerf import ops
    p = _params(dev, 0)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(300, 90, generator=g).to(dev)
    zs, zt = (torch.randn(1, 256, generator=g) * 0.3).to(dev), (torch.randn(1, 256, generator=g) * 0.3).to(dev)
    raw = torch.ops.codenerf.codenerf_mlp(zs.expand(300, -1), zt.expand(300, -1), x, p, "f32")
    # precision "f32" runs the 16x16x4 two-waves-per-SIMD kernel (format f32_w16); the training
    # forward (codenerf_mlp_train) is the 32x32x2 kernel: same fp32 products, other summation order
    cb = ops.code_bias(p, zs, zt)
    ref_w16 = ops.mlp_forward(ops.mlp_pack(p, "f32_w16"), cb, x, precision="f32_w16")
    assert torch.equal(raw, ref_w16)
    ref = ops.mlp_forward(ops.mlp_pack(p, "f32"), cb, x)
    assert (ref_w16 - ref).abs().max().item() <= 1e-5
    pr = [t.clone().requires_grad_(True) for t in p]
    xg, zsg = x.clone().requires_grad_(True), zs.clone().requires_grad_(True)
    raw_t, _ = torch.ops.codenerf.codenerf_mlp_train(zsg, zt, xg, pr)
    assert (raw_t - ref).abs().max().item() == 0.0
    raw_t.square().sum().backward()
    assert xg.grad is not None and zsg.grad is not None and all(t.grad is not None for t in pr)
    assert np.isfinite(xg.grad.cpu().numpy()).all()


@pytest.mark.gpu
def test_render_rays_op_matches_module(dev):
    from codenerf import nerf
    from codenerf.models import CodeNeRFModel
    from codenerf import synthetic
    ms = []
    for s in (0, 1):
        m = CodeNeRFModel(hidden_size=256, shape_code_size=256, texture_code_size=256, num_encoding_fn_xyz=10,
                          num_encoding_fn_dir=4)
        m.load_state_dict(synthetic.codenerf_params(s))
        m.precision = "f32"
        ms.append(m.to(dev).eval())
    g = torch.Generator().manual_seed(2)
    ro = (torch.randn(500, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(500, 3, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    zse, zte = zs.expand(500, -1), zt.expand(500, -1)
    ps = nerf.PointSampler(32, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    emb = (nerf.PositionalEmbedder(10, True, True, torch.float32, dev),
           nerf.PositionalEmbedder(4, True, True, torch.float32, dev))
    with torch.no_grad():
        ref = nerf.render_rays(ro, rd, zse, zte, ps, emb, ms[0], ms[1], 128)
        out = torch.ops.codenerf.render_rays(ro, rd, zse, zte, ms[0].param_list(), ms[1].param_list(), 0.8, 1.8, 32,
                                             64, "lindepth", False, 10, 4, True, True, 128)
    assert torch.equal(out[0], ref["rgb_coarse"]) and torch.equal(out[1], ref["rgb_fine"])
    assert torch.equal(out[2], ref["depth_fine"]) and torch.equal(out[5], ref["z_fine"])
