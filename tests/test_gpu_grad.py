"""Backward pass on the HIP kernels vs torch autograd of the oracle.

Every gradient here is computed by the gfx950 backward kernels through the C
ABI (codenerf.autograd) and compared with ``torch.autograd`` run over the CPU
oracle (oracle/codenerf_oracle.py, pinned to the reference by
tests/golden/*.npz) on the same inputs, and against the reference's own eval
step gradients (tests/golden/eval_grad.npz).

Tolerance: gradients are sums over many samples taken in a different order
(MFMA tiles, atomics), so they are compared relative to the tensor's largest
magnitude: max|g - g_ref| <= GRAD_RTOL * max|g_ref| (+1e-7 absolute).
Forward outputs keep the render tolerance (1e-4 absolute).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

GRAD_RTOL = 2e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import codenerf
    codenerf.load_library()
    return torch.device("cuda", 0)


def O():
    import oracle.codenerf_oracle as o
    return o


def close(g, ref, rtol=GRAD_RTOL, what=""):
    g, ref = torch.as_tensor(g).double().cpu(), torch.as_tensor(ref).double().cpu()
    assert g.shape == ref.shape, (what, g.shape, ref.shape)
    scale = ref.abs().max().item() if ref.numel() else 0.0
    err = (g - ref).abs().max().item() if ref.numel() else 0.0
    assert err <= rtol * scale + 1e-7, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def model(dev, seed):
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    m = CodeNeRFModel(hidden_size=256, shape_code_size=256, texture_code_size=256, num_encoding_fn_xyz=10,
                      num_encoding_fn_dir=4)
    m.load_state_dict(synthetic.codenerf_params(seed))
    return m.to(dev)


def oracle_params(m):
    return {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}


def embedders(dev):
    from codenerf.nerf import PositionalEmbedder
    return PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev)


# ---------------------------------------------------------------- GEMM building blocks


# 3xbf16 (split operands, Ah.Bh + Ah.Bl + Al.Bh): ~2^-17 relative error per product, so the
# tolerance relative to the result's largest magnitude is 3e-5 instead of fp32's 1e-5.
GEMM_TOL = {"f32": 1e-5, "bf16x3": 3e-5}


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("m,n,k", [(1000, 257, 283), (64, 3, 256), (4097, 256, 27), (20001, 256, 256), (300, 63, 3),
                                   (65536, 256, 256)])
def test_gemm_nn_masked(dev, m, n, k, precision):
    from codenerf import ops
    g = torch.Generator().manual_seed(m + n + k)
    a, b = torch.randn(m, k, generator=g), torch.randn(k, n, generator=g)
    mask = torch.randn(m, n, generator=g)
    c = ops.gemm_nn(a.to(dev), b.to(dev), mask.to(dev), precision=precision)
    ref = (a.double() @ b.double()) * (mask > 0)
    close(c, ref, GEMM_TOL[precision], "gemm_nn " + precision)


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("m,k,lda", [(1000, 257, 260), (777, 256, 260), (129, 63, 90)])
def test_gemm_nn_strided_a(dev, m, k, lda, precision):
    """Row-strided A (lda > K, the field backward's rows of 260): the dwordx4 VEC path with a
    ragged K and the scalar tail, masked."""
    from codenerf import ops
    g = torch.Generator().manual_seed(m + k)
    store = torch.randn(m, lda, generator=g)
    a = store[:, :k]
    b = torch.randn(k, 256, generator=g)
    mask = torch.randn(m, 256, generator=g)
    c = ops.gemm_nn(store.to(dev)[:, :k], b.to(dev), mask.to(dev), precision=precision)
    close(c, (a.double() @ b.double()) * (mask > 0), GEMM_TOL[precision], f"gemm_nn lda={lda} " + precision)


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("m,n,k", [(5000, 257, 256), (33, 3, 256), (4096, 256, 63), (65536, 256, 256), (70001, 3, 283),
                                   (70001, 3, 256), (65537, 1, 256), (131075, 256, 256)])
@pytest.mark.parametrize("det", [False, True])
def test_gemm_tn_accumulates(dev, m, n, k, precision, det):
    from codenerf import ops
    g = torch.Generator().manual_seed(m * 3 + n + k)
    a, b = torch.randn(m, n, generator=g), torch.randn(m, k, generator=g)
    c0 = torch.randn(n, k, generator=g)
    ad, bd = a.to(dev), b.to(dev)
    c = ops.gemm_tn(ad, bd, c0.to(dev).clone(), precision=precision, deterministic=det)
    close(c, c0.double() + a.double().t() @ b.double(), GEMM_TOL[precision], "gemm_tn " + precision)
    if det:
        # the partial-tile path is bitwise reproducible
        c2 = ops.gemm_tn(ad, bd, c0.to(dev).clone(), precision=precision, deterministic=True)
        assert torch.equal(c, c2), "deterministic gemm_tn differs between two runs"


# ---------------------------------------------------------------- element-wise stages


@pytest.mark.parametrize("s", [2, 7, 24, 64, 128, 129, 192, 300, 512])
def test_volume_render_backward(dev, s):
    from codenerf.nerf import volume_render
    o = O()
    r = 53
    g = torch.Generator().manual_seed(s)
    raw = torch.randn(r, s, 4, generator=g) * 2.0
    raw[..., 3] += 2.0
    raw[0, :, 3] = 30.0            # softplus threshold branch
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values
    rd = torch.randn(r, 3, generator=g)
    wr, wd, wa, wdep = (torch.randn(r, 3, generator=g), torch.randn(r, generator=g), torch.randn(r, generator=g),
                        torch.randn(r, generator=g))
    ww = torch.randn(r, s, generator=g)

    def loss(outs):
        rgb, disp, acc, w, depth = outs
        dd = wd.to(disp.device)
        return ((rgb * wr.to(rgb.device)).sum() + 1e-2 * (disp * dd).sum() + (acc * wa.to(acc.device)).sum()
                + (w * ww.to(w.device)).sum() + (depth * wdep.to(depth.device)).sum())

    raw_c, rd_c = raw.clone().requires_grad_(True), rd.clone().requires_grad_(True)
    loss(o.volume_render(raw_c, z, rd_c)).backward()
    raw_g, rd_g = raw.to(dev).requires_grad_(True), rd.to(dev).requires_grad_(True)
    outs = volume_render(raw_g, z.to(dev), rd_g)
    loss(outs).backward()
    close(raw_g.grad, raw_c.grad, what="d raw")
    close(rd_g.grad, rd_c.grad, what="d rd")


def test_posenc_backward(dev):
    from codenerf.nerf import PositionalEmbedder
    o = O()
    x = torch.randn(777, 3) * 1.5
    gout = torch.randn(777, 63)
    xc = x.clone().requires_grad_(True)
    (o.posenc(xc, o.frequency_bands(10, True), True) * gout).sum().backward()
    xg = x.to(dev).requires_grad_(True)
    emb = PositionalEmbedder(10, True, True, torch.float32, dev)
    (emb.embed(xg) * gout.to(dev)).sum().backward()
    close(xg.grad, xc.grad, 1e-5, "posenc")


def test_ray_bundle_gather_points_backward(dev):
    """get_bundle -> sample gather -> pts = ro + rd z: d c2w (ray_sampler.py:77-99, point_sampler.py:70)."""
    from codenerf.nerf import RaySampler
    o = O()
    from codenerf import synthetic
    K = synthetic.srn_intrinsics(24, focal=30.0)
    h = w = 24
    rs = RaySampler(h, w, K, sample_size=100, device=dev, datatype=torch.float32)
    c2w = o.pose_spherical(torch.tensor([0.5]), torch.tensor([0.3]), torch.tensor([1.3]))[None]
    gz = torch.Generator().manual_seed(3)
    z = torch.sort(0.8 + torch.rand(100, 9, generator=gz), dim=-1).values
    gp = torch.randn(100, 9, 3, generator=gz)
    np.random.seed(11)
    c_g = c2w.to(dev).requires_grad_(True)
    ro, rd, sel = rs.sample(c_g)
    from codenerf.nerf import PointSampler  # noqa: F401
    from codenerf.autograd import sample_points_autograd
    pts = sample_points_autograd(ro, rd, z.to(dev))
    ((pts * gp.to(dev)).sum() + (rd * 0.5).sum()).backward()
    c_c = c2w.clone().requires_grad_(True)
    dirs = o.ray_directions(h, w, K)
    ro_c, rd_c = o.ray_bundle(dirs, c_c)
    ro_c, rd_c = o.gather_rays(ro_c, rd_c, sel)
    pts_c = ro_c[:, None, :] + rd_c[:, None, :] * z[..., None]
    ((pts_c * gp).sum() + (rd_c * 0.5).sum()).backward()
    close(c_g.grad, c_c.grad, 1e-5, "d c2w")


# ---------------------------------------------------------------- field (forward_pass + CodeNeRFModel)


def _oracle_field(o, p, rd, pts, zs, zt, chunk, masks=None, pre_out=None):
    emb = o.EmbedCfg()
    s = pts.shape[1]
    outs, pres = [], []
    for c0 in range(0, rd.shape[0], chunk):
        c1 = min(c0 + chunk, rd.shape[0])
        mk = None if masks is None else {k: v[c0 * s:c1 * s] for k, v in masks.items()}
        pre = {} if pre_out is not None else None
        outs.append(o.forward_pass(p, emb, rd[c0:c1], pts[c0:c1], zs[c0:c1], zt[c0:c1], mk, pre))
        pres.append(pre)
    if pre_out is not None:
        for k in pres[0]:
            pre_out[k] = torch.cat([q[k] for q in pres])
    return torch.cat(outs)


# ReLU decisions a kernel recorded may differ from an independent fp32 forward only where the
# pre-activation is within that kernel's arithmetic error of 0: fp32 MFMA (reassociated sums)
# ~1e-6 relative, 3xbf16 ~2^-17 per product; MASK_BAND is relative to the layer's max |pre|.
MASK_BAND = {"f32": 1e-5, "bf16x3": 1e-4}


def explained_by_kinks(got, own, fed, what, rtol=GRAD_RTOL):
    """|got - own| <= |fed - own| + rtol * scale elementwise: the kernel's deviation from the oracle
    run on its own decisions is no larger than what the (in-band) differing decisions move."""
    got, own, fed = [torch.as_tensor(t).double().cpu() for t in (got, own, fed)]
    scale = own.abs().max().item() if own.numel() else 0.0
    excess = ((got - own).abs() - (fed - own).abs() - rtol * scale - 1e-7).max().item() if own.numel() else -1.0
    assert excess <= 0.0, f"{what}: deviation from the independent oracle exceeds the kinks' effect by {excess:.3e}"


def check_mask_agreement(masks, pre, band_rel, what=""):
    """Every ReLU decision in ``masks`` ((M, 256) 0/1 per layer) that disagrees with the oracle's own
    pre-activation ``pre`` must sit inside the error band; returns the number of disagreements."""
    n_dis = 0
    for k, m in masks.items():
        p = pre[k].double()
        own = p > 0
        dis = m.bool() != own
        scale = p.abs().max().item()
        bad = dis & (p.abs() >= band_rel * scale)
        assert not bool(bad.any()), (f"{what} layer {k}: {int(bad.sum())} ReLU decisions differ from the oracle "
                                     f"outside the band (max |pre| there {p.abs()[bad].max().item():.3e}, "
                                     f"band {band_rel * scale:.3e})")
        n_dis += int(dis.sum())
    return n_dis


def decode_relu_masks(words: torch.Tensor, m_rows: int):
    """cn_radiance_field_masks' ReLU decisions -> {"h1", "h2", "v1", "v2"}: (m_rows, 256) 0/1 floats.

    Layout (csrc/mlp_x3.hip store_masks / put_mask / conv_piece): per 128-sample tile, wave w,
    layer slot l (h1, h2, feat, v1, v2) and lane L, 4 words; bit b of word q is sample
    tile*128 + 32w + (L & 31), feature 32(2q + (b >> 4)) + (i & 3) + 8(i >> 2) + 4(L >> 5), i = b & 15.
    """
    w = words.detach().cpu().to(torch.int64) & 0xFFFFFFFF
    tiles = w.numel() // (4 * 5 * 64 * 4)
    bits = ((w.view(tiles, 4, 5, 64, 4, 1) >> torch.arange(32)) & 1).float()
    lane = torch.arange(64).view(64, 1, 1)
    q = torch.arange(4).view(1, 4, 1)
    b = torch.arange(32).view(1, 1, 32)
    i = b & 15
    feat = 32 * (2 * q + (b >> 4)) + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5)
    row = (lane & 31).expand(64, 4, 32)
    out = torch.zeros(tiles, 4, 5, 32, 256)
    out[:, :, :, row, feat] = bits
    out = out.permute(0, 1, 3, 2, 4).reshape(tiles * 128, 5, 256)[:m_rows]
    return {k: out[:, l].contiguous() for k, l in (("h1", 0), ("h2", 1), ("v1", 3), ("v2", 4))}


def decode_relu_masks_w16(words: torch.Tensor, m_rows: int):
    """The fp32 16x16x4 kernel's masks (csrc/mlp_f32.hip relu_act) -> {"h1", "h2", "v1", "v2"}.

    Layout: per 128-sample tile, wave w (8), layer l (h1, h2, v1, v2) and lane L, 2 words; bit b of
    word q is sample tile*128 + 16w + (L & 15), feature 16(8q + (b >> 2)) + 4(L >> 4) + (b & 3).
    """
    w = words.detach().cpu().to(torch.int64) & 0xFFFFFFFF
    tiles = w.numel() // (8 * 4 * 64 * 2)
    bits = ((w.view(tiles, 8, 4, 64, 2, 1) >> torch.arange(32)) & 1).float()
    lane = torch.arange(64).view(64, 1, 1)
    q = torch.arange(2).view(1, 2, 1)
    b = torch.arange(32).view(1, 1, 32)
    feat = 16 * (8 * q + (b >> 2)) + 4 * (lane >> 4) + (b & 3)
    row = (lane & 15).expand(64, 2, 32)
    out = torch.zeros(tiles, 8, 4, 16, 256)
    out[:, :, :, row, feat] = bits
    out = out.permute(0, 1, 3, 2, 4).reshape(tiles * 128, 4, 256)[:m_rows]
    return {k: out[:, l].contiguous() for k, l in (("h1", 0), ("h2", 1), ("v1", 2), ("v2", 3))}


@pytest.mark.parametrize("mode,r,s,chunk,per_ray_codes", [
    ("rayz", 37, 16, 13, False),
    ("pts", 37, 16, 37, False),
    ("rayz", 20, 9, 20, True),
    ("rayz", 300, 64, 128, False),
])
@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_field_backward(dev, mode, r, s, chunk, per_ray_codes, precision):
    """Training-mode backward (weights need grad): f32 -- the fused fp32 training pair; bf16x3 --
    the fp32 forward keeping activations and the layer-wise 3xbf16 GEMM backward (the fused 3xbf16
    training pair, whose ReLU decisions differ from fp32 inside the rounding band, is checked the
    three-way way in test_gpu_train.py::test_train_minibatch_matches_oracle)."""
    from codenerf import nerf, synthetic
    o = O()
    m = model(dev, 0)
    m.precision = "f32"
    m.train_precision = precision
    p = oracle_params(m)
    g = torch.Generator().manual_seed(r * s)
    ro = torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])
    rd = torch.randn(r, 3, generator=g)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values
    if per_ray_codes:
        zs, zt = torch.randn(r, 256, generator=g) * 0.3, torch.randn(r, 256, generator=g) * 0.3
    else:
        zs, zt = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    gout = torch.randn(r, s, 4, generator=g)

    # oracle
    ro_c, rd_c = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
    zs_c, zt_c = zs.clone().requires_grad_(True), zt.clone().requires_grad_(True)
    pts_c = ro_c[:, None, :] + rd_c[:, None, :] * z[..., None]
    zse = zs_c if per_ray_codes else zs_c.expand(r, -1)
    zte = zt_c if per_ray_codes else zt_c.expand(r, -1)
    raw_c = _oracle_field(o, p, rd_c, pts_c, zse, zte, chunk)
    (raw_c * gout).sum().backward()

    # HIP
    ro_g, rd_g = ro.to(dev).requires_grad_(True), rd.to(dev).requires_grad_(True)
    zs_g, zt_g = zs.to(dev).requires_grad_(True), zt.to(dev).requires_grad_(True)
    zsg = zs_g if per_ray_codes else zs_g.expand(r, -1)
    ztg = zt_g if per_ray_codes else zt_g.expand(r, -1)
    emb = embedders(dev)
    if mode == "pts":
        from codenerf.autograd import sample_points_autograd
        raw_g = nerf._field(m, emb, rd_g, zsg, ztg, chunk, pts=sample_points_autograd(ro_g, rd_g, z.to(dev)))
    else:
        raw_g = nerf._field(m, emb, rd_g, zsg, ztg, chunk, ro=ro_g, z=z.to(dev))
    (raw_g * gout.to(dev)).sum().backward()

    assert (raw_g.detach().cpu() - raw_c.detach()).abs().max().item() <= 1e-4
    close(ro_g.grad, ro_c.grad, what="d ro")
    close(rd_g.grad, rd_c.grad, what="d rd")
    close(zs_g.grad, zs_c.grad, what="d z_s")
    close(zt_g.grad, zt_c.grad, what="d z_t")
    for (name, prm) in m.named_parameters():
        close(prm.grad, p[name].grad, what=name)


@pytest.mark.parametrize("mode,r,s,chunk,per_ray_codes", [
    ("rayz", 37, 16, 13, False),
    ("pts", 37, 16, 37, False),
    ("rayz", 20, 32, 20, True),
    ("rayz", 300, 64, 128, False),
    ("rayz", 64, 128, 64, False),
    ("rayz", 21, 16, 21, True),   # per-ray codes, 16-sample rays: fused for f32 (16-sample waves) only
    ("rayz", 20, 9, 20, True),    # codes change inside a wave: layer-wise fp32 path
    ("pts", 150, 7, 50, False),   # ragged: samples not a multiple of the wave, last tile partial
])
@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_field_backward_eval_fused(dev, monkeypatch, mode, r, s, chunk, per_ray_codes, precision):
    """Frozen model (the eval step): the forward with ReLU masks and ONE fused backward launch
    (cn_field_backward_fused: fp32 16x16x4 for "f32", 3xbf16 for "bf16x3") give the oracle's d ro /
    d rd / d z_s / d z_t.

    Checked three ways: (1) against the oracle with its own ReLU decisions (INDEPENDENT_RTOL);
    (2) every ReLU decision the kernel's forward recorded (decode_relu_masks) equals the oracle's
    own except where |pre-activation| is inside the 3xbf16 error band (check_mask_agreement); (3)
    with those recorded decisions, the oracle's gradients match at GRAD_RTOL -- a pre-activation
    within the kernel's error of 0 can fall on the other side of the kink, which moves that
    sample's gradient by a whole weight column."""
    from codenerf import nerf, ops, synthetic
    calls = {"fused": 0, "masks": None}
    real_bwd, real_fwd = ops.field_backward_x3, ops.radiance_field_masks

    def spy_bwd(*a, **k):
        calls["fused"] += 1
        return real_bwd(*a, **k)

    def spy_fwd(*a, **k):
        raw, masks = real_fwd(*a, **k)
        calls["masks"] = masks
        return raw, masks
    monkeypatch.setattr(ops, "field_backward_x3", spy_bwd)
    monkeypatch.setattr(ops, "radiance_field_masks", spy_fwd)
    o = O()
    m = model(dev, 0)
    p = oracle_params(m)
    m.precision = precision
    m.requires_grad_(False)
    fused = (not per_ray_codes) or s % (32 if precision == "bf16x3" else 16) == 0
    g = torch.Generator().manual_seed(r * s + 7)
    ro = torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])
    rd = torch.randn(r, 3, generator=g)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values
    if per_ray_codes:
        zs, zt = torch.randn(r, 256, generator=g) * 0.3, torch.randn(r, 256, generator=g) * 0.3
    else:
        zs, zt = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    gout = torch.randn(r, s, 4, generator=g)

    ro_g, rd_g = ro.to(dev).requires_grad_(True), rd.to(dev).requires_grad_(True)
    zs_g, zt_g = zs.to(dev).requires_grad_(True), zt.to(dev).requires_grad_(True)
    zsg = zs_g if per_ray_codes else zs_g.expand(r, -1)
    ztg = zt_g if per_ray_codes else zt_g.expand(r, -1)
    emb = embedders(dev)
    if mode == "pts":
        from codenerf.autograd import sample_points_autograd
        raw_g = nerf._field(m, emb, rd_g, zsg, ztg, chunk, pts=sample_points_autograd(ro_g, rd_g, z.to(dev)))
    else:
        raw_g = nerf._field(m, emb, rd_g, zsg, ztg, chunk, ro=ro_g, z=z.to(dev))
    (raw_g * gout.to(dev)).sum().backward()
    assert calls["fused"] == (1 if fused else 0)
    decode = decode_relu_masks if precision == "bf16x3" else decode_relu_masks_w16
    masks = decode(calls["masks"], r * s) if fused else None

    pd = {k: v.detach() for k, v in p.items()}

    def oracle(mk, pre=None):
        ro_c, rd_c = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
        zs_c, zt_c = zs.clone().requires_grad_(True), zt.clone().requires_grad_(True)
        pts_c = ro_c[:, None, :] + rd_c[:, None, :] * z[..., None]
        zse = zs_c if per_ray_codes else zs_c.expand(r, -1)
        zte = zt_c if per_ray_codes else zt_c.expand(r, -1)
        raw_c = _oracle_field(o, pd, rd_c, pts_c, zse, zte, chunk, mk, pre)
        (raw_c * gout).sum().backward()
        return raw_c.detach(), ro_c.grad, rd_c.grad, zs_c.grad, zt_c.grad

    # 1. the oracle with its OWN ReLU decisions, independent of anything the kernel recorded
    pre = {}
    own = oracle(None, pre)
    assert (raw_g.detach().cpu() - own[0]).abs().max().item() <= 1e-4
    got = (ro_g.grad, rd_g.grad, zs_g.grad, zt_g.grad)
    if not fused:
        for g_, ref, what in zip(got, own[1:], ("ro", "rd", "z_s", "z_t")):
            close(g_, ref, what="d " + what)
        return
    # 2. the kernel's recorded decisions equal the oracle's except inside the 3xbf16 band ...
    n_dis = check_mask_agreement(masks, pre, MASK_BAND[precision], "fused forward")
    print(f"ReLU decisions differing from the oracle (all in-band): {n_dis}")
    # 3. ... and with exactly those decisions the oracle's gradients match tightly
    fed = oracle(masks)
    for g_, ref, what in zip(got, fed[1:], ("ro", "rd", "z_s", "z_t")):
        close(g_, ref, what="d " + what)
    # so every deviation from the independent oracle is what those in-band kinks move
    for g_, ref, alt, what in zip(got, own[1:], fed[1:], ("ro", "rd", "z_s", "z_t")):
        explained_by_kinks(g_, ref, alt, "d " + what)
    if n_dis == 0:
        for g_, ref, what in zip(got, own[1:], ("ro", "rd", "z_s", "z_t")):
            close(g_, ref, what="d " + what + " (independent)")


@pytest.mark.parametrize("m_rows,dedupe", [(1000, True), (257, False)])
def test_model_forward_backward(dev, m_rows, dedupe):
    """CodeNeRFModel(z_s, z_t, x) with grads on x, codes and weights (model.py:160-194)."""
    o = O()
    m = model(dev, 1)
    p = oracle_params(m)
    g = torch.Generator().manual_seed(m_rows)
    x = torch.randn(m_rows, 90, generator=g)
    if dedupe:
        zs, zt = torch.randn(1, 256, generator=g) * 0.3, torch.randn(1, 256, generator=g) * 0.3
    else:
        zs, zt = torch.randn(m_rows, 256, generator=g) * 0.3, torch.randn(m_rows, 256, generator=g) * 0.3
    gout = torch.randn(m_rows, 4, generator=g)
    xc, zsc, ztc = [t.clone().requires_grad_(True) for t in (x, zs, zt)]
    e = (lambda t: t.expand(m_rows, -1)) if dedupe else (lambda t: t)
    (o.codenerf_mlp(p, e(zsc), e(ztc), xc, 63) * gout).sum().backward()
    xg, zsg, ztg = [t.to(dev).requires_grad_(True) for t in (x, zs, zt)]
    raw = m(e(zsg), e(ztg), xg)
    (raw * gout.to(dev)).sum().backward()
    close(xg.grad, xc.grad, what="d x")
    close(zsg.grad, zsc.grad, what="d z_s")
    close(ztg.grad, ztc.grad, what="d z_t")
    for (name, prm) in m.named_parameters():
        close(prm.grad, p[name].grad, what=name)


# ---------------------------------------------------------------- the reference's eval step (C5)


def test_eval_step_gradients_golden(dev):
    """eval.py:145-160 through the whole path, vs the reference's own autograd (eval_grad.npz)."""
    from codenerf import synthetic
    from codenerf.evaluate import pose_spherical
    from codenerf.nerf import PointSampler, RaySampler, predict_radiance_and_render
    gd = {k: torch.from_numpy(v) for k, v in np.load(os.path.join(GOLDEN, "eval_grad.npz")).items()}
    K = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays_small.npz"))["intrinsics"])
    models = {"nerf_coarse": model(dev, 0), "nerf_fine": model(dev, 1)}
    for mm in models.values():
        mm.train()
    emb = embedders(dev)
    ps = PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    rs = RaySampler(12, 16, K, sample_size=64, device=dev, datatype=torch.float32)
    theta, phi, rho = [gd[k].to(dev).requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = gd["z_s"].to(dev).requires_grad_(True), gd["z_t"].to(dev).requires_grad_(True)
    target = gd["target"].to(dev)
    np.random.seed(9)
    c2w = pose_spherical(theta, phi, rho)[None, :]
    ro, rd, sel = rs.sample(tform_cam2world=c2w)
    assert np.array_equal(sel, gd["select_inds"].numpy())
    tp = target[None][..., torch.as_tensor(sel, device=dev), :].squeeze()
    zse, zte = zs.expand(ro.shape[0], -1), zt.expand(ro.shape[0], -1)
    rgb_c, rgb_f = predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                               (zse, zte))
    assert (rgb_c.detach().cpu() - gd["rgb_coarse"]).abs().max().item() <= 1e-4
    assert (rgb_f.detach().cpu() - gd["rgb_fine"]).abs().max().item() <= 1e-4
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    assert abs(loss.item() - gd["loss"].item()) <= 1e-5
    for name, t in [("theta", theta), ("phi", phi), ("rho", rho)]:
        ref = gd["g_" + name]
        assert (t.grad.cpu() - ref).abs().max().item() <= 1e-3 * max(1.0, ref.abs().max().item()), name
    close(zs.grad, gd["g_z_s"], 1e-3, "g_z_s")
    close(zt.grad, gd["g_z_t"], 1e-3, "g_z_t")
    close(models["nerf_fine"].fc_rgb.weight.grad, gd["g_fine_fc_rgb_w"], 1e-3, "fine fc_rgb.weight")
    close(models["nerf_coarse"].fc_out.bias.grad, gd["g_coarse_fc_out_b"], 1e-3, "coarse fc_out.bias")
    for key, mm in models.items():
        for n, prm in mm.named_parameters():
            ref = gd[f"gnorm_{key}.{n}"].item()
            assert abs(prm.grad.norm().item() - ref) <= 1e-3 * ref + 1e-8, (key, n)


def test_test_time_optimize_runs(dev):
    """A few iterations of the eval loop run end to end on the HIP path and move codes and pose."""
    from codenerf.evaluate import test_time_optimize
    from codenerf.nerf import PointSampler, RaySampler
    K = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays_small.npz"))["intrinsics"])
    models = {"nerf_coarse": model(dev, 0), "nerf_fine": model(dev, 1)}
    emb = embedders(dev)
    ps = PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    rs = RaySampler(12, 16, K, sample_size=64, device=dev, datatype=torch.float32)
    target = torch.rand(12 * 16, 4, generator=torch.Generator().manual_seed(1)).to(dev)
    codes = (torch.randn(4, 256) * 0.3, torch.randn(4, 256) * 0.3)
    np.random.seed(0)
    zs, zt, (theta, phi, rho), hist, cam = test_time_optimize(target, (rs, ps), emb, models, codes, iterations=6,
                                                              val_lr=5e-2)
    assert cam.shape == (1, 4, 4)
    assert len(hist) == 6 and np.isfinite([h["total_loss"] for h in hist]).all()
    assert not torch.allclose(zs.detach().cpu(), codes[0].mean(0, keepdim=True))
    assert abs(theta.item() - 1.57) > 1e-4 and abs(rho.item() - 1.30) > 1e-4
    assert all(p.requires_grad for mm in models.values() for p in mm.parameters())



@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("mode,far", [("rayz", False), ("pts", False), ("pts", True), ("rayz", True)])
def test_field_backward_train_generated_encodings(dev, mode, far, precision):
    """The fused training backward's encoding-layer dW (layer_xyz1, layer_dir1's view columns) with
    the encodings generated inside the dW kernel (x_enc None, the training path) matches the
    x_enc-plane GEMMs at GEMM_TOL; every other gradient is the same deterministic computation and
    must agree bit for bit.  Run twice: the generated path is bitwise reproducible.  ``far``: samples
    past fast_sincosf's argument bound (pts: ONE sample of one 16-sample wave -- a mixed wave, which
    the fp32 forward and its dW kernel evaluate with sincosf throughout; rayz: one far ray), so both
    per-stage choices of the dW kernel run."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    r, s, chunk = 300, 64, 128
    g = torch.Generator().manual_seed(5)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    if far and mode == "rayz":
        ro[37] = torch.tensor([45.0, -38.0, 41.0], device=dev)
    pts = (ro[:, None, :] + rd[:, None, :] * z[..., None]).contiguous() if mode == "pts" else None
    if far and mode == "pts":
        pts[37, 5] = torch.tensor([45.0, -38.0, 41.0], device=dev)
    geo = dict(pts=pts) if mode == "pts" else dict(ro=ro, z=z)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    x3 = precision == "bf16x3"
    _, saved, masks = ops.radiance_field_train_w16(ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16"), cb, rd, s,
                                                   chunk, fx, fd, precision=precision, **geo)
    x_enc = ops.encode_inputs(rd, s, chunk, fx, fd, **geo)
    packed_t = ops.mlp_pack(params, "bf16x3_t" if x3 else "f32_w16_t")
    out = {}
    for name, xe in (("plane", x_enc), ("generated", None), ("generated2", None)):
        pg = [torch.zeros_like(p) for p in params]
        ops.field_backward_train(packed_t, params, masks, saved, xe, gout, r, s, chunk, 1, fx, fd, rd=rd,
                                 param_grads=pg, precision=precision, **geo)
        out[name] = pg
    # weights: layer_xyz1 0, layer_xyz2 2, fc_out 4, layer_dir1 12, layer_dir2 14, fc_rgb 16 (dW GEMMs,
    # deterministic); the biases are fixed-order column sums whose grouping follows the dW launches the
    # encoding source selects (checked to fp32 rounding across sources); every gradient is reproducible
    # bit for bit (one code row: no float atomics in the step, either precision)
    enc_layers, weights = {0, 12}, {0, 2, 4, 12, 14, 16}
    for k, (a, b) in enumerate(zip(out["generated"], out["plane"])):
        if k in enc_layers:
            close(a, b.double(), GEMM_TOL[precision], f"param {k} generated vs plane")
        elif k in weights:
            assert torch.equal(a, b), f"param {k}: non-encoding weight gradient changed"
        else:
            close(a, b.double(), 1e-5, f"bias {k}")
        assert torch.equal(a, out["generated2"][k]), f"param {k}: not reproducible"


@pytest.mark.parametrize("mode,r,s,chunk", [("rayz", 1056, 64, 256),   # 5 Q1 chunks, the last 32 rays
                                             ("rayz", 1056, 80, 4096),  # unit runs straddle direction groups
                                             ("pts", 4096, 32, 1024),
                                             ("rayz", 4096, 24, 1024),  # S < 32: unfolded path
                                             ("rayz", 1050, 64, 256)])  # n_rays % 16 != 0: unfolded path
def test_field_backward_train_dir1_fold(dev, mode, r, s, chunk):
    """At M >= 65536 (fp32) layer_dir1's view-encoding dW and bias come from per-direction column
    sums of its dPre plane taken during the [feat] pass (gemm_tn256_kernel DIRS +
    dir_enc_dw_kernel): the Q1 map makes rows j rcnt + d of a chunk share direction d.  Checked
    against the x_enc-plane GEMMs (the encodings as the forward made them) at GEMM_TOL; every other
    gradient is the same products, at fp32 rounding: with generated encodings layer_xyz1's dW joins the
    batched dW launch (grad.hip xenc_role_enabled), whose split of rows over the jobs -- so the other
    weights' partial-tile grouping -- follows its job list; two runs are bitwise identical."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    g = torch.Generator().manual_seed(r + s)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    pts = (ro[:, None, :] + rd[:, None, :] * z[..., None]).contiguous() if mode == "pts" else None
    geo = dict(pts=pts) if mode == "pts" else dict(ro=ro, z=z)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    _, saved, masks = ops.radiance_field_train_w16(ops.mlp_pack(params, "f32_w16"), cb, rd, s, chunk, fx, fd,
                                                   precision="f32", **geo)
    x_enc = ops.encode_inputs(rd, s, chunk, fx, fd, **geo)
    packed_t = ops.mlp_pack(params, "f32_w16_t")
    out = {}
    for name, xe in (("plane", x_enc), ("folded", None), ("folded2", None)):
        pg = [torch.zeros_like(p) for p in params]
        ops.field_backward_train(packed_t, params, masks, saved, xe, gout, r, s, chunk, 1, fx, fd, rd=rd,
                                 param_grads=pg, precision="f32", **geo)
        out[name] = pg
    # layer_xyz1 0 (generated encodings), layer_dir1 12 / its bias 13 (the fold) vs the plane GEMMs
    for k, (a, b) in enumerate(zip(out["folded"], out["plane"])):
        if k in (0, 12):
            close(a, b.double(), GEMM_TOL["f32"], f"param {k} folded vs plane")
        elif k == 13:
            close(a, b.double(), 1e-5, "layer_dir1 bias")
        else:
            close(a, b.double(), 1e-5, f"param {k}")
        assert torch.equal(a, out["folded2"][k]), f"param {k}: not reproducible"


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_field_backward_train_sigma_rgb_rows(dev, precision):
    """At M >= 65536 the fused training backward folds fc_out's sigma row (d sigma^T h2) into the
    whole-tile dW kernel's h2 stream; with fc_rgb's rows (d rgb^T v2) it is checked against fp64
    products of the forward's own saved planes and the d raw it was given (no oracle needed:
    the planes are the exact operands)."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    r, s = 1100, 64                              # M = 70400
    g = torch.Generator().manual_seed(9)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    x3 = precision == "bf16x3"
    _, saved, masks = ops.radiance_field_train_w16(ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16"), cb, rd, s,
                                                   4096, fx, fd, ro=ro, z=z, precision=precision)
    pg = [torch.zeros_like(p) for p in params]
    ops.field_backward_train(ops.mlp_pack(params, "bf16x3_t" if x3 else "f32_w16_t"), params, masks, saved, None,
                             gout, r, s, 4096, 1, fx, fd, rd=rd, ro=ro, z=z, param_grads=pg, precision=precision)
    d = gout.reshape(-1, 4).double().cpu()
    h2, v2 = saved[1].double().cpu(), saved[4].double().cpu()
    close(pg[4][0, :256], d[:, 3] @ h2, 1e-5, "fc_out sigma row")      # kWOut = 4
    close(pg[16][:, :256], d[:, :3].t() @ v2, 1e-5, "fc_rgb rows")     # kWRgb = 16


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("mode,r,s,n_codes", [("rayz", 1050, 64, 1),    # 525 tiles: 2-3 per workgroup, ragged
                                              ("rayz", 4096, 64, 1),    # C3-shaped: 8 tiles per workgroup
                                              ("pts", 777, 48, 1),
                                              ("rayz", 5, 16, 1),       # one (partial) tile
                                              ("rayz", 300, 24, 1),     # S % 16 != 0
                                              ("rayz", 1024, 64, 3)])   # in-kernel g_code sums
def test_field_backward_train_nogeo_bitwise(dev, precision, mode, r, s, n_codes):
    """train.py's rays are data (ray_sampler.py:53-82), so the training backward is asked for no d ro /
    d rd / d pts, and the fused kernel then skips the geometry-only chunks (view-direction rows of
    layer_dir1^T, both layer_xyz1^T chunks) and the encoding epilogue, storing layer_xyz1's dPre plane
    beside the next tile's fc_rgb^T.  Every weight and code gradient must be bitwise those of the
    geometry schedule on the same chunk (one code row: deterministic throughout, in both precisions --
    g_code is the dPre planes' column sums folded into the dW GEMMs; several: the per-code sums are float
    atomics, so g_code and the three biases formed from it agree to fp32 rounding)."""
    from codenerf import ops, synthetic
    if precision == "bf16x3" and s % 32:
        pytest.skip("3xbf16 fused backward: one code row per 32-sample wave")
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    g = torch.Generator().manual_seed(r + s + n_codes)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    pts = (ro[:, None, :] + rd[:, None, :] * z[..., None]).contiguous() if mode == "pts" else None
    geo = dict(pts=pts) if mode == "pts" else dict(ro=ro, z=z)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, n_codes).to(dev), synthetic.latent_codes(6, n_codes).to(dev)
    code_index = (torch.arange(r) * n_codes // r).to(dev) if n_codes > 1 else None
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    x3 = precision == "bf16x3"
    chunk = 256
    _, saved, masks = ops.radiance_field_train_w16(ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16"), cb, rd, s,
                                                   chunk, fx, fd, precision=precision, code_index=code_index, **geo)
    packed_t = ops.mlp_pack(params, "bf16x3_t" if x3 else "f32_w16_t")
    want = dict(want_pts=True) if mode == "pts" else dict(want_ro=True, want_rd=True)
    out = {}
    for name, w in (("geo", want), ("nogeo", {}), ("nogeo2", {})):
        pg = [torch.zeros_like(p) for p in params]
        res = ops.field_backward_train(packed_t, params, masks, saved, None, gout, r, s, chunk, n_codes, fx, fd, rd=rd,
                                       code_index=code_index, param_grads=pg, precision=precision, **w, **geo)
        out[name] = (pg, res["g_code"])
    torch.cuda.synchronize()
    atomic = n_codes > 1             # the per-code sums / biases of g_code: float atomics
    code_biases = {3, 5, 17}          # b_xyz2, b_out, b_rgb: column sums of g_code
    # float-atomic sums over ~67k samples whose partial sums exceed the total (cancellation): two orders
    # agree to 1e-5 of the total's magnitude in fp32; 3xbf16 (larger per-sample terms) measured 1.27e-5
    # (gpurun_out/r05n), bound at 2x that
    tol = 2.6e-5 if x3 else 1e-5
    for other in ("nogeo", "nogeo2"):
        for k, (a, b) in enumerate(zip(out[other][0], out["geo"][0])):
            if atomic and k in code_biases:
                close(a, b.double(), tol, f"bias {k}")
            else:
                assert torch.equal(a, b), f"param {k}: {other} differs from the geometry schedule"
        if atomic:
            from conftest import margin
            err = (out[other][1].double() - out["geo"][1].double()).abs().max().item()
            scale = max(out["geo"][1].abs().max().item(), 1e-30)
            margin(f"nogeo_bitwise[{precision},{r}x{s},codes{n_codes}]", f"g_code {other} vs geo (rel. max)",
                   err / scale, tol + 1e-7 / scale)
            close(out[other][1], out["geo"][1].double(), tol, "g_code")
        else:
            assert torch.equal(out[other][1], out["geo"][1]), f"g_code: {other}"


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("mode,r,s,chunk", [("rayz", 300, 64, 128),   # 3 Q1 chunks, the last one short
                                            ("rayz", 64, 128, 64),
                                            ("rayz", 2048, 64, 2048),  # C5's coarse pass
                                            ("pts", 37, 32, 37)])
def test_fused_backward_deterministic(dev, precision, mode, r, s, chunk):
    """The eval backward without float atomics (cn_field_backward_fused_ws, the default of
    ops.field_backward_x3 for one code row and whole waves per ray): per-wave g_code rows, per-wave
    ray rows and per-sample Q1 terms summed in a fixed order.  Two runs give the same bits; the
    float-atomic kernel agrees to fp32 reassociation; d ro / d rd are ADDED into given tensors."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    x3 = precision == "bf16x3"
    g = torch.Generator().manual_seed(r + s + chunk)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    pts = (ro[:, None, :] + rd[:, None, :] * z[..., None]).contiguous() if mode == "pts" else None
    geo = dict(pts=pts) if mode == "pts" else dict(ro=ro, z=z)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    _, masks = ops.radiance_field_masks(ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16"), cb, rd, s, chunk, fx,
                                        fd, precision=precision, **geo)
    packed_t = ops.mlp_pack(params, "bf16x3_t" if x3 else "f32_w16_t")
    want = dict(want_pts=True, want_rd=True) if mode == "pts" else dict(want_ro=True, want_rd=True)

    def run(det, **kw):
        out = ops.field_backward_x3(packed_t, masks, gout, r, s, chunk, 1, fx, fd, rd, precision=precision,
                                    deterministic=det, **geo, **want, **kw)
        return {k: v.clone() for k, v in out.items() if v is not None}
    a, b, c = run(True), run(True), run(False)
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), f"{k}: two deterministic runs differ"
        close(a[k], c[k].double(), 1e-5, f"{k} vs the float-atomic kernel")
    if mode == "rayz":
        base = (torch.randn(r, 3, generator=g).to(dev), torch.randn(r, 3, generator=g).to(dev))
        into = (base[0].clone(), base[1].clone())
        run(True, ray_into=into)
        assert torch.equal(into[0], base[0] + a["d_ro"]) and torch.equal(into[1], base[1] + a["d_rd"])


@pytest.mark.parametrize("n_codes,want_grads", [(1, True), (5, True), (5, False)])
def test_code_bias_backward_two_launch_bitwise(dev, n_codes, want_grads):
    """cn_code_bias_backward_ws (code layers split over 64 workgroups per code, two launches) gives
    bitwise the results of the single-launch cn_code_bias_backward: dz_s, dz_t, and with one code
    every accumulated parameter gradient (with several codes both add their float atomics in no
    fixed order: 1e-6 relative); a code no sample used (g row zero) gets dz = 0.  accumulate_dz
    (dz_into): the same dz added onto what the rows held, bit for bit, an unused code's rows kept."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    g = torch.Generator().manual_seed(n_codes)
    zs, zt = synthetic.latent_codes(5, n_codes).to(dev), synthetic.latent_codes(6, n_codes).to(dev)
    stride = ops.code_bias(params, zs, zt).shape[1]
    gc = (torch.randn(n_codes, stride, generator=g) * 1e-2).to(dev)
    if n_codes > 1:
        gc[1] = 0.0                                   # an unused code row
    out = {}
    for single in (True, False):
        pg = [torch.full_like(p, 0.5) for p in params] if want_grads else None
        dz_s, dz_t = ops.code_bias_backward(params, zs, zt, gc, pg, want_z=True, single_launch=single)
        out[single] = (dz_s, dz_t, pg)
    a, b = out[True], out[False]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    if n_codes > 1:
        assert not b[0][1].any() and not b[1][1].any()
    base = [(torch.randn(n_codes, 256, generator=g) * 1e-2).to(dev) for _ in range(2)]
    into = [t.clone() for t in base]
    r = ops.code_bias_backward(params, zs, zt, gc, None, dz_into=tuple(into))
    assert r[0] is into[0] and r[1] is into[1]
    assert torch.equal(into[0], base[0] + b[0]) and torch.equal(into[1], base[1] + b[1])
    if want_grads:
        for k, (x, y) in enumerate(zip(a[2], b[2])):
            if n_codes == 1:
                assert torch.equal(x, y), f"param {k}"
            else:
                # each of the n_codes atomic adds onto the 0.5 fill rounds at the fill's ulp (2^-24
                # near 0.5): two orders differ by up to n_codes ulps, whatever the gradient's scale
                err = (x.double() - y.double()).abs().max().item()
                assert err <= n_codes * 2.0 ** -23, f"param {k}: max err {err:.3e}"


@pytest.mark.parametrize("n_codes", [1, 5])
@pytest.mark.parametrize("pack,pack_t", [(True, True), (False, True), (False, False)])
def test_field_prepare_bitwise(dev, n_codes, pack, pack_t):
    """cn_field_prepare (the fp32 training step's one pre-field launch per model: code terms, both packs,
    a zeroed g_code) equals the separate cn_code_bias / cn_mlp_pack calls bit for bit."""
    from codenerf import ops, synthetic
    m = model(dev, 2)
    params = [p.detach() for p in m.param_list()]
    zs, zt = synthetic.latent_codes(7, n_codes).to(dev), synthetic.latent_codes(8, n_codes).to(dev)
    nz = n_codes * 520 + 3
    cb, pk, pkt, zero = ops.field_prepare(params, zs, zt, pack=pack, pack_t=pack_t, n_zero=nz)
    assert torch.equal(cb, ops.code_bias(params, zs, zt))
    assert (pk is None) == (not pack) and (pkt is None) == (not pack_t)
    if pack:
        assert torch.equal(pk, ops.mlp_pack(params, "f32_w16"))
    if pack_t:
        assert torch.equal(pkt, ops.mlp_pack(params, "f32_w16_t"))
    assert zero.shape == (nz,) and not zero.any()


@pytest.mark.parametrize("n_codes,want_grads", [(1, True), (4, True), (4, False)])
def test_code_backward_on_forward_activations(dev, n_codes, want_grads):
    """The code backward on the preparation launch's code-layer activations (cn_code_bias_backward_act +
    cn_code_dz): the activations are relu(W z + b) of the code layers (1e-6), dz and every parameter
    gradient agree with the recomputing two-launch form to fp32 rounding (the two dot orders of the
    activations differ in the last bits), an unused code gets dz = 0, and cn_code_dz over two fields
    equals the one-field launches added in the same order, bit for bit."""
    from codenerf import ops, synthetic
    m = model(dev, 0)
    params = [p.detach() for p in m.param_list()]
    pd = {n: p.detach() for n, p in m.named_parameters()}
    g = torch.Generator().manual_seed(40 + n_codes)
    zs, zt = synthetic.latent_codes(11, n_codes).to(dev), synthetic.latent_codes(12, n_codes).to(dev)
    ((cb, _, _, _, act),) = ops.field_prepare_models([(params, False, False, 0)], zs, zt, want_act=True)
    assert torch.equal(cb, ops.code_bias(params, zs, zt))
    ref_act = torch.cat([torch.relu(zs @ pd["shape_code_layer1.weight"].T + pd["shape_code_layer1.bias"]),
                         torch.relu(zs @ pd["shape_code_layer2.weight"].T + pd["shape_code_layer2.bias"]),
                         torch.relu(zt @ pd["texture_code_layer1.weight"].T + pd["texture_code_layer1.bias"])], 1)
    close(act, ref_act, 1e-6, "code_act")
    gc = (torch.randn(n_codes, cb.shape[1], generator=g) * 1e-2).to(dev)
    if n_codes > 1:
        gc[1] = 0.0
    pg_old = [torch.full_like(p, 0.5) for p in params] if want_grads else None
    dz_old = ops.code_bias_backward(params, zs, zt, gc, pg_old, want_z=True)
    pg_new = [torch.full_like(p, 0.5) for p in params] if want_grads else None
    ws = ops.code_ds_outer(params, zs, zt, act, gc, pg_new)
    dz_new = ops.code_dz([(params, gc, ws)], n_codes)
    for a, b, k in zip(dz_new, dz_old, ("dz_s", "dz_t")):
        close(a, b, 1e-5, k)
    if n_codes > 1:
        assert not dz_new[0][1].any() and not dz_new[1][1].any()
    if want_grads:
        for k, (x, y) in enumerate(zip(pg_new, pg_old)):
            close(x - 0.5, y - 0.5, 1e-5, f"param {k}")
    # two fields in one cn_code_dz launch == the one-field launches in the same order
    m2 = model(dev, 1)
    params2 = [p.detach() for p in m2.param_list()]
    ((_, _, _, _, act2),) = ops.field_prepare_models([(params2, False, False, 0)], zs, zt, want_act=True)
    gc2 = (torch.randn(n_codes, cb.shape[1], generator=g) * 1e-2).to(dev)
    ws2 = ops.code_ds_outer(params2, zs, zt, act2, gc2)
    both = ops.code_dz([(params, gc, ws), (params2, gc2, ws2)], n_codes)
    base = [(torch.randn(n_codes, 256, generator=g) * 1e-2).to(dev) for _ in range(2)]
    into = tuple(t.clone() for t in base)
    ops.code_dz([(params, gc, ws), (params2, gc2, ws2)], n_codes, dz_into=into)
    one = ops.code_dz([(params, gc, ws)], n_codes)
    seq = ops.code_dz([(params2, gc2, ws2)], n_codes, dz_into=tuple(t.clone() for t in one))
    for a, b in zip(both, seq):
        assert torch.equal(a, b)
    step = tuple(t.clone() for t in base)
    ops.code_dz([(params, gc, ws)], n_codes, dz_into=step)
    ops.code_dz([(params2, gc2, ws2)], n_codes, dz_into=step)
    for a, b in zip(into, step):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n_codes", [1, 3])
def test_field_prepare_models_bitwise(dev, n_codes):
    """cn_field_prepare_models (a render's coarse and fine fields prepared in one launch) equals each
    model's cn_field_prepare bit for bit, with different pack / zero requests per model."""
    from codenerf import ops, synthetic
    ps = [[p.detach() for p in model(dev, s).param_list()] for s in (3, 4)]
    zs, zt = synthetic.latent_codes(9, n_codes).to(dev), synthetic.latent_codes(10, n_codes).to(dev)
    reqs = [(ps[0], True, False, n_codes * 520), (ps[1], False, True, 777)]
    got = ops.field_prepare_models(reqs, zs, zt)
    for (params, pack, pack_t, nz), out in zip(reqs, got):
        ref = ops.field_prepare(params, zs, zt, pack=pack, pack_t=pack_t, n_zero=nz)
        for a, b in zip(out, ref):
            assert (a is None) == (b is None)
            if a is not None:
                assert torch.equal(a, b)


@pytest.mark.parametrize("far", [False, True])
@pytest.mark.parametrize("mode", ["rayz", "pts"])
def test_training_forward_encoding_plane(dev, mode, far):
    """The fp32 training forward's (M, 64) encoding plane (after the five activation planes; the
    layer_xyz1 dW reads it instead of regenerating the encodings): mapped through xenc_col it is the
    positional encoding of the sample points (position_embed.py:44-53) -- the oracle's to 2e-6 (both
    within ~2 ulp of sin / cos) -- and the padding slot is zero.  ``far``: one 16-sample wave with a
    point past fast_sincosf's bound (that wave takes ocml's sincosf throughout)."""
    from codenerf import ops, synthetic
    from oracle import codenerf_oracle as Or
    m_ = model(dev, 0)
    params = [p.detach() for p in m_.param_list()]
    r, s = 300, 64
    g = torch.Generator().manual_seed(17)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3]))
    rd = torch.randn(r, 3, generator=g)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values
    pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
    if far:
        pts[37, 5] = torch.tensor([45.0, -38.0, 41.0])
    geo = dict(pts=pts.to(dev)) if mode == "pts" or far else dict(ro=ro.to(dev), z=z.to(dev))
    if mode == "rayz" and far:
        ro2 = ro.clone()
        ro2[37] = torch.tensor([45.0, -38.0, 41.0])
        pts = ro2[:, None, :] + rd[:, None, :] * z[..., None]
        geo = dict(ro=ro2.to(dev), z=z.to(dev))
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    _, saved, _ = ops.radiance_field_train_w16(ops.mlp_pack(params, "f32_w16"), cb, rd.to(dev), s, r, fx, fd,
                                               precision="f32", **geo)
    m = r * s
    plane = torch.empty(0, device=dev).set_(saved.untyped_storage(), 5 * m * 256, (m, 64)).cpu()
    cols = ops.xenc_columns()
    ref = Or.posenc(pts.reshape(-1, 3), Or.frequency_bands(10, True), True)
    got = torch.zeros(m, 63)
    for cp, c in enumerate(cols):
        if c >= 0:
            got[:, c] = plane[:, cp]
        else:
            assert not plane[:, cp].any(), "padding slot"
    assert (got - ref).abs().max().item() <= 2e-6


@pytest.mark.parametrize("r,sc,sf", [(2048, 64, 128), (4096, 32, 160), (300, 16, 32)])
def test_fused_backward_pair_bitwise(dev, r, sc, sf):
    """cn_field_backward_fused_multi (the eval step's two fields on the same rays: one dX launch, one ray /
    g_code-row launch, one g_code reduction) against the two per-field deterministic calls with the
    in-between d rd added between them: g_code of both fields, d ro and d rd bit for bit.  Also the
    paired code backward first halves (cn_code_bias_backward_act_multi) against two single calls."""
    from codenerf import ops, synthetic
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    g = torch.Generator().manual_seed(r + sc)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    between = torch.randn(r, 3, generator=g).to(dev)
    start = torch.randn(2, r, 3, generator=g).to(dev)
    fields, acts = [], []
    for seed, s in ((1, sf), (0, sc)):                      # fine first, as the eval step's pair runs them
        m = model(dev, seed)
        params = [p.detach() for p in m.param_list()]
        z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
        (cb, _, _, _, act), = ops.field_prepare_models([(params, False, False, 0)], zs, zt, want_act=True)
        _, masks = ops.radiance_field_masks(ops.mlp_pack(params, "f32_w16"), cb, rd, s, r, fx, fd, ro=ro, z=z,
                                            precision="f32")
        fields.append(dict(packed_t=ops.mlp_pack(params, "f32_w16_t"), masks=masks,
                           d_raw=torch.randn(r, s, 4, generator=g).to(dev), n_rays=r, n_samples=s, chunk_rows=r,
                           n_codes=1, freqs_xyz=fx, freqs_dir=fd, rd=rd, ro=ro, z=z, want_ro=True, want_rd=True,
                           precision="f32"))
        acts.append((params, act))
    out = {}
    for mode in ("single", "pair"):
        d_ro, d_rd = start[0].clone(), start[1].clone()
        accs = [torch.zeros(ops.field_backward_x3_acc_floats(1, r, True, True), device=dev) for _ in fields]
        jobs = [dict(f, acc=a, ray_into=(d_ro, d_rd)) for f, a in zip(fields, accs)]
        if mode == "single":
            res = [ops.field_backward_x3(**jobs[0])]
            d_rd.add_(between)
            res.append(ops.field_backward_x3(**jobs[1]))
            wss = [ops.code_ds_outer(p, zs, zt, act, rr["g_code"]) for (p, act), rr in zip(acts, res)]
        else:
            res = ops.field_backward_x3_multi(jobs, d_rd_between=between)
            wss = ops.code_ds_outer_multi([(p, act, rr["g_code"], None) for (p, act), rr in zip(acts, res)], zs, zt)
        torch.cuda.synchronize()
        out[mode] = (d_ro, d_rd, [rr["g_code"].clone() for rr in res], wss)
    a, b = out["pair"], out["single"]
    assert torch.equal(a[0], b[0]), ("d ro", (a[0] - b[0]).abs().max().item())
    assert torch.equal(a[1], b[1]), ("d rd", (a[1] - b[1]).abs().max().item())
    for k in range(2):
        assert torch.equal(a[2][k], b[2][k]), ("g_code", k)
        # (the first half writes ds1 / ds2 / dt1 into workspace rows 3..5 of each code; rows 0..2 are cn_code_dz's)
        assert torch.equal(a[3][k][768:1536], b[3][k][768:1536]), ("code_ds_outer workspace", k)
