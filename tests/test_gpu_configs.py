"""BASELINE.json configs C1 (lego plumbing), C4 (chairs, 1/2/4/8 rank slices) and C5 (eval step at
size), and trained-magnitude weights, on the HIP path against the reference's own outputs
(tests/golden/make_golden.py gen_lego / gen_chairs / gen_c5 / gen_trained).

Tolerances (north_star): rendered rgb / depth / acc 1e-4 absolute; ray directions, depth bins and
rank splits bit-exact; raw MLP outputs RAW_RTOL relative to the largest |raw| (trained nets reach
|raw| ~ 80, where 1e-4 absolute is below fp32's own reassociation error); gradients as in
test_gpu_grad (relative to the tensor's largest magnitude).
"""
import numpy as np
import pytest
import torch

from conftest import margin
from test_gpu_parity import dev, embedders, load, maxdiff  # noqa: F401

pytestmark = pytest.mark.gpu

TOL_RENDER = 1e-4
RAW_RTOL = 1e-5
# the 3xbf16 split drops Wl.Xl and rounds Xl to bf16: ~3 * 2^-18 = 1.1e-5 relative per product at
# worst; both 3xbf16 kernels (32x32x16 and 16x16x32 accumulation orders) land at 0.99-1.09e-5 on
# the t3 net (tools/x3w_err.py), so their raw-output bound is 1.5e-5 (rendered outputs keep 1e-4)
RAW_RTOL_X3 = 1.5e-5
PRECISIONS = ["f32", "f32_v1", "bf16x3", "bf16x3_w16"]
# C5 at-size gradient bounds (max |g - g_ref| over the tensor's largest |g_ref|; d theta / phi / rho
# relative to max(1e-2, |g_ref|)), about twice the achieved values (r04b, profiles/r04): the pose and
# code gradients at <= 4.7e-5, so 1e-4; the weight gradients (not frozen): fine fc_rgb 3.9e-6 and the
# norms 2.7e-5 against 1e-4, coarse layer_xyz1 3.2e-4 -- its input is the encodings of every sample,
# where the fine depths that moved across a bin (test_train_c3_decisions_at_size counts them for the
# C3 step) enter directly
C5_GRAD_RTOL = {"f32": 1e-4, "bf16x3": 1e-4}
C5_XYZ1_RTOL = 6.5e-4


def model_from(dev, params, precision):
    from codenerf.models import CodeNeRFModel
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(params)
    m.precision = precision
    return m.to(dev).eval()


def rays_of(dev, g, size):
    from codenerf.nerf import RaySampler
    rs = RaySampler(size, size, g["intrinsics"].cpu(), sample_size=min(4096, size * size), device=dev,
                    datatype=torch.float32)
    ro, rd = rs.get_bundle(g["pose"])
    return rs, ro.reshape(-1, 3), rd.reshape(-1, 3)


# ---------------------------------------------------------------- trained-magnitude weights


@pytest.mark.parametrize("case", ["t4", "t3"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_trained_mlp(dev, precision, case):
    from codenerf import synthetic
    g = load("render_trained.npz", dev)
    m = model_from(dev, synthetic.trained_params(0, case), precision)
    with torch.no_grad():
        raw = m(synthetic.trained_codes(7, 1000, case).to(dev), synthetic.trained_codes(8, 1000, case).to(dev), g["x"])
    ref = g[case + "_mlp_raw"]
    scale = ref.abs().max().item()
    err = maxdiff(raw, ref)
    print(f"{precision} {case}: raw max|d| {err:.3e} (max|raw| {scale:.1f}, rel {err / scale:.2e})")
    assert err <= (RAW_RTOL_X3 if precision.startswith("bf16x3") else RAW_RTOL) * scale


@pytest.mark.parametrize("case", ["t4", "t3"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_trained_render_c2_c3(dev, precision, case):
    """Full 128x128 C2 (coarse) and C3 (64+64) renders of a trained-magnitude net vs the reference."""
    from codenerf import synthetic
    from codenerf.nerf import PointSampler, render_rays
    g = load("render_trained.npz", dev)
    _, ro, rd = rays_of(dev, g, 128)
    n = ro.shape[0]
    mc = model_from(dev, synthetic.trained_params(0, case), precision)
    mf = model_from(dev, synthetic.trained_params(1, case), precision)
    zs = synthetic.trained_codes(5, 1, case).to(dev).expand(n, -1)
    zt = synthetic.trained_codes(6, 1, case).to(dev).expand(n, -1)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    with torch.no_grad():
        o = render_rays(ro, rd, zs, zt, ps, embedders(dev), mc, mf, chunk_rows=4096)
    d = {k: maxdiff(o[a], g[f"{case}_{k}"]) for a, k in [("rgb_coarse", "rgb_c"), ("depth_coarse", "depth_c"),
                                                        ("acc_coarse", "acc_c"), ("rgb_fine", "rgb_f"),
                                                        ("depth_fine", "depth_f"), ("acc_fine", "acc_f")]}
    for k, v in d.items():
        margin(f"render_trained_{case}[{precision}]", k, v, TOL_RENDER)


# ---------------------------------------------------------------- C4: chairs, rank slices


@pytest.mark.parametrize("n_ranks", [1, 2, 4, 8])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_chairs_c4_rank_slices(dev, precision, n_ranks):
    """srn-chairs-code.yml at 128x128 (Nc 32 / Nf 128 -> 160 fine samples, near 1.25, far 2.75,
    validation chunk 4096): each rank's Q5 slice rendered with the reference's per-rank chunking,
    concatenated as rank 0's gather would, vs parallel_image_render of the reference."""
    from codenerf import synthetic
    from codenerf.nerf import PointSampler, render_rays
    from codenerf.utils import split_sizes
    g = load("render_chairs.npz", dev)
    _, ro, rd = rays_of(dev, g, 128)
    n = ro.shape[0]
    per, _ = split_sizes(n, n_ranks)
    if n_ranks > 1:
        assert per == g[f"n{n_ranks}_split"].tolist()
    mc = model_from(dev, synthetic.codenerf_params(0), precision)
    mf = model_from(dev, synthetic.codenerf_params(1), precision)
    ps = PointSampler(32, 128, 1.25, 2.75, "lindepth", False, torch.float32, dev)
    outs, start = [], 0
    with torch.no_grad():
        for r in range(n_ranks):
            sl = slice(start, start + per[r])
            start += per[r]
            outs.append(render_rays(ro[sl], rd[sl], g["z_s"].expand(n, -1)[sl], g["z_t"].expand(n, -1)[sl], ps,
                                    embedders(dev), mc, mf, chunk_rows=4096))
    rgb = torch.cat([o["rgb_fine"] for o in outs])
    tag = f"chairs_c4_n{n_ranks}[{precision}]"
    margin(tag, "rgb_f", maxdiff(rgb, g[f"n{n_ranks}_rgb"]), TOL_RENDER)
    if n_ranks == 1:
        margin(tag, "depth_f", maxdiff(outs[0]["depth_fine"], g["depth_f"]), TOL_RENDER)
        margin(tag, "acc_f", maxdiff(outs[0]["acc_fine"], g["acc_f"]), TOL_RENDER)
        margin(tag, "rgb_c", maxdiff(outs[0]["rgb_coarse"], g["rgb_c"]), TOL_RENDER)
        assert outs[0]["z_fine"].shape == (n, 160)


# ---------------------------------------------------------------- C1: lego plumbing


def lego_uniforms(g):
    torch.manual_seed(123)
    t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
    assert torch.equal(t_rand[:4], g["t_rand_head"].cpu()) and torch.equal(u[:4], g["u_head"].cpu())
    return t_rand, u


@pytest.mark.parametrize("tag", ["d", "p"])
def test_lego_c1_leaf_ops(dev, tag):
    """Every HIP leaf op with config/lego.yml's parameters (64x64, near 2, far 6, lindepth, Nc 32 per
    BASELINE.json, Nf 128, validation chunk 8192 -> the whole 4096-ray image in one chunk)."""
    from codenerf import synthetic
    from codenerf.nerf import PointSampler, RaySampler, forward_pass, render_rays, volume_render
    g = load("lego_c1.npz", dev)
    rs = RaySampler(64, 64, g["intrinsics"].cpu(), sample_size=1024, device=dev, datatype=torch.float32)
    assert maxdiff(rs.directions, g["directions"]) == 0.0
    ro, rd = rs.get_bundle(g["pose"])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    assert maxdiff(ro, g["ro"]) == 0.0 and maxdiff(rd, g["rd"]) <= 1e-6
    t_rand, u = (None, None)
    if tag == "p":
        t_rand, u = [t.to(dev) for t in lego_uniforms(g)]
    ps = PointSampler(32, 128, 2.0, 6.0, "lindepth", tag == "p", torch.float32, dev)
    pts, z = ps.sample_uniform(ro, rd, t_rand=t_rand)
    assert maxdiff(z[:512], g[tag + "_z"]) == 0.0
    emb = embedders(dev)
    if tag == "d":
        # pts = ro + rd z: bit-exact on the fixture's own rays (cn_ray_points), and within rd's
        # einsum-order ulp x far on ours
        assert maxdiff(ps.sample_uniform(g["ro"], g["rd"])[0][:64], g["d_pts"]) == 0.0
        assert maxdiff(pts[:64], g["d_pts"]) <= 6e-6
        assert maxdiff(emb[0].embed(g["d_pts"][:8].reshape(-1, 3)), g["enc_xyz"]) <= 2e-6
    mc = model_from(dev, synthetic.codenerf_params(2), "f32")
    mf = model_from(dev, synthetic.codenerf_params(3), "f32")
    zs, zt = g["z_s"].expand(4096, -1), g["z_t"].expand(4096, -1)
    with torch.no_grad():
        raw = forward_pass(mc, emb, rd, pts, (zs, zt))
        assert maxdiff(raw[:64], g[tag + "_raw"]) <= 1e-4
        w = volume_render(raw, z, rd)[3]
        assert maxdiff(w[:512], g[tag + "_w_c"]) <= 1e-5
        # inverse-CDF resampling on the reference's own coarse weights (identical inputs): the
        # fine depths to 1e-5 (near-empty bins amplify a weight's last bit by 1/pdf, so a
        # resampling of OUR weights is checked end to end through the rendered maps below)
        _, z_f = ps.sample_pdf(ro[:512], rd[:512], g[tag + "_w_c"][..., 1:-1], z[:512],
                               u=None if u is None else u[:512])
        assert maxdiff(z_f, g[tag + "_z_f"]) <= 1e-5
        o = render_rays(ro, rd, zs, zt, ps, emb, mc, mf, chunk_rows=8192, t_rand=t_rand, u=u)
    for a, k in [("rgb_coarse", "rgb_c"), ("acc_coarse", "acc_c"), ("depth_coarse", "depth_c"), ("rgb_fine", "rgb_f"),
                 ("depth_fine", "depth_f"), ("acc_fine", "acc_f")]:
        margin(f"lego_c1[{tag}]", k, maxdiff(o[a], g[f"{tag}_{k}"]), TOL_RENDER)


# ---------------------------------------------------------------- C5: one eval step at size


@pytest.mark.parametrize("frozen,precision", [(False, "f32"), (True, "f32"), (True, "bf16x3")])
def test_eval_c5_step_at_size(dev, frozen, precision):
    """eval.py:141-167 at srn-cars-code-3080-val.yml's size: 2048 rays of a 128x128 view, 64 + 64
    perturbed samples (the reference's draws injected), one predict_radiance_and_render over the
    whole batch; gradients into theta, phi, rho and both codes vs the reference's autograd.
    ``frozen``: weights not requiring grad (what the eval optimiser reads; the fused backward)."""
    from codenerf import synthetic
    from codenerf.evaluate import pose_spherical
    from codenerf.nerf import PointSampler, RaySampler, render_rays
    g = load("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = {}
    for key, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
        m = model_from(dev, synthetic.codenerf_params(seed), precision).train()
        m.requires_grad_(not frozen)
        models[key] = m
    theta, phi, rho = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    np.random.seed(17)
    c2w = pose_spherical(theta, phi, rho)[None, :]
    ro, rd, sel = rs.sample(tform_cam2world=c2w)
    assert np.array_equal(sel, g["select_inds"].cpu().numpy())
    tp = g["target"][None][..., torch.as_tensor(sel, device=dev), :].squeeze()
    n = ro.shape[0]
    zse, zte = zs.expand(n, -1), zt.expand(n, -1)
    o = render_rays(ro, rd, zse, zte, ps, embedders(dev), models["nerf_coarse"], models["nerf_fine"], chunk_rows=n,
                    t_rand=g["t_rand"], u=g["u"])
    rgb_c, rgb_f = o["rgb_coarse"], o["rgb_fine"]
    tag = f"eval_c5[{precision},{'frozen' if frozen else 'weights'}]"
    margin(tag, "rgb_c", maxdiff(rgb_c, g["rgb_coarse"]), TOL_RENDER)
    margin(tag, "rgb_f", maxdiff(rgb_f, g["rgb_fine"]), TOL_RENDER)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    margin(tag, "loss", abs(loss.item() - g["loss"].item()), 1e-5)
    rtol = C5_GRAD_RTOL[precision]
    for name, t in [("theta", theta), ("phi", phi), ("rho", rho)]:
        ref = g["g_" + name].cpu()
        margin(tag, "d " + name, (t.grad.cpu() - ref).abs().max().item() / max(1e-2, ref.abs().max().item()), rtol)
    for name, t in [("z_s", zs), ("z_t", zt)]:
        ref = g["g_" + name].cpu()
        margin(tag, "d " + name, (t.grad.cpu() - ref).abs().max().item() / ref.abs().max().item(), rtol)
    if not frozen:
        for what, t, key, bound in [("fine fc_rgb.weight", models["nerf_fine"].fc_rgb.weight, "g_fine_fc_rgb_w", rtol),
                                    ("coarse layer_xyz1.weight", models["nerf_coarse"].layer_xyz1.weight,
                                     "g_coarse_layer_xyz1_w", C5_XYZ1_RTOL)]:
            ref = g[key].cpu()
            margin(tag, "d " + what, (t.grad.cpu() - ref).abs().max().item() / ref.abs().max().item(), bound)
        worst = (0.0, "")
        for key, mm in models.items():
            for nm, prm in mm.named_parameters():
                ref = g[f"gnorm_{key}.{nm}"].item()
                worst = max(worst, (abs(prm.grad.norm().item() - ref) / (ref + 1e-8), f"{key}.{nm}"))
        margin(tag, "weight-grad norms (worst: %s)" % worst[1], worst[0], rtol)
