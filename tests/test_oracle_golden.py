"""The CPU oracle reproduces the reference's own outputs (fixtures from tests/golden/make_golden.py).

Bit-exact (max |d| == 0) wherever the oracle runs the reference's op sequence on
the same aten CPU kernels; this is what pins the oracle.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import codenerf_oracle as O
from codenerf import synthetic


def load(name):
    return {k: torch.from_numpy(v) for k, v in np.load(os.path.join(GOLDEN, name)).items()}


def same(a, b, tol=0.0):
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    d = (a.double() - b.double()).abs().max().item() if a.numel() else 0.0
    assert d <= tol, d


def test_rays():
    g = load("rays_small.npz")
    d = O.ray_directions(12, 16, g["intrinsics"])
    same(d, g["directions"])
    ro, rd = O.ray_bundle(d, g["poses"])
    same(ro, g["ro"])
    same(rd, g["rd"])
    o, r = O.gather_rays(ro, rd, g["select_inds"].numpy())
    same(o, g["ro_sel"])
    same(r, g["rd_sel"])


@pytest.mark.parametrize("tag", ["nc8_nf8_lindepth_d", "nc8_nf8_lindepth_p", "nc8_nf8_lindisp_d", "nc8_nf8_lindisp_p",
                                 "nc32_nf128_lindepth_d", "nc32_nf128_lindepth_p", "nc64_nf64_lindepth_d",
                                 "nc64_nf64_lindepth_p"])
def test_points(tag):
    g = load("points_small.npz")
    nc, nf = [int(x[2:]) for x in tag.split("_")[:2]]
    mode = tag.split("_")[2]
    bins = O.depth_bins(nc, 0.8, 1.8, mode)
    same(bins["z"], g[tag + "_zbins"])
    same(bins["lower"], g[tag + "_lower"])
    same(bins["upper"], g[tag + "_upper"])
    pts, z = O.sample_uniform(g["ro"], g["rd"], bins, g.get(tag + "_t_rand"))
    same(z, g[tag + "_z"])
    same(pts, g[tag + "_pts"])
    pf, zf = O.sample_pdf(g["ro"], g["rd"], g[tag + "_w"], z, nf, g.get(tag + "_u"))
    same(zf, g[tag + "_zf"])
    if tag + "_ptsf" in g:
        same(pf, g[tag + "_ptsf"])


def test_posenc():
    g = load("posenc.npz")
    for L, log, inc in [(10, True, True), (4, True, True), (6, False, True), (3, True, False)]:
        k = f"L{L}_{int(log)}_{int(inc)}"
        f = O.frequency_bands(L, log)
        same(f, g[k + "_freqs"])
        same(O.posenc(g["x"], f, inc), g[k])


def test_mlp():
    g = load("mlp.npz")
    p = synthetic.codenerf_params(0)
    same(O.codenerf_mlp(p, g["z_s"], g["z_t"], g["x"], 63), g["raw"])


def test_volume_render():
    g = load("volrender.npz")
    rgb, disp, acc, w, depth = O.volume_render(g["raw"], g["z"], g["rd"])
    for a, k in zip([rgb, disp, acc, w, depth], ["rgb", "disp", "acc", "weights", "depth"]):
        same(a, g[k])


@pytest.mark.parametrize("nc,nf", [(8, 8), (32, 128)])
@pytest.mark.parametrize("n_ranks", [1, 2, 3])
def test_render_small(nc, nf, n_ranks):
    g = load("render_small.npz")
    d = O.ray_directions(12, 16, g["intrinsics"])
    ro, rd = O.ray_bundle(d, g["pose"])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    n = ro.shape[0]
    if n_ranks > 1:
        per, _ = O.split_sizes(n, n_ranks)
        assert per == g[f"nc{nc}_n{n_ranks}_split"].tolist()
    smp = O.Sampling(nc, nf, 0.8, 1.8)
    emb = O.EmbedCfg()
    with torch.no_grad():
        out = O.render_image(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), smp, emb,
                             synthetic.codenerf_params(0), synthetic.codenerf_params(1), 50, n_ranks)
    same(out["rgb_fine"], g[f"nc{nc}_n{n_ranks}_rgb"])


def test_render_small_perturbed():
    g = load("render_small.npz")
    d = O.ray_directions(12, 16, g["intrinsics"])
    ro, rd = O.ray_bundle(d, g["pose"])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    n = ro.shape[0]
    with torch.no_grad():
        out = O.render_image(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), O.Sampling(8, 8, 0.8, 1.8),
                             O.EmbedCfg(), synthetic.codenerf_params(0), synthetic.codenerf_params(1), 50,
                             t_rand=g["p_t_rand"], u=g["p_u"])
    same(out["rgb_coarse"], g["p_rgb_coarse"])
    same(out["rgb_fine"], g["p_rgb_fine"])


def test_render_full_coarse():
    """C2 at full size (128x128, 64 coarse samples, 4096-ray chunks)."""
    g = load("render_full.npz")
    d = O.ray_directions(128, 128, g["intrinsics"])
    ro, rd = O.ray_bundle(d, g["pose"])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    n = ro.shape[0]
    with torch.no_grad():
        out = O.render_image(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), O.Sampling(64, 64, 0.8, 1.8),
                             O.EmbedCfg(), synthetic.codenerf_params(0), synthetic.codenerf_params(1), 4096,
                             coarse_only=True)
    same(out["rgb_coarse"], g["rgb_c"])
    same(out["depth_coarse"], g["depth_c"])
    same(out["acc_coarse"], g["acc_c"])


def test_eval_step_gradients():
    """eval.py:145-167 autograd (codes + spherical pose) through the oracle."""
    g = load("eval_grad.npz")
    theta = g["theta"].clone().requires_grad_(True)
    phi = g["phi"].clone().requires_grad_(True)
    rho = g["rho"].clone().requires_grad_(True)
    zs = g["z_s"].clone().requires_grad_(True)
    zt = g["z_t"].clone().requires_grad_(True)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    for p in list(pc.values()) + list(pf.values()):
        p.requires_grad_(True)
    c2w = O.pose_spherical(theta, phi, rho)[None]
    d = O.ray_directions(12, 16, load("render_small.npz")["intrinsics"])
    ro, rd = O.ray_bundle(d, c2w)
    ro, rd = O.gather_rays(ro, rd, g["select_inds"].numpy())
    n = ro.shape[0]
    tp = g["target"][None][..., g["select_inds"].numpy(), :].squeeze()
    zse, zte = zs.expand(n, -1), zt.expand(n, -1)
    out = O.predict_radiance_and_render(ro, rd, O.Sampling(8, 8, 0.8, 1.8), O.EmbedCfg(), pc, pf, zse, zte)
    lc = torch.nn.functional.mse_loss(out["rgb_coarse"][..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(out["rgb_fine"][..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    same(out["rgb_coarse"].detach(), g["rgb_coarse"])
    same(out["rgb_fine"].detach(), g["rgb_fine"])
    same(loss.detach(), g["loss"])
    for t, k in [(theta, "theta"), (phi, "phi"), (rho, "rho"), (zs, "z_s"), (zt, "z_t")]:
        same(t.grad, g["g_" + k], 1e-9)
    same(pf["fc_rgb.weight"].grad, g["g_fine_fc_rgb_w"], 1e-9)
    same(pc["fc_out.bias"].grad, g["g_coarse_fc_out_b"], 1e-9)


def test_split_sizes():
    """Q5: truncating split, last rank takes the remainder."""
    assert O.split_sizes(1024, 3)[0] == [341, 341, 342]
    assert O.split_sizes(16384, 8)[0] == [2048] * 8
    per, pad = O.split_sizes(100, 7)
    assert per == [14] * 6 + [16] and pad == [2] * 6 + [0]


# ---------------------------------------------------------------- round-2 fixtures (make_golden.py gen_*)


def _srn_rays(g, size=128):
    d = O.ray_directions(size, size, g["intrinsics"])
    ro, rd = O.ray_bundle(d, g["pose"])
    return ro.reshape(-1, 3), rd.reshape(-1, 3)


@pytest.mark.parametrize("case", sorted(synthetic.TRAINED_CASES))
def test_trained_magnitude(case):
    """Trained-magnitude weights: the MLP rows and the first 4096-ray chunk of the C3 render."""
    g = load("render_trained.npz")
    pc, pf = synthetic.trained_params(0, case), synthetic.trained_params(1, case)
    with torch.no_grad():
        raw = O.codenerf_mlp(pc, synthetic.trained_codes(7, 1000, case), synthetic.trained_codes(8, 1000, case),
                             g["x"], 63)
    same(raw, g[case + "_mlp_raw"])
    assert raw[:, 3].median() > 10.0             # sigma_raw in the trained range
    ro, rd = _srn_rays(g)
    n = 4096
    zs, zt = synthetic.trained_codes(5, 1, case).expand(n, -1), synthetic.trained_codes(6, 1, case).expand(n, -1)
    with torch.no_grad():
        out = O.predict_radiance_and_render(ro[:n], rd[:n], O.Sampling(64, 64, 0.8, 1.8), O.EmbedCfg(), pc, pf, zs, zt)
    for a, k in [("rgb_coarse", "rgb_c"), ("depth_coarse", "depth_c"), ("rgb_fine", "rgb_f"), ("depth_fine", "depth_f"),
                 ("acc_fine", "acc_f")]:
        same(out[a], g[f"{case}_{k}"][:n])


def test_chairs_c4_chunk():
    """C4 (chairs, Nc 32 / Nf 128, near 1.25 far 2.75): the first chunk of the 1-rank image and the
    8-rank split (2048-ray slices -> 2048-ray chunks, Q1) of rank 0."""
    g = load("render_chairs.npz")
    ro, rd = _srn_rays(g)
    assert O.split_sizes(16384, 8)[0] == g["n8_split"].tolist()
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    smp = O.Sampling(32, 128, 1.25, 2.75)
    for n, key in [(4096, "n1_rgb"), (2048, "n8_rgb")]:
        zs, zt = g["z_s"].expand(n, -1), g["z_t"].expand(n, -1)
        with torch.no_grad():
            out = O.predict_radiance_and_render(ro[:n], rd[:n], smp, O.EmbedCfg(), pc, pf, zs, zt)
        same(out["rgb_fine"], g[key][:n])
    same(g["n1_rgb"], g["n2_rgb"])             # 8192-ray slices keep the 4096-ray chunks
    same(g["n1_rgb"], g["n4_rgb"])


def lego_uniforms(g):
    torch.manual_seed(123)
    t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
    same(t_rand[:4], g["t_rand_head"])
    same(u[:4], g["u_head"])
    assert abs(t_rand.double().sum().item() - g["t_rand_sum"].item()) < 0.05      # stored as fp32
    assert abs(u.double().sum().item() - g["u_sum"].item()) < 0.05
    return t_rand, u


@pytest.mark.parametrize("tag", ["d", "p"])
def test_lego_c1(tag):
    """C1: every leaf with lego's parameters (64x64, Nc 32, Nf 128, near 2, far 6, one 4096-ray chunk)."""
    g = load("lego_c1.npz")
    d = O.ray_directions(64, 64, g["intrinsics"])
    same(d, g["directions"])
    ro, rd = O.ray_bundle(d, g["pose"])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    same(ro, g["ro"])
    same(rd, g["rd"])
    smp = O.Sampling(32, 128, 2.0, 6.0)
    t_rand, u = lego_uniforms(g) if tag == "p" else (None, None)
    pc, pf = synthetic.codenerf_params(2), synthetic.codenerf_params(3)
    zs, zt = g["z_s"].expand(4096, -1), g["z_t"].expand(4096, -1)
    pts, z = O.sample_uniform(ro, rd, smp.bins, t_rand)
    same(z[:512], g[tag + "_z"])
    if tag == "d":
        same(pts[:64], g["d_pts"])
        same(O.posenc(pts.reshape(-1, 3)[:256], O.frequency_bands(10, True), True), g["enc_xyz"])
    with torch.no_grad():
        raw = O.forward_pass(pc, O.EmbedCfg(), rd, pts, zs, zt)
        out = O.predict_radiance_and_render(ro, rd, smp, O.EmbedCfg(), pc, pf, zs, zt, t_rand, u)
    same(raw[:64], g[tag + "_raw"])
    same(out["weights_coarse"][:512], g[tag + "_w_c"])
    same(out["z_fine"][:512], g[tag + "_z_f"])
    for a, k in [("rgb_coarse", "rgb_c"), ("acc_coarse", "acc_c"), ("depth_coarse", "depth_c"), ("rgb_fine", "rgb_f"),
                 ("depth_fine", "depth_f"), ("acc_fine", "acc_f")]:
        same(out[a], g[f"{tag}_{k}"])


def test_eval_c5_gradients():
    """C5 at size: one eval step (2048 rays of a 128x128 view, 64 + 64 perturbed) through the oracle's
    autograd equals the reference's own."""
    g = load("eval_c5.npz")
    theta, phi, rho = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    for p in list(pc.values()) + list(pf.values()):
        p.requires_grad_(True)
    c2w = O.pose_spherical(theta, phi, rho)[None]
    d = O.ray_directions(128, 128, synthetic.srn_intrinsics(128))
    ro, rd = O.ray_bundle(d, c2w)
    sel = g["select_inds"].numpy()
    ro, rd = O.gather_rays(ro, rd, sel)
    n = ro.shape[0]
    tp = g["target"][None][..., sel, :].squeeze()
    zse, zte = zs.expand(n, -1), zt.expand(n, -1)
    out = O.predict_radiance_and_render(ro, rd, O.Sampling(64, 64, 0.8, 1.8), O.EmbedCfg(), pc, pf, zse, zte,
                                        g["t_rand"], g["u"])
    lc = torch.nn.functional.mse_loss(out["rgb_coarse"][..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(out["rgb_fine"][..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    same(out["rgb_coarse"].detach(), g["rgb_coarse"])
    same(out["rgb_fine"].detach(), g["rgb_fine"])
    same(loss.detach(), g["loss"])
    for t, k in [(theta, "theta"), (phi, "phi"), (rho, "rho"), (zs, "z_s"), (zt, "z_t")]:
        same(t.grad, g["g_" + k], 1e-8)
    same(pf["fc_rgb.weight"].grad, g["g_fine_fc_rgb_w"], 1e-8)


# ---------------------------------------------------------------- round 2: pose metric, loss, SRN format


def test_se3_pose_error():
    """lieutils.SE3.Log of inverse(gt) @ cam (eval.py:161-162), incl. near-identity poses."""
    g = load("se3_pose_error.npz")
    tw = O.se3_log(torch.matmul(torch.inverse(g["gt"]), g["cam"]))
    same(tw, g["twist"], 1e-6)
    same(O.pose_error(g["gt"], g["cam"]), g["err"], 1e-6)


def test_loss_terms():
    g = load("loss.npz")
    rc, rf = g["rgb_c"].clone().requires_grad_(True), g["rgb_f"].clone().requires_grad_(True)
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    loss = O.render_loss(rc, rf, g["target"], zs.expand(300, -1), zt.expand(300, -1), float(g["lam"]))
    loss.backward()
    same(loss, g["loss"])
    for t, k in ((rc, "g_rgb_c"), (rf, "g_rgb_f"), (zs, "g_z_s"), (zt, "g_z_t")):
        same(t.grad, g[k])


def test_srn_item_restatement(tmp_path):
    """dataset.py:60-94 on the tiny synthetic SRN tree: the oracle's restatement reproduces the
    reference loader's every output (decode, /255, mask, crop, pose flip, principal point)."""
    import sys
    sys.path.insert(0, GOLDEN)
    import srn_tree
    g = np.load(os.path.join(GOLDEN, "srn_tiny.npz"))
    base = srn_tree.write_tree(str(tmp_path))
    for stage in ("train", "val"):
        files = list(g[f"{stage}_files"])
        obj_dirs = sorted({f.split("/rgb/")[0] for f in files})
        for i, f in enumerate(files):
            obj = f.split("/rgb/")[0]
            view = os.path.basename(f)[:-4]
            item = O.srn_item(os.path.join(base, f), os.path.join(base, obj, "pose", view + ".txt"),
                              os.path.join(base, obj, "intrinsics.txt"), obj_dirs.index(obj))
            for k in ("color", "mask", "pose", "intrinsic", "object_id"):
                ref = g[f"{stage}_{i}_{k}"]
                assert np.array_equal(np.asarray(item[k]), ref), (stage, i, k)


def test_train_c3_chunk_gradients():
    """C3 at size (train_c3.npz): the reference's own train.py:96-114 chunk step -- 4096 rays of two
    objects of a 2458-object table, 64 + 64 perturbed samples -- through the oracle's autograd: the
    losses, every parameter gradient's norm, five full gradients and the touched code rows."""
    g = load("train_c3.npz")
    torch.manual_seed(4343)
    t_rand, u = torch.rand(4096, 64), torch.rand(4096, 64)
    same(t_rand[:4], g["t_rand_head"])
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    ts, tt = synthetic.latent_codes(40, 2458).requires_grad_(True), synthetic.latent_codes(41, 2458).requires_grad_(True)
    for p in list(pc.values()) + list(pf.values()):
        p.requires_grad_(True)
    ids = g["ids"].long()
    out = O.predict_radiance_and_render(g["ro"], g["rd"], O.Sampling(64, 64, 0.8, 1.8), O.EmbedCfg(), pc, pf,
                                        ts[ids], tt[ids], t_rand, u)
    tgt = g["target"]
    lc = torch.nn.functional.mse_loss(out["rgb_coarse"][..., :3], tgt[..., :3])
    lf = torch.nn.functional.mse_loss(out["rgb_fine"][..., :3], tgt[..., :3])
    reg = 1e-5 * (torch.norm(ts.data.reshape(-1), p=2) + torch.norm(tt.data.reshape(-1), p=2))
    (lc + lf + reg).backward()
    same(lc.detach(), g["lc"], 1e-7)
    same(lf.detach(), g["lf"], 1e-7)
    same(reg, g["reg"], 1e-9)
    named = {**{f"nerf_coarse.{k}": v for k, v in pc.items()}, **{f"nerf_fine.{k}": v for k, v in pf.items()}}
    for k, p in named.items():
        ref = g["gnorm_" + k].item()
        assert abs(p.grad.norm().item() - ref) <= 1e-5 * ref + 1e-9, k
    for k in ("nerf_coarse.layer_dir1.weight", "nerf_coarse.shape_code_layer1.weight", "nerf_fine.fc_rgb.weight",
              "nerf_fine.fc_out.bias", "nerf_fine.layer_xyz1.weight"):
        same(named[k].grad, g["g_" + k], 1e-5 * g["g_" + k].abs().max().item())
    for t, k in ((ts, "shape_embedding"), (tt, "texture_embedding")):
        ref = g[f"grows_embedding.{k}.weight"]
        same(t.grad[[17, 1234]], ref, 1e-5 * ref.abs().max().item())


# ---------------------------------------------------------------- round 6: the reference's runnable shapes


@pytest.mark.parametrize("name", ["train_cars_code", "train_3080"])
def test_train_shape_chunk_gradients(name):
    """train.py:76-114 at srn-cars-code.yml (32 + 128, chunk 4096) and srn-cars-code-3080.yml (64 + 128,
    the first 1024-ray chunk of a 4096-ray draw): the reference's own chunk step (make_golden.py
    gen_train_shape, one object per chunk) through the oracle's autograd -- losses, every gradient's
    norm and its 16 projections, five full gradients, the touched code row."""
    g = load(name + ".npz")
    nc, nf, chunk = int(g["nc"]), int(g["nf"]), int(g["chunk"])
    torch.manual_seed(4343)
    t_rand, u = torch.rand(chunk, nc), torch.rand(chunk, nf)
    same(t_rand[:4], g["t_rand_head"])
    same(u[:4], g["u_head"])
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    ts, tt = synthetic.latent_codes(40, 2458).requires_grad_(True), synthetic.latent_codes(41, 2458).requires_grad_(True)
    for p in list(pc.values()) + list(pf.values()):
        p.requires_grad_(True)
    ids = g["ids"].long()
    smp = O.Sampling(nc, nf, float(g["near"]), float(g["far"]))
    out = O.predict_radiance_and_render(g["ro"], g["rd"], smp, O.EmbedCfg(), pc, pf, ts[ids], tt[ids], t_rand, u)
    tgt = g["target"]
    lc = torch.nn.functional.mse_loss(out["rgb_coarse"][..., :3], tgt[..., :3])
    lf = torch.nn.functional.mse_loss(out["rgb_fine"][..., :3], tgt[..., :3])
    reg = 1e-5 * (torch.norm(ts.data.reshape(-1), p=2) + torch.norm(tt.data.reshape(-1), p=2))
    (lc + lf + reg).backward()
    same(out["rgb_coarse"].detach(), g["rgb_coarse"], 1e-6)
    same(out["rgb_fine"].detach(), g["rgb_fine"], 1e-6)
    same(lc.detach(), g["lc"], 1e-7)
    same(lf.detach(), g["lf"], 1e-7)
    same(reg, g["reg"], 1e-9)
    named = {**{f"nerf_coarse.{k}": v for k, v in pc.items()}, **{f"nerf_fine.{k}": v for k, v in pf.items()}}
    for idx, k in enumerate(sorted(named), start=2):   # make_golden's index counts the two embedding tables
        p = named[k]
        ref = g["gnorm_" + k].item()
        assert abs(p.grad.norm().item() - ref) <= 1e-5 * ref + 1e-9, k
        r = torch.randn((16,) + tuple(p.shape), generator=torch.Generator().manual_seed(7000 + idx))
        pr = (r.double() * p.grad.double()[None]).reshape(16, -1).sum(1)
        assert (pr - g["gproj_" + k].double()).abs().max().item() <= 1e-4 * ref + 1e-9, k
    for k in ("nerf_coarse.layer_dir1.weight", "nerf_coarse.shape_code_layer1.weight", "nerf_fine.fc_rgb.weight",
              "nerf_fine.fc_out.bias", "nerf_fine.layer_xyz1.weight"):
        same(named[k].grad, g["g_" + k], 1e-5 * g["g_" + k].abs().max().item())
    oid = int(ids[0])
    assert torch.equal(ids, torch.full_like(ids, oid))
    for t, k in ((ts, "shape_embedding"), (tt, "texture_embedding")):
        ref = g[f"grows_embedding.{k}.weight"]
        same(t.grad[[oid]], ref, 1e-5 * ref.abs().max().item())


def test_eval_c5_chairs_gradients():
    """eval.py:141-168 at srn-chairs-code.yml's shape (4096 rays, 32 + 128 perturbed, near 1.25 far
    2.75, make_golden.py gen_c5_chairs) through the oracle's autograd equals the reference's own."""
    g = load("eval_c5_chairs.npz")
    torch.manual_seed(4244)
    t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
    same(t_rand[:4], g["t_rand_head"])
    same(u[:4], g["u_head"])
    theta, phi, rho = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    for p in list(pc.values()) + list(pf.values()):
        p.requires_grad_(True)
    c2w = O.pose_spherical(theta, phi, rho)[None]
    d = O.ray_directions(128, 128, synthetic.srn_intrinsics(128))
    ro, rd = O.ray_bundle(d, c2w)
    sel = g["select_inds"].numpy()
    ro, rd = O.gather_rays(ro, rd, sel)
    n = ro.shape[0]
    tp = g["target"][None][..., sel, :].squeeze()
    zse, zte = zs.expand(n, -1), zt.expand(n, -1)
    out = O.predict_radiance_and_render(ro, rd, O.Sampling(32, 128, 1.25, 2.75), O.EmbedCfg(), pc, pf, zse, zte,
                                        t_rand, u)
    lc = torch.nn.functional.mse_loss(out["rgb_coarse"][..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(out["rgb_fine"][..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    same(out["rgb_coarse"].detach(), g["rgb_coarse"], 1e-6)
    same(out["rgb_fine"].detach(), g["rgb_fine"], 1e-6)
    same(loss.detach(), g["loss"], 1e-7)
    for t, k in [(theta, "theta"), (phi, "phi"), (rho, "rho"), (zs, "z_s"), (zt, "z_t")]:
        ref = g["g_" + k]
        same(t.grad, ref, 1e-5 * max(1e-2, ref.abs().max().item()))
    same(pf["fc_rgb.weight"].grad, g["g_fine_fc_rgb_w"], 1e-5 * g["g_fine_fc_rgb_w"].abs().max().item())
