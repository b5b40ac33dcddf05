"""Generate the golden fixtures from the REAL reference (run in the build container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

The reference (akashsharma02/code-nerf at /root/reference, pure Python on
PyTorch) is imported with three harness-side shims that touch no reference
file: ``torch.cuda.Device = torch.device`` (annotation-only name removed in
torch 2.x, quirk Q10) and stub ``imageio`` / ``torch.utils.tensorboard``
modules (logging / PNG decode only).  Everything is computed by the
reference's own functions on CPU fp32; this script only prepares inputs and
saves outputs.  Inputs are synthetic (``codenerf.synthetic``): there is no
dataset or checkpoint offline.

The fixtures are data (inputs + expected outputs).  They are what pins
``oracle/codenerf_oracle.py`` (tests/test_oracle_golden.py) and, through it,
the HIP path (tests/test_gpu_*.py).
"""
from __future__ import annotations

import importlib
import os
import sys
import types
from itertools import product

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "code-nerf_amd"))
from codenerf import synthetic  # noqa: E402

REF = "/root/reference"


def import_reference():
    torch.cuda.Device = torch.device
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb
    sys.modules.setdefault("imageio", types.ModuleType("imageio"))
    sys.path.insert(0, REF)
    import importlib
    nerf = importlib.import_module("view_synthesis.nerf")
    model = importlib.import_module("view_synthesis.models.model")
    util = importlib.import_module("view_synthesis.utils.util")
    spec = importlib.util.spec_from_file_location("ref_eval", os.path.join(REF, "eval.py"))
    ev = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ev)
    return nerf, model, util, ev


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32) if t.dtype.is_floating_point else t.detach().cpu().numpy()


def save(name, **arrs):
    path = os.path.join(HERE, name)
    arrs = {k: (np32(v) if torch.is_tensor(v) else np.asarray(v)) for k, v in arrs.items()}
    np.savez_compressed(path, **arrs)
    print(f"wrote {name}: {len(arrs)} arrays, {os.path.getsize(path) // 1024} KiB")


def make_model(model_mod, seed, hidden=256, code=256):
    m = model_mod.CodeNeRFModel(hidden_size=hidden, num_embeddings=1, shape_code_size=code,
                                texture_code_size=code, num_encoding_fn_xyz=10, num_encoding_fn_dir=4,
                                include_input_xyz=True, include_input_dir=True)
    m.load_state_dict(synthetic.codenerf_params(seed, hidden, code))
    return m.eval()


class Cfg(dict):
    """Minimal attribute dict standing in for CfgNode in parallel_image_render."""

    def __getattr__(self, k):
        return self[k]


def small_intrinsics():
    k = torch.eye(4, dtype=torch.float32)
    k[0, 0] = k[1, 1] = 9.5
    k[0, 2], k[1, 2] = 7.0, 5.5
    return k


def main(only=None):
    nerf, model_mod, util, ev = import_reference()
    torch.set_num_threads(8)
    if only:
        for name in only:
            {**ROUND2, **ROUND3, **ROUND6}[name](nerf, model_mod, ev)
        return
    pose = lambda th, ph, rh: ev.pose_spherical(torch.tensor([th]), torch.tensor([ph]), torch.tensor([rh]))  # noqa: E731

    # ---------------------------------------------------------------- rays
    H, W = 12, 16
    K = small_intrinsics()
    rs = nerf.RaySampler(H, W, K, sample_size=40, device="cpu", datatype=torch.float32)
    poses = torch.stack([pose(0.5, 0.3, 1.3), pose(1.1, -0.7, 2.0)])
    ro_b, rd_b = rs.get_bundle(poses)
    np.random.seed(7)
    ro_s, rd_s, sel = rs.sample(poses)
    save("rays_small.npz", intrinsics=K, poses=poses, directions=rs.directions, ro=ro_b.contiguous(),
         rd=rd_b, select_inds=sel.astype(np.int64), ro_sel=ro_s, rd_sel=rd_s)

    # ---------------------------------------------------------------- points
    g = torch.Generator().manual_seed(11)
    R = 37
    ro = torch.randn(R, 3, generator=g) * 0.2 + torch.tensor([0.3, -0.2, 1.2])
    rd = torch.randn(R, 3, generator=g)
    rd = rd / rd.norm(dim=-1, keepdim=True) * (1.0 + 0.3 * torch.rand(R, 1, generator=g))
    out = {"ro": ro, "rd": rd}
    cases = list(product([(8, 8)], ["lindepth", "lindisp"], [False, True]))
    cases += list(product([(32, 128), (64, 64)], ["lindepth"], [False, True]))
    for (nc, nf), mode, pert in cases:
        tag = f"nc{nc}_nf{nf}_{mode}_{'p' if pert else 'd'}"
        ps = nerf.PointSampler(nc, nf, 0.8, 1.8, spacing_mode=mode, perturb=pert, dtype=torch.float32, device="cpu")
        torch.manual_seed(1000 + nc)
        pts, z = ps.sample_uniform(ro, rd)
        if pert:
            torch.manual_seed(1000 + nc)
            out[tag + "_t_rand"] = torch.rand(R, nc)
        w = torch.rand(R, nc - 2, generator=g) ** 3
        w[0] = 0.0                      # all-zero weights -> uniform pdf
        w[1, 3:] = 0.0                  # mass only at the front
        torch.manual_seed(2000 + nc)
        pts_f, z_f = ps.sample_pdf(ro, rd, w, z)
        if pert:
            torch.manual_seed(2000 + nc)
            out[tag + "_u"] = torch.rand(R, nf)
        out.update({tag + "_zbins": ps.z_vals, tag + "_lower": ps.lower, tag + "_upper": ps.upper,
                    tag + "_z": z, tag + "_pts": pts, tag + "_w": w, tag + "_zf": z_f})
        if nc == 8:
            out[tag + "_ptsf"] = pts_f
    save("points_small.npz", **out)

    # ---------------------------------------------------------------- posenc
    x = (torch.rand(50, 3, generator=g) * 2 - 1) * 3.0
    x[0] = torch.tensor([1.7, -2.9, 0.0])
    out = {"x": x}
    for L, log, inc in [(10, True, True), (4, True, True), (6, False, True), (3, True, False)]:
        e = nerf.PositionalEmbedder(L, log, inc, dtype=torch.float32, device="cpu")
        out[f"L{L}_{int(log)}_{int(inc)}"] = e.embed(x)
        out[f"L{L}_{int(log)}_{int(inc)}_freqs"] = e.frequency_bands
    save("posenc.npz", **out)

    # ---------------------------------------------------------------- MLP
    m = make_model(model_mod, 0)
    M = 64
    z_s = synthetic.latent_codes(3, M)
    z_t = synthetic.latent_codes(4, M)
    xin = torch.randn(M, 90, generator=g)
    with torch.no_grad():
        raw = m(z_s, z_t, xin)
    save("mlp.npz", z_s=z_s, z_t=z_t, x=xin, raw=raw)

    # ---------------------------------------------------------------- volume render
    R, S = 29, 24
    raw = torch.randn(R, S, 4, generator=g) * 3.0
    raw[0, :, 3] = 30.0                 # softplus threshold branch (Q12)
    raw[1, :, 3] = -40.0                # transparent ray
    z = torch.sort(0.8 + torch.rand(R, S, generator=g), dim=-1).values
    rdv = torch.randn(R, 3, generator=g)
    rgb, disp, acc, wts, depth = nerf.volume_render(raw, z, rdv)
    save("volrender.npz", raw=raw, z=z, rd=rdv, rgb=rgb, disp=disp, acc=acc, weights=wts, depth=depth)

    # ---------------------------------------------------------------- small render, n ranks
    emb = nerf.PositionalEmbedder(10, True, True, torch.float32, "cpu"), nerf.PositionalEmbedder(4, True, True, torch.float32, "cpu")
    models = {"nerf_coarse": make_model(model_mod, 0), "nerf_fine": make_model(model_mod, 1)}
    zs1, zt1 = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    cam = pose(0.5, 0.3, 1.3)[None]
    out = {"intrinsics": K, "pose": cam, "z_s": zs1, "z_t": zt1}
    for nc, nf in [(8, 8), (32, 128)]:
        ps = nerf.PointSampler(nc, nf, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device="cpu")
        for n_ranks in [1, 2, 3]:
            cfg = Cfg(is_distributed=n_ranks > 1, gpus=n_ranks,
                      nerf=Cfg(validation=Cfg(chunksize=50)))
            if n_ranks == 1:
                img = nerf.parallel_image_render(cfg, cam, [zs1, zt1], models, (rs, ps), emb, "cpu")
            else:
                pieces = {}
                real_rank, real_gather = nerf.dist.get_rank, torch.distributed.all_gather
                for r in range(n_ranks):
                    nerf.dist.get_rank = lambda r=r: r
                    torch.distributed.all_gather = lambda lst, t, r=r: pieces.__setitem__(r, t.clone())
                    nerf.parallel_image_render(cfg, cam, [zs1, zt1], models, (rs, ps), emb, "cpu")
                nerf.dist.get_rank, torch.distributed.all_gather = real_rank, real_gather
                per = torch.full([n_ranks], (H * W / n_ranks), dtype=int)
                per[-1] = H * W - torch.sum(per[:-1])
                img = torch.cat([pieces[r][: per[r]] for r in range(n_ranks)], dim=0)
                out[f"nc{nc}_n{n_ranks}_split"] = per.numpy()
            out[f"nc{nc}_n{n_ranks}_rgb"] = img

    # perturbed chunks with recorded uniforms, via predict_radiance_and_render
    ps = nerf.PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=True, dtype=torch.float32, device="cpu")
    ro_i, rd_i = rs.get_bundle(cam)
    ro_i, rd_i = ro_i.reshape(-1, 3), rd_i.reshape(-1, 3)
    torch.manual_seed(77)
    rgbc, rgbf = [], []
    with torch.no_grad():
        for c0 in range(0, H * W, 50):
            sl = slice(c0, min(c0 + 50, H * W))
            n = sl.stop - sl.start
            a, b = nerf.predict_radiance_and_render((ro_i[sl], rd_i[sl]), ps, emb, models["nerf_coarse"],
                                                   models["nerf_fine"], (zs1.expand(n, -1), zt1.expand(n, -1)))
            rgbc.append(a)
            rgbf.append(b)
    torch.manual_seed(77)
    t_rand, u = [], []
    for c0 in range(0, H * W, 50):
        n = min(c0 + 50, H * W) - c0
        t_rand.append(torch.rand(n, 8))
        u.append(torch.rand(n, 8))
    out.update(p_t_rand=torch.cat(t_rand), p_u=torch.cat(u), p_rgb_coarse=torch.cat(rgbc), p_rgb_fine=torch.cat(rgbf))
    save("render_small.npz", **out)

    # ---------------------------------------------------------------- full size 128x128 (C2 / C3)
    Kf = synthetic.srn_intrinsics(128)
    rsf = nerf.RaySampler(128, 128, Kf, sample_size=4096, device="cpu", datatype=torch.float32)
    camf = pose(0.5, 0.3, 1.3)[None]
    ro_f, rd_f = rsf.get_bundle(camf)
    ro_f, rd_f = ro_f.reshape(-1, 3), rd_f.reshape(-1, 3)
    zsf, ztf = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    out = {"intrinsics": Kf, "pose": camf, "z_s": zsf, "z_t": ztf}
    ps = nerf.PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device="cpu")
    cols = {k: [] for k in ["rgb_c", "depth_c", "acc_c", "rgb_f", "depth_f", "acc_f"]}
    with torch.no_grad():
        for c0 in range(0, ro_f.shape[0], 4096):
            o, d = ro_f[c0:c0 + 4096], rd_f[c0:c0 + 4096]
            n = o.shape[0]
            lat = (zsf.expand(n, -1), ztf.expand(n, -1))
            # the body of predict_radiance_and_render (nerf/__init__.py:81-89), keeping depth/acc
            pts, z = ps.sample_uniform(o, d)
            raw_c = nerf.forward_pass(models["nerf_coarse"], emb, d, pts, lat)
            rgb_c, _, acc_c, w_c, depth_c = nerf.volume_render(raw_c, z, d)
            pts2, z2 = ps.sample_pdf(o, d, w_c[..., 1:-1], z)
            raw_f = nerf.forward_pass(models["nerf_fine"], emb, d, pts2, lat)
            rgb_f, _, acc_f, _, depth_f = nerf.volume_render(raw_f, z2, d)
            for k, v in zip(cols, [rgb_c, depth_c, acc_c, rgb_f, depth_f, acc_f]):
                cols[k].append(v)
    out.update({k: torch.cat(v) for k, v in cols.items()})
    save("render_full.npz", **out)

    # ---------------------------------------------------------------- eval-step gradients (C5)
    ps = nerf.PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device="cpu")
    rs64 = nerf.RaySampler(H, W, K, sample_size=64, device="cpu", datatype=torch.float32)
    theta = torch.tensor([0.6]).requires_grad_(True)
    phi = torch.tensor([0.2]).requires_grad_(True)
    rho = torch.tensor([1.4]).requires_grad_(True)
    zs = synthetic.latent_codes(5, 1).clone().requires_grad_(True)
    zt = synthetic.latent_codes(6, 1).clone().requires_grad_(True)
    target = torch.rand(H * W, 4, generator=g)
    np.random.seed(9)
    c2w = ev.pose_spherical(theta, phi, rho)[None, :]
    ro_e, rd_e, sel = rs64.sample(tform_cam2world=c2w)
    tp = target[None][..., sel, :].squeeze()
    zse, zte = zs.expand(ro_e.shape[0], -1), zt.expand(ro_e.shape[0], -1)
    for mm in models.values():
        mm.train()
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro_e, rd_e), ps, emb, models["nerf_coarse"], models["nerf_fine"], (zse, zte))
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    pw = {f"gnorm_{k}.{n}": p.grad.norm() for k, mm in models.items() for n, p in mm.named_parameters()}
    save("eval_grad.npz", target=target, select_inds=sel.astype(np.int64), theta=theta, phi=phi, rho=rho,
         z_s=zs, z_t=zt, rgb_coarse=rgb_c, rgb_fine=rgb_f, loss=loss, g_theta=theta.grad, g_phi=phi.grad,
         g_rho=rho.grad, g_z_s=zs.grad, g_z_t=zt.grad,
         g_fine_fc_rgb_w=models["nerf_fine"].fc_rgb.weight.grad, g_coarse_fc_out_b=models["nerf_coarse"].fc_out.bias.grad,
         **pw)
    print("split(1024,3) =", util.get_minibatches(torch.arange(10), 4))
    for fn in list(ROUND2.values()) + list(ROUND3.values()) + list(ROUND6.values()):
        fn(nerf, model_mod, ev)


# ==================================================================== round 2 fixtures
# Each writes one .npz; ``python make_golden.py trained chairs lego c5`` regenerates a subset.


def _pose(ev, th, ph, rh):
    return ev.pose_spherical(torch.tensor([th]), torch.tensor([ph]), torch.tensor([rh]))


def _make_model_p(model_mod, params):
    m = model_mod.CodeNeRFModel(hidden_size=256, num_embeddings=1, shape_code_size=256, texture_code_size=256,
                                num_encoding_fn_xyz=10, num_encoding_fn_dir=4, include_input_xyz=True,
                                include_input_dir=True)
    m.load_state_dict(params)
    return m.eval()


def _full_render(nerf, ps, emb, models, ro, rd, zs, zt, chunk, keep_coarse=True):
    """The body of predict_radiance_and_render (nerf/__init__.py:81-89) per chunk, keeping depth/acc."""
    cols = {k: [] for k in ["rgb_c", "depth_c", "acc_c", "rgb_f", "depth_f", "acc_f"]}
    with torch.no_grad():
        for c0 in range(0, ro.shape[0], chunk):
            o, d = ro[c0:c0 + chunk], rd[c0:c0 + chunk]
            n = o.shape[0]
            lat = (zs.expand(n, -1), zt.expand(n, -1))
            pts, z = ps.sample_uniform(o, d)
            raw_c = nerf.forward_pass(models["nerf_coarse"], emb, d, pts, lat)
            rgb_c, _, acc_c, w_c, depth_c = nerf.volume_render(raw_c, z, d)
            pts2, z2 = ps.sample_pdf(o, d, w_c[..., 1:-1], z)
            raw_f = nerf.forward_pass(models["nerf_fine"], emb, d, pts2, lat)
            rgb_f, _, acc_f, _, depth_f = nerf.volume_render(raw_f, z2, d)
            for k, v in zip(cols, [rgb_c, depth_c, acc_c, rgb_f, depth_f, acc_f]):
                cols[k].append(v)
    out = {k: torch.cat(v) for k, v in cols.items()}
    if not keep_coarse:
        out = {k: v for k, v in out.items() if k.endswith("_f")}
    return out


def _embedders(nerf):
    return (nerf.PositionalEmbedder(10, True, True, torch.float32, "cpu"),
            nerf.PositionalEmbedder(4, True, True, torch.float32, "cpu"))


def gen_trained(nerf, model_mod, ev):
    """Trained-magnitude weights (synthetic.TRAINED_CASES: weights x3/x4, codes ~unit variance,
    sigma_raw 10-50): the MLP on 1000 random rows and the full 128x128 C2/C3 render."""
    out = {}
    g = torch.Generator().manual_seed(21)
    x = torch.randn(1000, 90, generator=g)
    x[:, :63] *= 1.5
    out["x"] = x
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=4096, device="cpu", datatype=torch.float32)
    cam = _pose(ev, 0.5, 0.3, 1.3)[None]
    ro, rd = rs.get_bundle(cam)
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    out.update(intrinsics=K, pose=cam)
    emb = _embedders(nerf)
    ps = nerf.PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32,
                           device="cpu")
    for case in synthetic.TRAINED_CASES:
        models = {"nerf_coarse": _make_model_p(model_mod, synthetic.trained_params(0, case)),
                  "nerf_fine": _make_model_p(model_mod, synthetic.trained_params(1, case))}
        zs, zt = synthetic.trained_codes(5, 1, case), synthetic.trained_codes(6, 1, case)
        zr_s, zr_t = synthetic.trained_codes(7, 1000, case), synthetic.trained_codes(8, 1000, case)
        with torch.no_grad():
            out[case + "_mlp_raw"] = models["nerf_coarse"](zr_s, zr_t, x)
        r = _full_render(nerf, ps, emb, models, ro, rd, zs, zt, 4096)
        out.update({f"{case}_{k}": v for k, v in r.items()})
    save("render_trained.npz", **out)


def gen_chairs(nerf, model_mod, ev):
    """C4 (srn-chairs-code.yml:53-60): 128x128, Nc 32 / Nf 128, near 1.25, far 2.75, validation
    chunk 4096, rendered by parallel_image_render's per-rank slicing for 1/2/4/8 ranks."""
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=4096, device="cpu", datatype=torch.float32)
    cam = _pose(ev, 0.5, 0.3, 2.0)[None]
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 0), "nerf_fine": make_model(model_mod, 1)}
    zs, zt = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    ps = nerf.PointSampler(32, 128, 1.25, 2.75, spacing_mode="lindepth", perturb=False, dtype=torch.float32,
                           device="cpu")
    out = {"intrinsics": K, "pose": cam, "z_s": zs, "z_t": zt}
    n_all = 128 * 128
    for n_ranks in (1, 2, 4, 8):
        cfg = Cfg(is_distributed=n_ranks > 1, gpus=n_ranks, nerf=Cfg(validation=Cfg(chunksize=4096)))
        if n_ranks == 1:
            img = nerf.parallel_image_render(cfg, cam, [zs, zt], models, (rs, ps), emb, "cpu")
        else:
            pieces = {}
            real_rank, real_gather = nerf.dist.get_rank, torch.distributed.all_gather
            for r in range(n_ranks):
                nerf.dist.get_rank = lambda r=r: r
                torch.distributed.all_gather = lambda lst, t, r=r: pieces.__setitem__(r, t.clone())
                nerf.parallel_image_render(cfg, cam, [zs, zt], models, (rs, ps), emb, "cpu")
            nerf.dist.get_rank, torch.distributed.all_gather = real_rank, real_gather
            per = torch.full([n_ranks], (n_all / n_ranks), dtype=int)
            per[-1] = n_all - torch.sum(per[:-1])
            img = torch.cat([pieces[r][: per[r]] for r in range(n_ranks)], dim=0)
            out[f"n{n_ranks}_split"] = per.numpy()
        out[f"n{n_ranks}_rgb"] = img
    ro, rd = rs.get_bundle(cam)
    r = _full_render(nerf, ps, emb, models, ro.reshape(-1, 3), rd.reshape(-1, 3), zs, zt, 4096)
    out.update(depth_f=r["depth_f"], acc_f=r["acc_f"], rgb_c=r["rgb_c"])
    save("render_chairs.npz", **out)


LEGO_FOCAL = 0.5 * 64 / float(np.tan(0.5 * 0.6911112070083618))   # Blender lego camera_angle_x at 64 px


def gen_lego(nerf, model_mod, ev):
    """C1 plumbing (config/lego.yml:37-46 with BASELINE.json's 64x64 / 32 samples): every leaf
    component driven with lego's parameters -- near 2, far 6, lindepth, Nc 32, Nf 128, chunk 8192
    (validation) -- deterministic and perturbed (uniforms recorded)."""
    K = torch.eye(4, dtype=torch.float32)
    K[0, 0] = K[1, 1] = LEGO_FOCAL
    K[0, 2] = K[1, 2] = 32.0
    rs = nerf.RaySampler(64, 64, K, sample_size=1024, device="cpu", datatype=torch.float32)
    cam = _pose(ev, 0.6, -0.4, 4.0)[None]
    ro, rd = rs.get_bundle(cam)
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 2), "nerf_fine": make_model(model_mod, 3)}
    zs, zt = synthetic.latent_codes(9, 1), synthetic.latent_codes(10, 1)
    out = {"intrinsics": K, "pose": cam, "directions": rs.directions, "ro": ro, "rd": rd, "z_s": zs, "z_t": zt}
    for pert in (False, True):
        tag = "p" if pert else "d"
        ps = nerf.PointSampler(32, 128, 2.0, 6.0, spacing_mode="lindepth", perturb=pert, dtype=torch.float32,
                               device="cpu")
        torch.manual_seed(123)
        pts, z = ps.sample_uniform(ro, rd)
        raw = nerf.forward_pass(models["nerf_coarse"], emb, rd, pts, (zs.expand(4096, -1), zt.expand(4096, -1)))
        rgb_c, disp_c, acc_c, w_c, depth_c = nerf.volume_render(raw, z, rd)
        pts_f, z_f = ps.sample_pdf(ro, rd, w_c[..., 1:-1], z)
        raw_f = nerf.forward_pass(models["nerf_fine"], emb, rd, pts_f, (zs.expand(4096, -1), zt.expand(4096, -1)))
        rgb_f, _, acc_f, _, depth_f = nerf.volume_render(raw_f, z_f, rd)
        if pert:
            # the draws are re-made by the tests from the same seed (torch CPU Philox, same image);
            # their head and sums are stored so a different generator fails loudly
            torch.manual_seed(123)
            t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
            out.update(t_rand_head=t_rand[:4], u_head=u[:4], t_rand_sum=t_rand.double().sum(),
                       u_sum=u.double().sum())
        # row subsets keep the fixture small; every row was computed over the whole 4096-ray list (Q1)
        out.update({f"{tag}_z": z[:512], f"{tag}_raw": raw[:64], f"{tag}_rgb_c": rgb_c, f"{tag}_acc_c": acc_c,
                    f"{tag}_depth_c": depth_c, f"{tag}_w_c": w_c[:512], f"{tag}_z_f": z_f[:512], f"{tag}_rgb_f": rgb_f,
                    f"{tag}_depth_f": depth_f, f"{tag}_acc_f": acc_f})
        if not pert:
            out["enc_xyz"] = emb[0].embed(pts.reshape(-1, 3)[:256])
            out["d_pts"] = pts[:64]
    save("lego_c1.npz", **out)


def gen_c5(nerf, model_mod, ev):
    """C5 at size (srn-cars-code-3080-val.yml): one eval.py:141-167 step, 2048 rays over a 128x128
    view, 64 + 64 perturbed samples (uniforms recorded), whole batch in one predict_radiance_and_render
    call; gradients into theta, phi, rho and both codes (weights also require grad, as in eval.py)."""
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=2048, device="cpu", datatype=torch.float32)
    ps = nerf.PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=True, dtype=torch.float32,
                           device="cpu")
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 0), "nerf_fine": make_model(model_mod, 1)}
    for mm in models.values():
        mm.train()
    g = torch.Generator().manual_seed(31)
    target = torch.rand(128 * 128, 4, generator=g)
    theta = torch.tensor([1.2]).requires_grad_(True)
    phi = torch.tensor([0.4]).requires_grad_(True)
    rho = torch.tensor([1.35]).requires_grad_(True)
    zs = synthetic.latent_codes(5, 1).clone().requires_grad_(True)
    zt = synthetic.latent_codes(6, 1).clone().requires_grad_(True)
    np.random.seed(17)
    c2w = ev.pose_spherical(theta, phi, rho)[None, :]
    ro, rd, sel = rs.sample(tform_cam2world=c2w)
    tp = target[None][..., sel, :].squeeze()
    zse, zte = zs.expand(ro.shape[0], -1), zt.expand(ro.shape[0], -1)
    torch.manual_seed(4242)
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                                    (zse, zte))
    torch.manual_seed(4242)
    t_rand, u = torch.rand(2048, 64), torch.rand(2048, 64)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    pw = {f"gnorm_{k}.{n}": p.grad.norm() for k, mm in models.items() for n, p in mm.named_parameters()}
    save("eval_c5.npz", target=target, select_inds=sel.astype(np.int64), theta=theta, phi=phi, rho=rho,
         z_s=zs, z_t=zt, t_rand=t_rand, u=u, rgb_coarse=rgb_c, rgb_fine=rgb_f, loss=loss, g_theta=theta.grad,
         g_phi=phi.grad, g_rho=rho.grad, g_z_s=zs.grad, g_z_t=zt.grad,
         g_fine_fc_rgb_w=models["nerf_fine"].fc_rgb.weight.grad,
         g_coarse_layer_xyz1_w=models["nerf_coarse"].layer_xyz1.weight.grad, **pw)


def gen_se3(nerf, model_mod, ev):
    """eval.py:161-162's pose error through the reference's own utils.SE3.Log (lieutils.py:709-718)."""
    import importlib
    util = importlib.import_module("view_synthesis.utils")
    g = torch.Generator().manual_seed(23)
    gts, cams = [], []
    for k in range(24):
        th, ph, rh = (torch.rand(3, generator=g) * torch.tensor([3.0, 6.2, 1.0]) + torch.tensor([-1.5, -3.1, 0.8]))
        gt = ev.pose_spherical(th[None], ph[None], rh[None])
        d = torch.randn(3, generator=g) * (0.3 if k < 16 else 1e-4)   # small and tiny perturbations
        cam = ev.pose_spherical((th + d[0])[None], (ph + d[1])[None], (rh + d[2])[None])
        gts.append(gt)
        cams.append(cam)
    gts.append(gts[0])
    cams.append(gts[0].clone())                       # identical poses: (tr - 1) / 2 rounds to >= 1
    gt, cam = torch.stack(gts), torch.stack(cams)
    twist = torch.stack([util.SE3.Log(torch.matmul(torch.inverse(a), b)) for a, b in zip(gt, cam)])
    err = torch.stack([torch.norm(util.SE3.Log(torch.matmul(torch.inverse(a), b)), p=2) for a, b in zip(gt, cam)])
    save("se3_pose_error.npz", gt=gt, cam=cam, twist=twist, err=err)


def gen_srn(nerf, model_mod, ev):
    """The reference's SRNDataset (dataset.py:10-94) over the tiny synthetic tree of srn_tree.py.
    imageio is not installed: the harness maps imageio.imread to Pillow (imageio's PNG backend)."""
    import importlib
    import tempfile
    from PIL import Image
    sys.path.insert(0, HERE)
    import srn_tree
    sys.modules["imageio"].imread = lambda path: np.asarray(Image.open(path))
    ds_mod = importlib.import_module("view_synthesis.datasets.dataset")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        base = srn_tree.write_tree(tmp)
        for stage in ("train", "val"):
            ds = ds_mod.SRNDataset(base, stage)
            out[f"{stage}_num_objects"] = ds.num_objects
            out[f"{stage}_num_views"] = ds.num_views
            out[f"{stage}_files"] = np.array([os.path.relpath(str(p), base) for _, p in ds.rgb_all_filenames])
            for i in range(len(ds)):       # RGB and RGBA files: channel counts differ per item
                for k, v in ds[i].items():
                    out[f"{stage}_{i}_{k}"] = np.asarray(v)
    save("srn_tiny.npz", **out)


def gen_loss(nerf, model_mod, ev):
    """train.py:103-107 / eval.py:157-160 loss terms and their gradients on random inputs."""
    g = torch.Generator().manual_seed(31)
    R = 300
    rgb_c, rgb_f = torch.rand(R, 3, generator=g).requires_grad_(True), torch.rand(R, 3, generator=g).requires_grad_(True)
    target = torch.rand(R, 4, generator=g)
    zs, zt = (torch.randn(1, 256, generator=g) * 0.3).requires_grad_(True), (torch.randn(1, 256, generator=g) * 0.3).requires_grad_(True)
    zse, zte = zs.expand(R, -1), zt.expand(R, -1)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], target[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], target[..., :3])
    reg = 1e-2 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss = lc + lf + reg
    loss.backward()
    save("loss.npz", rgb_c=rgb_c, rgb_f=rgb_f, target=target, z_s=zs, z_t=zt, lam=np.float32(1e-2), lc=lc, lf=lf,
         reg=reg, loss=loss, g_rgb_c=rgb_c.grad, g_rgb_f=rgb_f.grad, g_z_s=zs.grad, g_z_t=zt.grad)


C3_OBJECTS = 2458                    # SRN cars train objects (BASELINE.json config 3)
C3_IDS = (17, 1234)                  # the two objects of the chunk (2048 rays each)
C3_FULL = ("nerf_coarse.layer_dir1.weight", "nerf_coarse.shape_code_layer1.weight", "nerf_fine.fc_rgb.weight",
           "nerf_fine.fc_out.bias", "nerf_fine.layer_xyz1.weight")


def gen_c3train(nerf, model_mod, ev):
    """C3 training at size (srn-cars-code.yml with 64 + 64 samples): the reference's own chunk step,
    train.py:96-114 -- embedding lookup, predict_radiance_and_render, mse(coarse) + mse(fine) +
    lambda (||shape table|| + ||texture table||), zero_grad, backward, AdamW (util.py:157-162 groups:
    coarse, fine, embedding at embedding_lr), LambdaLR -- on ONE 4096-ray chunk made of two views of
    two objects of a 2458-object table (2048 rays each, ray_sampler.sample), perturbed samples
    (uniforms recorded).  Stored: the inputs the test cannot regenerate (rays, ids, targets, draws),
    the losses, and element-wise evidence for every parameter: nerf_fine's gradients and post-step
    values in full; for nerf_coarse (size: the full set would double the fixture) the full five
    tensors of round 3 plus, for EVERY tensor, C3_PROJ seeded Gaussian projections of its gradient
    and of its post-step change (proj_seed: the test regenerates the same directions) -- a
    projection sees any error pattern (sign, swapped block) of a size a norm would miss; the
    touched code-table rows' gradients and post-step values.  Weights: codenerf.synthetic
    (seeds 0 / 1), table: synthetic.latent_codes(40 / 41, 2458)."""
    util = importlib.import_module("view_synthesis.utils.util")
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=2048, device="cpu", datatype=torch.float32)
    ps = nerf.PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=True, dtype=torch.float32,
                           device="cpu")
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 0).train(), "nerf_fine": make_model(model_mod, 1).train()}
    table = model_mod.ShapeTextureEmbedding(C3_OBJECTS, 256, 256)
    with torch.no_grad():
        table.shape_embedding.weight.copy_(synthetic.latent_codes(40, C3_OBJECTS))
        table.texture_embedding.weight.copy_(synthetic.latent_codes(41, C3_OBJECTS))
    models["embedding"] = table
    cfg = Cfg(optimizer=Cfg(type="AdamW", lr=1e-4, embedding_lr=1e-3, scheduler_gamma=0.1,
                            scheduler_step_size=5000000))
    optimizer, scheduler = util.prepare_optimizer(cfg, models)
    g = torch.Generator().manual_seed(61)
    colors = torch.rand(2, 128, 128, 4, generator=g)
    poses = torch.cat([_pose(ev, 0.5, 0.3, 1.3)[None], _pose(ev, 1.0, -0.6, 1.3)[None]])
    ids = torch.tensor(C3_IDS)
    np.random.seed(29)
    ro, rd, sel = rs.sample(tform_cam2world=poses)                       # train.py:76
    tgt = torch.cat([colors.flatten(1, 2)[k, sel[k], :] for k in range(2)], dim=0)   # train.py:77-80
    oid = ids[:, None].expand(-1, 2048).reshape(-1)
    before = {f"{k}.{n}": p.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    torch.manual_seed(4343)
    target_object_embedding = models["embedding"](oid)                  # train.py:96-101
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                                    target_object_embedding)
    torch.manual_seed(4343)
    t_rand, u = torch.rand(4096, 64), torch.rand(4096, 64)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tgt[..., :3])    # train.py:103-108
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tgt[..., :3])
    sp, tpar = model_mod.get_params_tensor(models["embedding"], False)
    reg = 1e-5 * (torch.norm(sp, p=2) + torch.norm(tpar, p=2))
    loss = lc + lf + reg
    optimizer.zero_grad()                                               # train.py:111-114
    loss.backward()
    grads = {f"{k}.{n}": p.grad.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    optimizer.step()
    scheduler.step()
    after = {f"{k}.{n}": p.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    # the draws are re-made by the test from the same seed (torch CPU generator); head + sums pin them
    out = dict(ro=ro, rd=rd, ids=oid, target=tgt, t_rand_head=t_rand[:4], u_head=u[:4],
               t_rand_sum=t_rand.double().sum(), u_sum=u.double().sum(), select_inds=sel.astype(np.int64),
               rgb_coarse=rgb_c, rgb_fine=rgb_f, lc=lc, lf=lf, reg=reg, loss=loss)
    for k in grads:
        if k.startswith("embedding."):
            out["grows_" + k] = grads[k][list(C3_IDS)]
            out["prows_" + k] = after[k][list(C3_IDS)]
            # every other row: no gradient, weight decay only (AdamW decays every row of the table)
            out["gnorm_rest_" + k] = grads[k].norm() ** 2 - grads[k][list(C3_IDS)].norm() ** 2
        else:
            out["gnorm_" + k] = grads[k].norm()
            out["pdelta_norm_" + k] = (after[k] - before[k]).norm()
    for k in C3_FULL:
        out["g_" + k] = grads[k]
        out["p_" + k] = after[k]
    for idx, k in enumerate(sorted(grads)):
        if k.startswith("embedding."):
            continue
        if k.startswith("nerf_fine."):
            out["g_" + k] = grads[k]
            out["p_" + k] = after[k]
        r = proj_directions(idx, grads[k].shape)
        out["gproj_" + k] = proj(r, grads[k])
        out["pproj_" + k] = proj(r, after[k] - before[k])
    save("train_c3.npz", **out)


C3_PROJ = 16

# The reference's runnable training shapes (round 6): one chunk step each, like gen_c3train but with
# ONE object per chunk (train_batch_size images of num_random_rays each, chunk <= num_random_rays: a
# chunk is always a slice of one image).  (config file, Nc, Nf, near, far, rays drawn per image, chunk,
# object id, pose).  Stored like train_c3.npz minus the full nerf_fine tensors (size): C3_FULL in full,
# 16 projections of every tensor's gradient and post-step change, the touched code rows.
TRAIN_SHAPES = {
    "train_cars_code": ("config/srn-cars-code.yml:45-48,63", 32, 128, 0.8, 1.8, 4096, 4096, 611, (0.7, -0.4, 1.3)),
    "train_3080": ("config/srn-cars-code-3080.yml:45-48,62", 64, 128, 0.8, 1.8, 4096, 1024, 2001, (0.9, 1.1, 1.3)),
}


def gen_train_shape(nerf, model_mod, ev, name):
    """train.py:76-114 at one of TRAIN_SHAPES: ray_sampler.sample of one view (num_random_rays), the
    target gather, get_minibatches' FIRST chunk, then the chunk step (embedding lookup,
    predict_radiance_and_render with perturbed samples -- draws re-made by the tests from
    torch.manual_seed(4343): t_rand (chunk, Nc) then u (chunk, Nf) -- losses, zero_grad, backward, AdamW +
    LambdaLR).  Weights: codenerf.synthetic seeds 0 / 1; tables synthetic.latent_codes(40 / 41, 2458)."""
    util = importlib.import_module("view_synthesis.utils.util")
    _src, nc, nf, near, far, n_rays, chunk, oid_v, cam = TRAIN_SHAPES[name]
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=n_rays, device="cpu", datatype=torch.float32)
    ps = nerf.PointSampler(nc, nf, near, far, spacing_mode="lindepth", perturb=True, dtype=torch.float32,
                           device="cpu")
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 0).train(), "nerf_fine": make_model(model_mod, 1).train()}
    table = model_mod.ShapeTextureEmbedding(C3_OBJECTS, 256, 256)
    with torch.no_grad():
        table.shape_embedding.weight.copy_(synthetic.latent_codes(40, C3_OBJECTS))
        table.texture_embedding.weight.copy_(synthetic.latent_codes(41, C3_OBJECTS))
    models["embedding"] = table
    cfg = Cfg(optimizer=Cfg(type="AdamW", lr=1e-4, embedding_lr=1e-3, scheduler_gamma=0.1,
                            scheduler_step_size=5000000))
    optimizer, scheduler = util.prepare_optimizer(cfg, models)
    g = torch.Generator().manual_seed(62)
    colors = torch.rand(1, 128, 128, 4, generator=g)
    poses = _pose(ev, *cam)[None]
    np.random.seed(30)
    ro_b, rd_b, sel = rs.sample(tform_cam2world=poses)                    # train.py:76
    tgt_b = colors.flatten(1, 2)[0, sel[0], :]                            # train.py:77-80
    ro, rd, tgt = util.get_minibatches(ro_b, chunk)[0], util.get_minibatches(rd_b, chunk)[0], \
        util.get_minibatches(tgt_b, chunk)[0]                             # train.py:84-85
    oid = torch.full((chunk,), oid_v, dtype=torch.int64)
    before = {f"{k}.{n}": p.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    torch.manual_seed(4343)
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                                    models["embedding"](oid))
    torch.manual_seed(4343)
    t_rand, u = torch.rand(chunk, nc), torch.rand(chunk, nf)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tgt[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tgt[..., :3])
    sp, tpar = model_mod.get_params_tensor(models["embedding"], False)
    reg = 1e-5 * (torch.norm(sp, p=2) + torch.norm(tpar, p=2))
    loss = lc + lf + reg
    optimizer.zero_grad()
    loss.backward()
    grads = {f"{k}.{n}": p.grad.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    optimizer.step()
    scheduler.step()
    after = {f"{k}.{n}": p.detach().clone() for k, m in models.items() for n, p in m.named_parameters()}
    out = dict(nc=nc, nf=nf, near=np.float32(near), far=np.float32(far), chunk=chunk,
               ro=ro, rd=rd, ids=oid, target=tgt, t_rand_head=t_rand[:4], u_head=u[:4],
               t_rand_sum=t_rand.double().sum(), u_sum=u.double().sum(), select_inds=sel.astype(np.int64),
               rgb_coarse=rgb_c, rgb_fine=rgb_f, lc=lc, lf=lf, reg=reg, loss=loss)
    for k in grads:
        if k.startswith("embedding."):
            out["grows_" + k] = grads[k][[oid_v]]
            out["prows_" + k] = after[k][[oid_v]]
            out["gnorm_rest_" + k] = grads[k].norm() ** 2 - grads[k][[oid_v]].norm() ** 2
        else:
            out["gnorm_" + k] = grads[k].norm()
            out["pdelta_norm_" + k] = (after[k] - before[k]).norm()
    for k in C3_FULL:
        out["g_" + k] = grads[k]
        out["p_" + k] = after[k]
    for idx, k in enumerate(sorted(grads)):
        if k.startswith("embedding."):
            continue
        r = proj_directions(idx, grads[k].shape)
        out["gproj_" + k] = proj(r, grads[k])
        out["pproj_" + k] = proj(r, after[k] - before[k])
    save(name + ".npz", **out)


def gen_train_cars_code(nerf, model_mod, ev):
    gen_train_shape(nerf, model_mod, ev, "train_cars_code")


def gen_train_3080(nerf, model_mod, ev):
    gen_train_shape(nerf, model_mod, ev, "train_3080")


def gen_c5_chairs(nerf, model_mod, ev):
    """eval.py:141-168 at srn-chairs-code.yml:47-54's shape: num_random_rays 4096 of a 128x128 view, 32
    coarse + 128 fine perturbed samples, near 1.25 / far 2.75, the whole batch in one
    predict_radiance_and_render; gradients into theta, phi, rho and both codes (weights require grad, as
    in eval.py).  The draws are re-made by the tests from torch.manual_seed(4244): t_rand (4096, 32), then
    u (4096, 128); head and sums stored."""
    K = synthetic.srn_intrinsics(128)
    rs = nerf.RaySampler(128, 128, K, sample_size=4096, device="cpu", datatype=torch.float32)
    ps = nerf.PointSampler(32, 128, 1.25, 2.75, spacing_mode="lindepth", perturb=True, dtype=torch.float32,
                           device="cpu")
    emb = _embedders(nerf)
    models = {"nerf_coarse": make_model(model_mod, 0), "nerf_fine": make_model(model_mod, 1)}
    for mm in models.values():
        mm.train()
    g = torch.Generator().manual_seed(32)
    target = torch.rand(128 * 128, 4, generator=g)
    theta = torch.tensor([1.1]).requires_grad_(True)
    phi = torch.tensor([-0.5]).requires_grad_(True)
    rho = torch.tensor([2.0]).requires_grad_(True)
    zs = synthetic.latent_codes(7, 1).clone().requires_grad_(True)
    zt = synthetic.latent_codes(8, 1).clone().requires_grad_(True)
    np.random.seed(18)
    c2w = ev.pose_spherical(theta, phi, rho)[None, :]
    ro, rd, sel = rs.sample(tform_cam2world=c2w)
    tp = target[None][..., sel, :].squeeze()
    zse, zte = zs.expand(ro.shape[0], -1), zt.expand(ro.shape[0], -1)
    torch.manual_seed(4244)
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                                    (zse, zte))
    torch.manual_seed(4244)
    t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    loss = lc + lf + 1e-5 * (torch.norm(zse, p=2) + torch.norm(zte, p=2))
    loss.backward()
    pw = {f"gnorm_{k}.{n}": p.grad.norm() for k, mm in models.items() for n, p in mm.named_parameters()}
    save("eval_c5_chairs.npz", target=target,
         select_inds=sel.astype(np.int64), theta=theta, phi=phi, rho=rho, z_s=zs, z_t=zt,
         t_rand_head=t_rand[:4], u_head=u[:4], t_rand_sum=t_rand.double().sum(), u_sum=u.double().sum(),
         rgb_coarse=rgb_c, rgb_fine=rgb_f, loss=loss, g_theta=theta.grad, g_phi=phi.grad, g_rho=rho.grad,
         g_z_s=zs.grad, g_z_t=zt.grad, g_fine_fc_rgb_w=models["nerf_fine"].fc_rgb.weight.grad,
         g_coarse_layer_xyz1_w=models["nerf_coarse"].layer_xyz1.weight.grad, **pw)


def proj_directions(idx: int, shape) -> torch.Tensor:
    """C3_PROJ seeded N(0, 1) directions for parameter ``idx`` (sorted-name order), float32 CPU."""
    return torch.randn((C3_PROJ,) + tuple(shape), generator=torch.Generator().manual_seed(7000 + idx))


def proj(r: torch.Tensor, t: torch.Tensor) -> np.ndarray:
    """<r_k, t> for every direction, accumulated in float64."""
    return (r.double() * t.detach().double()[None]).reshape(r.shape[0], -1).sum(1).numpy()


ROUND2 = {"trained": gen_trained, "chairs": gen_chairs, "lego": gen_lego, "c5": gen_c5, "se3": gen_se3,
          "srn": gen_srn, "loss": gen_loss}
ROUND3 = {"c3train": gen_c3train}
ROUND6 = {"train_cars_code": gen_train_cars_code, "train_3080": gen_train_3080, "c5_chairs": gen_c5_chairs}


if __name__ == "__main__":
    main(sys.argv[1:] or None)
