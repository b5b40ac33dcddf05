"""Round-2 rows of SURVEY.md section 8(f) on the HIP path: the fused pose path (row 3), the fused
step loss, the SE3 pose metric and checkpoint resume (row 4), the HBM-resident SRN store (row 2),
and the end of eval.py's validate() (the full-view render + PSNR after test-time optimisation).

Oracles: oracle/codenerf_oracle.py (pinned to the reference by tests/golden/*.npz, see
test_oracle_golden.py) and the reference's own fixtures (eval_grad.npz, eval_c5.npz,
se3_pose_error.npz, loss.npz, srn_tiny.npz).  Tolerances as the rest of the GPU suite: rays 1e-6,
rendered rgb 1e-4, gradients relative to the tensor's largest magnitude (test_gpu_grad.close).
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from test_gpu_grad import GRAD_RTOL, close, dev, embedders, model  # noqa: F401

pytestmark = pytest.mark.gpu


def O():
    import oracle.codenerf_oracle as o
    return o


def gload(name, dev):
    return {k: torch.from_numpy(v).to(dev) for k, v in np.load(os.path.join(GOLDEN, name)).items()}


def small_sampler(dev, rng="numpy", sample_size=64):
    from codenerf.nerf import RaySampler
    K = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays_small.npz"))["intrinsics"])
    return RaySampler(12, 16, K, sample_size=sample_size, device=dev, datatype=torch.float32, rng=rng), K


# ---------------------------------------------------------------- fused pose path (8(f) row 3)


def test_sample_c2w_equals_bundle_then_gather(dev):
    """RaySampler.sample now computes only the selected rays (one cn_pose_rays launch): bit for bit
    the rays of get_bundle + the gather (ray_sampler.py:53-99), same numpy draws."""
    from codenerf import ops
    rs, _ = small_sampler(dev, sample_size=40)
    g = np.load(os.path.join(GOLDEN, "rays_small.npz"))
    poses = torch.from_numpy(g["poses"]).to(dev)
    np.random.seed(7)
    ro, rd, sel = rs.sample(poses)
    assert np.array_equal(sel, g["select_inds"])
    ro_b, rd_b = ops.ray_bundle(rs.directions, poses)
    o, d = ops.gather_rays(ro_b.reshape(2, -1, 3), rd_b.reshape(2, -1, 3), torch.from_numpy(sel).to(dev))
    assert torch.equal(ro, o) and torch.equal(rd, d)
    assert torch.equal(ro.cpu(), torch.from_numpy(g["ro_sel"]))
    assert (rd.cpu() - torch.from_numpy(g["rd_sel"])).abs().max().item() <= 1e-6


def test_pose_rays_spherical_forward_and_grads(dev):
    """pose_spherical -> selected rays -> target rows, and d(theta, phi, rho) through the analytic
    d c2w, vs torch autograd over the oracle (eval.py:22-38 + ray_sampler.py:84-99)."""
    o = O()
    from codenerf.autograd import pose_rays_autograd
    rs, K = small_sampler(dev)
    g = torch.Generator().manual_seed(3)
    B, S = 3, 50
    ang = [torch.rand(B, generator=g) * 2 - 1, torch.rand(B, generator=g) * 6 - 3, torch.rand(B, generator=g) + 1]
    sel = torch.stack([torch.randperm(192, generator=g)[:S] for _ in range(B)])
    target = torch.rand(B, 192, 4, generator=g)
    g_ro, g_rd = torch.randn(B * S, 3, generator=g), torch.randn(B * S, 3, generator=g)
    th, ph, rh = [a.to(dev).requires_grad_(True) for a in ang]
    ro, rd, c2w, tp = pose_rays_autograd(rs.directions, th, ph, rh, sel=sel.to(dev), target=target.to(dev))
    ((ro * g_ro.to(dev)).sum() + (rd * g_rd.to(dev)).sum()).backward()
    # oracle
    tc, pc, rc = [a.clone().requires_grad_(True) for a in ang]
    poses = torch.stack([o.pose_spherical(tc[b:b + 1], pc[b:b + 1], rc[b:b + 1]) for b in range(B)])
    d = o.ray_directions(12, 16, K)
    ro_b, rd_b = o.ray_bundle(d, poses)
    ro_r, rd_r = o.gather_rays(ro_b, rd_b, sel.numpy())
    ((ro_r * g_ro).sum() + (rd_r * g_rd).sum()).backward()
    assert (c2w.cpu() - poses.detach()).abs().max().item() <= 1e-6
    assert (ro.detach().cpu() - ro_r.detach()).abs().max().item() <= 1e-6
    assert (rd.detach().cpu() - rd_r.detach()).abs().max().item() <= 1e-6
    assert torch.equal(tp.cpu(), torch.cat([target[b, sel[b]] for b in range(B)]))
    for got, ref, what in ((th.grad, tc.grad, "theta"), (ph.grad, pc.grad, "phi"), (rh.grad, rc.grad, "rho")):
        close(got, ref, 1e-5, what)


def test_pose_rays_c2w_grad(dev):
    """The c2w path's backward (train.py's sample of given poses, differentiable in c2w) vs the
    get_bundle + gather backward kernels."""
    from codenerf import ops
    from codenerf.autograd import pose_rays_autograd, ray_bundle_autograd, gather_rays_autograd
    rs, _ = small_sampler(dev)
    g = torch.Generator().manual_seed(5)
    c2w = (torch.eye(4).repeat(2, 1, 1) + 0.1 * torch.randn(2, 4, 4, generator=g)).to(dev)
    sel = torch.stack([torch.randperm(192, generator=g)[:30] for _ in range(2)]).to(dev)
    go, gd = torch.randn(60, 3, generator=g).to(dev), torch.randn(60, 3, generator=g).to(dev)
    a = c2w.clone().requires_grad_(True)
    ro, rd, _, _ = pose_rays_autograd(rs.directions, c2w=a, sel=sel)
    ((ro * go).sum() + (rd * gd).sum()).backward()
    b = c2w.clone().requires_grad_(True)
    rob, rdb = ray_bundle_autograd(rs.directions, b)
    ro2, rd2 = gather_rays_autograd(rob.reshape(2, -1, 3), rdb.reshape(2, -1, 3), sel)
    ((ro2 * go).sum() + (rd2 * gd).sum()).backward()
    close(a.grad, b.grad, 1e-5, "d c2w")
    assert ops is not None


def test_random_select_device(dev):
    """cn_random_select: distinct in-range pixels per image, reproducible per (seed, offset), a new
    draw per offset, and uniform over pixels (chi-square over many draws)."""
    from codenerf import ops
    a = ops.random_select(4, 16384, 4096, seed=11, offset=0, device=dev)
    b = ops.random_select(4, 16384, 4096, seed=11, offset=0, device=dev)
    c = ops.random_select(4, 16384, 4096, seed=11, offset=1, device=dev)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert a.min().item() >= 0 and a.max().item() < 16384
    for row in a.cpu():
        assert row.unique().numel() == 4096
    assert not torch.equal(a[0], a[1])
    counts = torch.zeros(192, dtype=torch.float64)
    draws = ops.random_select(2000, 192, 48, seed=3, offset=9, device=dev).cpu()
    counts.index_add_(0, draws.reshape(-1), torch.ones(draws.numel(), dtype=torch.float64))
    exp = draws.numel() / 192
    chi2 = (((counts - exp) ** 2) / exp).sum().item()
    assert chi2 < 191 + 6 * (2 * 191) ** 0.5, chi2          # ~6 sigma for 191 degrees of freedom
    # first-position uniformity: the order is random too
    first = torch.bincount(draws[:, 0], minlength=192).double()
    assert first.max().item() < 2000 / 192 * 4


def test_random_select_rejects_large_images(dev):
    from codenerf import ops
    from codenerf._lib import CodeNerfError
    with pytest.raises(CodeNerfError):
        ops.random_select(1, 16385, 10, seed=0, offset=0, device=dev)


def test_sampler_device_rng_mode(dev):
    rs, _ = small_sampler(dev, rng="device")
    th, ph, rh = (torch.tensor([v], device=dev) for v in (0.5, 0.3, 1.3))
    target = torch.rand(192, 4, device=dev)
    ro, rd, sel, cam, tp = rs.sample_spherical(th, ph, rh, target=target)
    assert torch.is_tensor(sel) and sel.shape == (1, 64) and sel.device.type == "cuda"
    assert torch.equal(tp, target[sel[0]])
    ro2, rd2, sel2, _, _ = rs.sample_spherical(th, ph, rh)
    assert not torch.equal(sel, sel2)


# ---------------------------------------------------------------- the fused eval step vs the reference


def _eval_models(dev, frozen=True):
    ms = {"nerf_coarse": model(dev, 0), "nerf_fine": model(dev, 1)}
    for m in ms.values():
        m.train()
        m.requires_grad_(not frozen)
    return ms


def test_eval_step_fused_golden(dev):
    """eval.py:145-160 through the fused pose path + fused loss vs the reference's own autograd
    (eval_grad.npz: 12x16 view, 64 rays, 8+8 samples)."""
    from codenerf.evaluate import eval_step_loss
    from codenerf.nerf import PointSampler
    gd = gload("eval_grad.npz", dev)
    rs, _ = small_sampler(dev)
    ps = PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    models = _eval_models(dev)
    theta, phi, rho = [gd[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = gd["z_s"].clone().requires_grad_(True), gd["z_t"].clone().requires_grad_(True)
    np.random.seed(9)
    loss, logs = eval_step_loss(theta, phi, rho, zs, zt, gd["target"], (rs, ps), embedders(dev), models, 1e-5)
    loss.backward()
    assert abs(loss.item() - gd["loss"].item()) <= 1e-5
    for name, t in [("theta", theta), ("phi", phi), ("rho", rho)]:
        ref = gd["g_" + name]
        assert (t.grad - ref).abs().max().item() <= 1e-3 * max(1.0, ref.abs().max().item()), name
    close(zs.grad, gd["g_z_s"], 1e-3, "g_z_s")
    close(zt.grad, gd["g_z_t"], 1e-3, "g_z_t")


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_eval_c5_fused_at_size(dev, precision):
    """C5 at size (2048 rays of 128x128, 64+64 perturbed, the reference's draws injected) through
    eval_step_loss's fused path: loss and d(theta, phi, rho, z_s, z_t) vs the reference."""
    from codenerf import synthetic
    from codenerf.evaluate import eval_step_loss
    from codenerf.nerf import PointSampler, RaySampler
    g = gload("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    for m in models.values():
        m.precision = precision
    theta, phi, rho = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho")]
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    np.random.seed(17)
    loss, logs = eval_step_loss(theta, phi, rho, zs, zt, g["target"], (rs, ps), embedders(dev), models, 1e-5,
                                t_rand=g["t_rand"], u=g["u"])
    loss.backward()
    assert abs(loss.item() - g["loss"].item()) <= 1e-5
    for name, t in [("theta", theta), ("phi", phi), ("rho", rho)]:
        ref = g["g_" + name]
        err = (t.grad - ref).abs().max().item()
        print(f"{precision} {name}: grad {t.grad.item():.6e} ref {ref.item():.6e}")
        assert err <= 2e-3 * max(1e-2, ref.abs().max().item()), name
    close(zs.grad, g["g_z_s"], 2e-3, "g_z_s")
    close(zt.grad, g["g_z_t"], 2e-3, "g_z_t")


# twice the largest error the first GPU run measured (d z_s 4.83e-5, loss 3.9e-7; gpurun_out/r06a,
# profiles/r06/parity_margins.json); the eval step is bit-reproducible
C5_CHAIRS_RTOL = 1e-4
C5_CHAIRS_LOSS = 1e-6


def test_eval_c5_chairs_fused_at_size(dev):
    """eval.py:141-168 at srn-chairs-code.yml's shape (make_golden.py gen_c5_chairs: num_random_rays 4096
    of a 128x128 view, 32 + 128 perturbed samples -- a 160-sample fine pass -- near 1.25 / far 2.75, the
    reference's draws re-made from its seed) through eval_step_loss's fused path, fp32: rendered rgb,
    loss and d(theta, phi, rho, z_s, z_t) vs the reference; a second run bit for bit."""
    from codenerf import synthetic
    from codenerf.evaluate import eval_step_loss
    from codenerf.nerf import PointSampler, RaySampler
    from conftest import margin
    g = gload("eval_c5_chairs.npz", dev)
    torch.manual_seed(4244)
    t_rand, u = torch.rand(4096, 32), torch.rand(4096, 128)
    assert torch.equal(t_rand[:4].to(dev), g["t_rand_head"]) and torch.equal(u[:4].to(dev), g["u_head"])
    t_rand, u = t_rand.to(dev), u.to(dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=4096, device=dev, datatype=torch.float32)
    ps = PointSampler(32, 128, 1.25, 2.75, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    runs = []
    for rep in range(2):
        lv = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]
        np.random.seed(18)
        loss, logs = eval_step_loss(*lv, g["target"], (rs, ps), embedders(dev), models, 1e-5, t_rand=t_rand, u=u)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.item(), [t.grad.clone() for t in lv]))
    assert runs[0][0] == runs[1][0]
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)
    tag = "eval_c5_chairs[f32]"
    margin(tag, "loss", abs(runs[0][0] - g["loss"].item()), C5_CHAIRS_LOSS)
    for name, t in zip(("theta", "phi", "rho", "z_s", "z_t"), runs[0][1]):
        ref = g["g_" + name]
        scale = max(1e-2, ref.abs().max().item()) if name in ("theta", "phi", "rho") else ref.abs().max().item()
        margin(tag, "d " + name, (t - ref).abs().max().item() / scale, C5_CHAIRS_RTOL)


def test_ray_sharded_step_equals_full_batch(dev):
    """The ray-sharded eval step's weighting (evaluate.sharded_eval_step: each share's loss weighted by
    share / rays, the regulariser expanded over ALL the iteration's rows, the shares' gradients summed)
    against the unsharded full-batch step.  The one intended difference -- each share is its own Q1
    chunk, so the view direction paired with a sample differs -- is taken out by zeroing the view-direction
    columns of both fields' layer_dir1 (the radiance then does not depend on the view direction at all):
    the two shares' summed loss terms and code / pose gradients must then equal the full batch's to fp32
    reassociation.  A weighting error common to the sharded path (the rows_total expand, the n / N scale)
    would show here."""
    from codenerf import synthetic
    from codenerf.evaluate import eval_step_loss, shard_of
    from codenerf.nerf import PointSampler, RaySampler
    g = gload("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    with torch.no_grad():
        for m in models.values():
            m.layer_dir1.weight[:, 256:].zero_()        # [feat | 27 view-encoding columns]: no view dependence
    sel = torch.from_numpy(g["select_inds"].cpu().numpy().reshape(1, -1)).to(dev)
    n = sel.shape[1]
    runs = {}
    for mode in ("full", "sharded"):
        lv = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]
        parts = [slice(0, n)] if mode == "full" else [shard_of(n, 2, r) for r in range(2)]
        total, terms = 0.0, torch.zeros(3, dtype=torch.float64)
        for sl in parts:
            kw = {} if mode == "full" else dict(rows_total=n)
            loss, logs = eval_step_loss(*lv, g["target"], (rs, ps), embedders(dev), models, 1e-5, t_rand=g["t_rand"][sl],
                                        u=g["u"][sl], sel=sel[:, sl], **kw)
            loss.backward()
            w = (sl.stop - sl.start) / n
            total += loss.item()
            terms += torch.tensor([float(logs["nerf_loss_coarse"]) * w, float(logs["nerf_loss_fine"]) * w,
                                   float(logs["embedding_loss"])], dtype=torch.float64)
        runs[mode] = (total, terms, [t.grad.detach().clone() for t in lv])
    (lf, tf, gf), (ls, ts, gs) = runs["full"], runs["sharded"]
    assert abs(ls - lf) <= 1e-6 * abs(lf), (ls, lf)
    assert abs(ts[0] - tf[0]) <= 1e-6 * tf[0] and abs(ts[1] - tf[1]) <= 1e-6 * tf[1], (ts, tf)
    assert ts[2] / 2 == tf[2], "the regulariser of each share is the whole iteration's (expanded over all rows)"
    for name, a, b in zip(("theta", "phi", "rho", "z_s", "z_t"), gs, gf):
        err = (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)
        assert err <= 1e-5, (name, err)


def test_eval_step_paired_fields(dev, monkeypatch):
    """eval_step_loss pairs the two fields' fused backwards (autograd.FieldPair: the fine field's waits, the
    coarse volume render's d rd is held for it, then ONE cn_field_backward_fused_multi call runs both and one
    cn_code_bias_backward_act_multi their code halves): every gradient -- codes and pose -- and the loss bit
    for bit those of the unpaired step, on the C5 fixture."""
    from codenerf import autograd as A, ops, synthetic
    from codenerf.evaluate import eval_step_loss
    from codenerf.nerf import PointSampler, RaySampler
    from codenerf.optim import AdamW
    g = gload("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    calls = []
    real = ops.field_backward_x3_multi

    def spy(*a, **k):
        calls.append(1)
        return real(*a, **k)
    monkeypatch.setattr(ops, "field_backward_x3_multi", spy)
    out = []
    for paired in (True, False):
        if not paired:
            monkeypatch.setattr(A, "new_field_pair", lambda: None)
        calls.clear()
        lv = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]
        opt = AdamW([{"params": lv[3:]}, {"params": lv[:2]}, {"params": lv[2:3]}], lr=1e-2)
        opt.zero_grad()
        np.random.seed(17)
        loss, _ = eval_step_loss(*lv, g["target"], (rs, ps), embedders(dev), models, 1e-5, t_rand=g["t_rand"],
                                 u=g["u"])
        A.backward_from(loss)
        torch.cuda.synchronize()
        out.append((loss.item(), [t.grad.clone() for t in lv], len(calls)))
    assert out[0][2] == 1 and out[1][2] == 0, (out[0][2], out[1][2])
    assert out[0][0] == out[1][0]
    for name, a, b in zip(("theta", "phi", "rho", "z_s", "z_t"), out[0][1], out[1][1]):
        assert torch.equal(a, b), (name, (a - b).abs().max().item())


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_eval_step_in_place_gradients(dev, monkeypatch, precision):
    """The eval step's gradient sinks (C5 inputs, the flat AdamW's zeroed slots handed out by zero_grad):
    the codes' gradients added in place into the leaves' slots by the loss and both fields (one dz launch
    for both; code_rows_with_sink's CodeGradSink), the rays' by both volume renders and both fields into
    the fine field's zeroed accumulators (RaySink), the pose angles' written into their slots -- every
    leaf's .grad is then its flat slice (no autograd adds, no copy into the flat buffer) -- against the
    route through autograd: the loss and every gradient bit for bit (the same sums in the same order, and
    the eval backward's g_code / ray sums are fixed-order, cn_field_backward_fused_ws).
    torch.autograd.grad through the sinks returns the same code gradients."""
    from codenerf import autograd as A, synthetic
    from codenerf.evaluate import eval_step_loss
    from codenerf.models import model as M
    from codenerf.nerf import PointSampler, RaySampler
    from codenerf.optim import AdamW
    g = gload("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    for m in models.values():
        m.precision = precision
    out = []
    for on in (True, False):
        if not on:
            monkeypatch.setattr(M.CodeGradSink, "rows", lambda self: None)
            monkeypatch.setattr(A, "_ray_sink", lambda rd, ro=None: None)
        lv = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]
        opt = AdamW([{"params": lv[3:]}, {"params": lv[:2]}, {"params": lv[2:3]}], lr=1e-2)
        opt.zero_grad()
        np.random.seed(17)
        loss, _ = eval_step_loss(*lv, g["target"], (rs, ps), embedders(dev), models, 1e-5, t_rand=g["t_rand"],
                                 u=g["u"])
        A.backward_from(loss)
        torch.cuda.synchronize()
        if on:
            flat = opt.flat_buffers()["grad"]
            lo, hi = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
            for t in lv:
                assert lo <= t.grad.data_ptr() < hi, "a leaf's .grad is not its flat slice"
        out.append((loss.item(), [t.grad.clone() for t in lv]))
    (l0, g0), (l1, g1) = out
    assert l0 == l1
    for name, a, b in zip(("theta", "phi", "rho", "z_s", "z_t"), g0, g1):
        assert torch.equal(a, b), (name, (a - b).abs().max().item())
    # torch.autograd.grad (no .grad accumulation) through the sinks: the same code gradients
    monkeypatch.undo()
    lv = [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]
    opt = AdamW([{"params": lv[3:]}, {"params": lv[:2]}, {"params": lv[2:3]}], lr=1e-2)
    opt.zero_grad()
    np.random.seed(17)
    loss, _ = eval_step_loss(*lv, g["target"], (rs, ps), embedders(dev), models, 1e-5, t_rand=g["t_rand"], u=g["u"])
    gz = torch.autograd.grad(loss, lv[3:])
    for name, a, b in zip(("z_s", "z_t"), gz, g0[3:]):
        assert torch.equal(a, b), ("autograd.grad " + name, (a - b).abs().max().item())


# ---------------------------------------------------------------- the fused step loss


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_graphed_eval_step_matches_eager(dev, precision):
    """GraphedEvalStep (the eval iteration captured once as a HIP graph, replayed per iteration) vs
    the eager eval_step_loss + backward on the same C5 inputs (the reference's injected uniforms,
    the same numpy draws), over two replays: loss and every gradient, bit for bit (the same kernels on
    the same inputs; the eval backward sums in a fixed order)."""
    from codenerf import synthetic
    from codenerf.evaluate import GraphedEvalStep, eval_step_loss
    from codenerf.nerf import PointSampler, RaySampler
    from codenerf.optim import AdamW
    g = gload("eval_c5.npz", dev)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    models = _eval_models(dev)
    for m in models.values():
        m.precision = precision

    def leaves():
        return [g[k].clone().requires_grad_(True) for k in ("theta", "phi", "rho", "z_s", "z_t")]

    eager = []
    np.random.seed(17)
    for _ in range(2):
        th, ph, rh, zs, zt = lv = leaves()
        loss, _ = eval_step_loss(th, ph, rh, zs, zt, g["target"], (rs, ps), embedders(dev), models, 1e-5,
                                 t_rand=g["t_rand"], u=g["u"])
        loss.backward()
        eager.append((loss.item(), [t.grad.clone() for t in lv]))
    th, ph, rh, zs, zt = lv = leaves()
    opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(17)
    step = GraphedEvalStep(th, ph, rh, zs, zt, g["target"], (rs, ps), embedders(dev), models, opt, 1e-5,
                           t_rand=g["t_rand"], u=g["u"], optimizer_in_graph=False)
    for i in range(2):
        loss, _ = step.step()
        torch.cuda.synchronize()
        le, ge = eager[i]
        assert loss.item() == le, (i, loss.item(), le)
        for name, t, ref in zip(("theta", "phi", "rho", "z_s", "z_t"), lv, ge):
            assert torch.equal(t.grad, ref), (f"replay {i} {name}", (t.grad - ref).abs().max().item())


@pytest.mark.parametrize("perturb", [False, True])
def test_time_optimize_graph_matches_eager(dev, perturb):
    """test_time_optimize(graph=True) -- forward, backward and the AdamW update in one replay --
    runs the same iterations as the eager loop (the same numpy draws; perturbed: the same device
    uniforms, since the graph's warm-up draws are rolled back): loss history, codes and pose, bit for
    bit over three iterations (the replayed AdamW is cn_adamw_step's arithmetic, and the eval backward
    sums in a fixed order -- before it did, the two drifted apart at the last bits of g_code's atomic
    sums, which AdamW's per-element normalisation grows towards lr)."""
    from codenerf import synthetic
    from codenerf.evaluate import test_time_optimize
    from codenerf.nerf import PointSampler, RaySampler
    g = gload("eval_c5.npz", dev)
    out = {}
    for graph in (False, True):
        rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev,
                        datatype=torch.float32)
        ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", perturb, torch.float32, dev)
        codes = (synthetic.latent_codes(5, 4).to(dev), synthetic.latent_codes(6, 4).to(dev))
        models = _eval_models(dev)
        np.random.seed(23)
        torch.manual_seed(31)
        zs, zt, pose, hist, cam = test_time_optimize(g["target"], (rs, ps), embedders(dev), models, codes,
                                                     iterations=3, graph=graph)
        out[graph] = (zs.detach(), zt.detach(), torch.cat([p.detach().reshape(-1) for p in pose]), hist, cam)
    e, q = out[False], out[True]
    assert e[3] == q[3], (e[3], q[3])
    for name, x, y in (("z_s", q[0], e[0]), ("z_t", q[1], e[1]), ("pose", q[2], e[2]), ("cam_pose", q[4], e[4])):
        assert torch.equal(x, y), (name, (x - y).abs().max().item())


def test_render_loss_golden(dev):
    """train.py:103-107 / eval.py:157-160 loss terms and gradients vs the reference (loss.npz)."""
    from codenerf.autograd import render_loss_autograd
    g = gload("loss.npz", dev)
    rc, rf = g["rgb_c"].clone().requires_grad_(True), g["rgb_f"].clone().requires_grad_(True)
    zs, zt = g["z_s"].clone().requires_grad_(True), g["z_t"].clone().requires_grad_(True)
    loss, stats = render_loss_autograd(rc, rf, g["target"], zs, zt, expand=300, lam=float(g["lam"]))
    loss.backward()
    # the reference sums 300 x 256 squares of the expanded codes in fp32 (~2e-6 relative rounding);
    # cn_render_loss accumulates in double: 1e-5 relative
    for got, k in ((stats[0], "lc"), (stats[1], "lf"), (stats[2], "reg"), (loss, "loss")):
        assert abs(got.item() - g[k].item()) <= 1e-5 * max(1.0, abs(g[k].item())), k
    for t, k in ((rc, "g_rgb_c"), (rf, "g_rgb_f"), (zs, "g_z_s"), (zt, "g_z_t")):
        close(t.grad, g[k], 1e-5, k)


@pytest.mark.parametrize("n_obj", [7, 2458])
def test_render_loss_train_regulariser_is_constant(dev, n_obj):
    """train.py:106-107: the regulariser over the whole tables' .data has no gradient (2458 objects:
    the multi-workgroup partial sums)."""
    from codenerf.autograd import render_loss_autograd
    g = torch.Generator().manual_seed(2)
    rc = torch.rand(100, 3, generator=g).to(dev).requires_grad_(True)
    t = torch.rand(100, 4, generator=g).to(dev)
    tab_s, tab_t = torch.randn(n_obj, 256, generator=g).to(dev), torch.randn(n_obj, 256, generator=g).to(dev)
    loss, stats = render_loss_autograd(rc, rc, t, tab_s, tab_t, 1, 1e-5)
    loss.backward()
    ref = 2 * torch.nn.functional.mse_loss(rc.detach()[..., :3], t[..., :3]) + 1e-5 * (tab_s.double().norm() +
                                                                                       tab_t.double().norm())
    assert abs(loss.item() - ref.item()) <= 1e-6 * max(1.0, ref.item())
    assert abs(stats[4].item() - tab_s.double().norm().item()) <= 1e-6 * tab_s.double().norm().item()
    close(rc.grad, 2 * 2 * (rc.detach() - t[..., :3]) / 300, 1e-5, "d rgb")


# ---------------------------------------------------------------- SE3 pose error (8(f) row 4)


def test_pose_error_golden(dev):
    """eval.py:161-162 (lieutils.SE3.Log of inverse(gt) @ cam) vs the reference's values."""
    from codenerf import ops
    g = gload("se3_pose_error.npz", dev)
    twist, err = ops.pose_error(g["gt"], g["cam"])
    close(twist, g["twist"], 1e-4, "twist")
    d = (err - g["err"]).abs()
    assert (d <= 2e-5 * g["err"].abs() + 2e-6).all(), d.max().item()


# ---------------------------------------------------------------- SRN data resident in HBM (8(f) row 2)


@pytest.mark.parametrize("stage", ["train", "val"])
def test_srn_resident_batches(dev, tmp_path, stage):
    """Views decoded once into HBM and unpacked per batch on the device equal the reference
    loader's items bit for bit (srn_tiny.npz); the resident store keeps one shape per split, so
    each object parity (RGB / RGBA) is checked through the per-item path."""
    sys.path.insert(0, GOLDEN)
    import srn_tree
    from codenerf.datasets import SRNDataset
    g = np.load(os.path.join(GOLDEN, "srn_tiny.npz"))
    base = srn_tree.write_tree(str(tmp_path))
    ds = SRNDataset(base, stage)
    # group the views by channel count: one resident store per group
    groups = {}
    for i in range(len(ds)):
        groups.setdefault(g[f"{stage}_{i}_color"].shape[-1], []).append(i)
    for ch, views in groups.items():
        sub = SRNDataset(base, stage)
        sub.rgb_all_filenames = [ds.rgb_all_filenames[i] for i in views]
        sub.pose_all_filenames = [ds.pose_all_filenames[i] for i in views]
        sub.load_resident(dev, threads=4)
        assert sub.resident["images"].dtype == torch.uint8 and sub.resident["images"].shape[-1] == ch
        idx = list(range(len(views)))[::-1]
        bt = sub.batch(idx)
        for j, k in enumerate(idx):
            i = views[k]
            for key in ("color", "mask", "pose", "intrinsic"):
                assert np.array_equal(bt[key][j].cpu().numpy(), g[f"{stage}_{i}_{key}"]), (stage, i, key)
            assert int(bt["object_id"][j]) == int(g[f"{stage}_{i}_object_id"])


def test_srn_resident_rejects_mixed_shapes(dev, tmp_path):
    sys.path.insert(0, GOLDEN)
    import srn_tree
    from codenerf.datasets import SRNDataset
    base = srn_tree.write_tree(str(tmp_path))
    with pytest.raises(ValueError, match="one image shape per split"):
        SRNDataset(base, "train", device=dev)


# ---------------------------------------------------------------- the end of validate() (eval.py:182-205)


def test_validate_renders_and_scores(dev):
    """validate(): test-time optimisation, then the whole view from the optimised pose through
    parallel_image_render and its PSNR -- vs the oracle's render of the same pose and codes."""
    from types import SimpleNamespace as NS
    from codenerf import synthetic
    from codenerf.evaluate import validate
    from codenerf.models import ShapeTextureEmbedding
    from codenerf.nerf import PointSampler
    o = O()
    rs, K = small_sampler(dev)
    ps = PointSampler(8, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    models = _eval_models(dev, frozen=False)
    emb = ShapeTextureEmbedding(5, 256, 256)
    with torch.no_grad():
        emb.shape_embedding.weight.mul_(0.3)
        emb.texture_embedding.weight.mul_(0.3)
    models["embedding"] = emb.to(dev)
    cfg = NS(is_distributed=False, gpus=1, nerf=NS(validation=NS(chunksize=100)),
             experiment=NS(val_iterations=4, regularizer_lambda=1e-5),
             optimizer=NS(val_type="AdamW", val_lr=1e-2, angle_lr=5e-2, radius_lr=1e-1))
    gt = o.pose_spherical(torch.tensor([1.5]), torch.tensor([0.1]), torch.tensor([1.3]))[None]
    color = torch.rand(1, 12, 16, 4, generator=torch.Generator().manual_seed(4))
    np.random.seed(1)
    out = validate(cfg, {"color": color.to(dev), "pose": gt.to(dev)}, models, (rs, ps), embedders(dev), dev)
    assert len(out["history"]) == 4 and all(np.isfinite(h["total_loss"]) for h in out["history"])
    zs, zt = [z.cpu() for z in out["codes"]]
    cam = out["cam_pose"].cpu()
    d = o.ray_directions(12, 16, K)
    ro, rd = o.ray_bundle(d, cam)
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    pc = {k: v.detach().cpu() for k, v in models["nerf_coarse"].state_dict().items()}
    pf = {k: v.detach().cpu() for k, v in models["nerf_fine"].state_dict().items()}
    ref = o.render_image(ro, rd, zs.expand(192, -1), zt.expand(192, -1), o.Sampling(8, 8, 0.8, 1.8), o.EmbedCfg(),
                         pc, pf, 100)["rgb_fine"]
    assert (out["rgb"].cpu() - ref).abs().max().item() <= 1e-4
    mse = torch.nn.functional.mse_loss(ref, color.reshape(-1, 4)[..., :3]).item()
    assert abs(out["psnr"] - o.mse2psnr(mse)) <= 1e-3
    assert abs(out["pose_error"] - o.pose_error(gt, cam).item()) <= 1e-5
    assert out["history"][-1]["pose_error"] > 0


# ---------------------------------------------------------------- checkpoint resume on the device


def test_checkpoint_resume_matches_torch(dev, tmp_path):
    """A reference-format checkpoint loaded into the flat AdamW continues exactly like
    torch.optim.AdamW resumed from the same checkpoint (util.py:175-213 + train.py:111-114)."""
    from types import SimpleNamespace as NS
    from codenerf.checkpoint import load_checkpoint
    from codenerf.optim import AdamW
    from test_checkpoint_cpu import _groups, _models, _reference_checkpoint
    path = tmp_path / "checkpoint    1.ckpt"
    _reference_checkpoint(path)
    m_ref, m_new = _models(7), _models(8)
    for m in list(m_ref.values()) + list(m_new.values()):
        m.to(dev)
    opt_ref = torch.optim.AdamW(_groups(m_ref), lr=1e-4, foreach=False)
    opt_new = AdamW(_groups(m_new), lr=1e-4)
    cfg = NS(load_checkpoint=str(path), is_distributed=False)
    assert load_checkpoint(cfg, m_ref, opt_ref) == 7
    assert load_checkpoint(cfg, m_new, opt_new) == 7
    g = torch.Generator().manual_seed(9)
    for _ in range(2):
        grads = [torch.randn(p.shape, generator=g) for p in m_ref["nerf_coarse"].parameters()]
        for mset, opt in ((m_ref, opt_ref), (m_new, opt_new)):
            opt.zero_grad()
            for p, gr in zip(mset["nerf_coarse"].parameters(), grads):
                p.grad = gr.to(dev)
            opt.step()
    for a, b in zip(m_ref["nerf_coarse"].parameters(), m_new["nerf_coarse"].parameters()):
        assert (a.detach() - b.detach()).abs().max().item() <= 1e-7
