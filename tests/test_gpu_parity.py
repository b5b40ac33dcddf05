"""HIP path vs the reference (golden fixtures) and the CPU oracle, through the C ABI.

Tolerances (north_star: rendered RGB/depth within 1e-4 absolute on fp32; ray /
pixel integer indexing bit-exact):
  * ray directions / bundle / gather, uniform depths, ray points: bit-exact or
    1 ulp-level (1e-6) where the reference's einsum/bmm order differs;
  * positional encoding: 2e-6 (accurate sinf/cosf vs torch CPU, both <= 2 ulp);
  * raw MLP output: 1e-4 absolute (fp32 MFMA, reassociated sums);
  * rendered rgb / depth / acc: 1e-4 absolute.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

TOL_RENDER = 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import codenerf
    codenerf.load_library()
    return torch.device("cuda", 0)


def load(name, device):
    return {k: torch.from_numpy(v).to(device) for k, v in np.load(os.path.join(GOLDEN, name)).items()}


def maxdiff(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    return (a - b).abs().max().item() if a.numel() else 0.0


@pytest.fixture(params=["f32", "f32_v1", "bf16x3", "bf16x3_w16"])
def precision(request):
    """Every field kernel is held to the same tolerances: fp32 on 16x16x4 MFMA (two waves per
    SIMD, the default), fp32 on 32x32x2 MFMA (one wave per SIMD, also the training forward) and
    the opt-in 3xbf16 split on 32x32x16 (one wave per SIMD) and on 16x16x32 (two waves per SIMD)."""
    return request.param


def models(dev, seeds=(0, 1), precision="f32"):
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    out = []
    for s in seeds:
        m = CodeNeRFModel(hidden_size=256, shape_code_size=256, texture_code_size=256, num_encoding_fn_xyz=10,
                          num_encoding_fn_dir=4)
        m.load_state_dict(synthetic.codenerf_params(s))
        m.precision = precision
        out.append(m.to(dev).eval())
    return out


def embedders(dev):
    from codenerf.nerf import PositionalEmbedder
    return PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev)


# ---------------------------------------------------------------- rays


def test_rays_bit_exact(dev):
    from codenerf.nerf import RaySampler
    g = load("rays_small.npz", dev)
    rs = RaySampler(12, 16, g["intrinsics"].cpu(), sample_size=40, device=dev, datatype=torch.float32)
    assert maxdiff(rs.directions, g["directions"]) == 0.0
    ro, rd = rs.get_bundle(g["poses"])
    assert maxdiff(ro, g["ro"]) == 0.0
    assert maxdiff(rd, g["rd"]) <= 1e-6
    np.random.seed(7)
    o, d, sel = rs.sample(g["poses"])
    assert np.array_equal(sel, g["select_inds"].cpu().numpy())       # host RNG: bit-exact indices
    assert maxdiff(o, g["ro_sel"]) == 0.0
    assert maxdiff(d, g["rd_sel"]) <= 1e-6


# ---------------------------------------------------------------- points

TAGS = ["nc8_nf8_lindepth_d", "nc8_nf8_lindepth_p", "nc8_nf8_lindisp_d", "nc8_nf8_lindisp_p",
        "nc32_nf128_lindepth_d", "nc32_nf128_lindepth_p", "nc64_nf64_lindepth_d", "nc64_nf64_lindepth_p"]


@pytest.mark.parametrize("tag", TAGS)
def test_points(dev, tag):
    from codenerf.nerf import PointSampler
    g = load("points_small.npz", dev)
    nc, nf = [int(x[2:]) for x in tag.split("_")[:2]]
    mode, pert = tag.split("_")[2], tag.endswith("_p")
    ps = PointSampler(nc, nf, 0.8, 1.8, spacing_mode=mode, perturb=pert, dtype=torch.float32, device=dev)
    assert maxdiff(ps.z_vals, g[tag + "_zbins"]) == 0.0
    pts, z = ps.sample_uniform(g["ro"], g["rd"], t_rand=g.get(tag + "_t_rand"))
    assert maxdiff(z, g[tag + "_z"]) == 0.0
    assert maxdiff(pts, g[tag + "_pts"]) == 0.0
    pf, zf = ps.sample_pdf(g["ro"], g["rd"], g[tag + "_w"], z, u=g.get(tag + "_u"))
    # inverse-CDF samples amplify 1-ulp differences of u / cdf by 1/pdf in near-empty
    # bins; exact bits are checked against the oracle with identical inputs below
    assert maxdiff(zf, g[tag + "_zf"]) <= 1e-5
    assert bool((zf[:, 1:] >= zf[:, :-1]).all())
    if tag + "_ptsf" in g:
        assert maxdiff(pf, g[tag + "_ptsf"]) <= 2e-6


@pytest.mark.parametrize("nc", [6, 13, 64])
@pytest.mark.parametrize("perturb", [False, True])
def test_sample_uniform_shapes_vs_oracle(dev, nc, perturb):
    """cn_sample_uniform's two forms: nc % 4 == 0 (16-B lanes, 64) and the per-sample kernel (6, 13),
    with and without the perturbed draw, bit-exact vs the oracle on the same inputs; plus an
    unaligned output (offset by one float) that must take the per-sample form and agree."""
    from codenerf import ops
    from codenerf.nerf import PointSampler
    from oracle import codenerf_oracle as O
    g = torch.Generator().manual_seed(nc)
    R = 1000
    ro = torch.randn(R, 3, generator=g)
    rd = torch.randn(R, 3, generator=g)
    ps = PointSampler(nc, 8, 0.8, 1.8, spacing_mode="lindepth", perturb=perturb, dtype=torch.float32, device=dev)
    t_rand = torch.rand(R, nc, generator=g) if perturb else None
    t_dev = None if t_rand is None else t_rand.to(dev)
    pts, z = ops.sample_uniform(ro.to(dev), rd.to(dev), ps.z_vals, ps.lower, ps.upper, t_dev)
    pts_o, z_o = O.sample_uniform(ro, rd, O.Sampling(nc, 8, 0.8, 1.8).bins, t_rand)
    assert torch.equal(z.cpu(), z_o) and torch.equal(pts.cpu(), pts_o)
    zbuf = torch.empty(R * nc + 1, device=dev)
    pbuf = torch.empty(R * nc * 3 + 1, device=dev)
    ro_d, rd_d = ro.to(dev), rd.to(dev)
    ops.check(ops._lib_ready().cn_sample_uniform(ops.ptr(ro_d), ops.ptr(rd_d), R, ops.ptr(ps.z_vals),
                                                 ops.ptr(ps.lower), ops.ptr(ps.upper), nc, ops.ptr(t_dev),
                                                 ops.ptr(zbuf[1:]), ops.ptr(pbuf[1:]), ops.stream_of(zbuf)),
              "cn_sample_uniform")
    torch.cuda.synchronize()
    assert torch.equal(zbuf[1:].view(R, nc).cpu(), z_o) and torch.equal(pbuf[1:].view(R, nc, 3).cpu(), pts_o)


def test_sample_pdf_strided_weights_and_indices(dev):
    """weights[..., 1:-1] view (nerf/__init__.py:87) and searchsorted indices vs the oracle."""
    from oracle import codenerf_oracle as O
    from codenerf import ops
    torch.manual_seed(3)
    n, nc, nf = 777, 64, 64
    ro, rd = torch.randn(n, 3), torch.randn(n, 3)
    w = torch.rand(n, nc) ** 4
    z = O.depth_bins(nc, 0.8, 1.8, "lindepth")["z"].expand(n, nc).contiguous()
    u = torch.rand(n, nf)
    _, zf_ref = O.sample_pdf(ro, rd, w[..., 1:-1], z, nf, u)
    wd = w.to(dev)
    _, zf = ops.sample_pdf(ro.to(dev), rd.to(dev), wd[..., 1:-1], z.to(dev), nf, u.to(dev), want_pts=False)
    assert maxdiff(zf, zf_ref) == 0.0   # same sum order, double cumsum, same searchsorted -> same bits


@pytest.mark.parametrize("n,nc,nf", [(37, 3, 5), (130, 13, 7), (257, 64, 64), (100, 64, 128), (64, 128, 128),
                                     (33, 256, 256)])
def test_sample_pdf_scan_and_sort_bitwise(dev, n, nc, nf):
    """cn_sample_pdf's wave-parallel cdf (a double scan, exact inside its bounds) and bitonic merge sort vs
    the oracle, bit for bit: per-ray weight regimes in one launch -- heavy-tailed, all zero (uniform pdf),
    one spike of 1e9 (pdf entries below 2^-28: the sequential cumsum fallback) and random scale --, depth
    lists with repeated values and draws quantised to 1/8 (ties between coarse and fine depths and among
    the fine ones), n not a multiple of the 4 rays per workgroup."""
    from oracle import codenerf_oracle as O
    from codenerf import ops
    g = torch.Generator().manual_seed(nc * 1000 + nf)
    ro, rd = torch.randn(n, 3, generator=g), torch.randn(n, 3, generator=g)
    w = torch.rand(n, nc, generator=g) ** 4
    kind = torch.arange(n) % 4
    w[kind == 1] = 0.0
    spike = w[kind == 2]
    spike.zero_()
    spike[:, nc // 2] = 1e9
    w[kind == 2] = spike
    w[kind == 3] *= torch.rand(n, 1, generator=g)[kind == 3] * 50.0
    z = O.depth_bins(nc, 0.8, 1.8, "lindepth")["z"].expand(n, nc).contiguous()
    z[::5, 1:] = torch.maximum(z[::5, 1:], z[::5, :-1]).clone()
    z[::5, nc // 2] = z[::5, nc // 2 - 1] if nc > 2 else z[::5, nc // 2]
    u = torch.rand(n, nf, generator=g)
    u[::3] = torch.floor(u[::3] * 8.0) / 8.0
    pf_ref, zf_ref = O.sample_pdf(ro, rd, w[..., 1:-1], z, nf, u)
    pf, zf = ops.sample_pdf(ro.to(dev), rd.to(dev), w.to(dev)[..., 1:-1], z.to(dev), nf, u.to(dev))
    assert torch.equal(zf.cpu(), zf_ref)
    assert torch.equal(pf.cpu(), pf_ref)
    # u = None: the kernel's linspace(0, 1, nf) -- torch's symmetric two-half formula, each op rounded
    # (linspace01); torch's own vectorised CPU linspace may differ by an ulp for nf >= 64, so the
    # oracle gets the kernel's u
    i = torch.arange(nf, dtype=torch.float32)
    step = torch.tensor(1.0) / float(max(nf - 1, 1))
    u_lin = torch.where(i < nf // 2, step * i, 1.0 - step * (nf - 1 - i)) if nf > 1 else torch.zeros(1)
    _, zl_ref = O.sample_pdf(ro, rd, w[..., 1:-1], z, nf, u_lin.expand(n, nf).contiguous())
    _, zl = ops.sample_pdf(ro.to(dev), rd.to(dev), w.to(dev)[..., 1:-1], z.to(dev), nf, None, want_pts=False)
    assert torch.equal(zl.cpu(), zl_ref)


# ---------------------------------------------------------------- encoding


def test_posenc(dev):
    from codenerf.nerf import PositionalEmbedder
    g = load("posenc.npz", dev)
    for L, log, inc in [(10, True, True), (4, True, True), (6, False, True), (3, True, False)]:
        k = f"L{L}_{int(log)}_{int(inc)}"
        e = PositionalEmbedder(L, log, inc, torch.float32, dev)
        assert maxdiff(e.frequency_bands, g[k + "_freqs"]) == 0.0
        assert maxdiff(e.embed(g["x"]), g[k]) <= 2e-6


# ---------------------------------------------------------------- compositing


def test_volume_render(dev):
    from codenerf.nerf import volume_render
    g = load("volrender.npz", dev)
    rgb, disp, acc, w, depth = volume_render(g["raw"], g["z"], g["rd"])
    for a, k, tol in [(rgb, "rgb", 1e-6), (acc, "acc", 1e-6), (w, "weights", 1e-6), (depth, "depth", 2e-6),
                      (disp, "disp", 1e-5)]:
        ref = g[k]
        if k == "disp":
            # disp = 1/(depth/acc) is ill-conditioned on transparent rays: acc is then a
            # few ulps of exp() (torch's SLEEF exp vs the device expf differ there)
            keep = g["acc"] > 1e-6
            a, ref = a[keep], ref[keep]
        fin = torch.isfinite(ref)
        assert bool((torch.isfinite(a) == fin).all()), k
        assert maxdiff(a[fin], ref[fin]) <= tol, k


@pytest.mark.parametrize("s", [1, 7, 64, 65, 128, 129, 192, 256, 300, 512])
def test_volume_render_sizes(dev, s):
    from oracle import codenerf_oracle as O
    from codenerf import ops
    torch.manual_seed(s)
    n = 129
    raw = torch.randn(n, s, 4) * 2
    z = torch.sort(1 + torch.rand(n, s), -1).values
    rd = torch.randn(n, 3)
    ref = O.volume_render(raw, z, rd)
    got = ops.volume_render(raw.to(dev), z.to(dev), rd.to(dev))
    # the per-ray sums (rgb, depth ~2, acc) are S-term fp32 sums in a lane-tree order vs torch's
    # sequential one: the bound grows with S past 256 (S = 512: 1e-5, ~40 ulp of a depth of 2)
    tol = 5e-6 * max(1.0, s / 256)
    for a, b in zip(got, ref):
        fin = torch.isfinite(b)
        assert maxdiff(a.cpu()[fin], b[fin]) <= tol


@pytest.mark.parametrize("n", [4, 1028, 262144])
def test_volume_render_grouped_path(dev, n):
    """S = 64 with n_rays % 4 == 0 takes the grouped launch (two ray groups per wave, the second's loads
    in flight during the first's integration, the grid's last wave past the end); n + 1 rays take the
    per-group kernel.  The first n rays must agree bit for bit (same arithmetic per ray), and with the
    oracle at test_volume_render_sizes' bound (n = 262144: the C2 launch, checked on a ray sample)."""
    from oracle import codenerf_oracle as O
    from codenerf import ops
    g = torch.Generator().manual_seed(n)
    raw = torch.randn(n + 1, 64, 4, generator=g) * 2
    z = torch.sort(1 + torch.rand(n + 1, 64, generator=g), -1).values
    rd = torch.randn(n + 1, 3, generator=g)
    grouped = ops.volume_render(raw[:n].to(dev), z[:n].to(dev), rd[:n].to(dev))
    single = ops.volume_render(raw.to(dev), z.to(dev), rd.to(dev))
    for a, b in zip(grouped, single):
        fa, fb = a.cpu(), b[:n].cpu()
        assert torch.equal(torch.isnan(fa), torch.isnan(fb))
        assert torch.equal(fa[~torch.isnan(fa)], fb[~torch.isnan(fb)])
    pick = torch.randperm(n, generator=g)[:4096] if n > 4096 else torch.arange(n)
    ref = O.volume_render(raw[pick], z[pick], rd[pick])
    for a, b in zip(grouped, ref):
        fin = torch.isfinite(b)
        assert maxdiff(a.cpu()[pick][fin], b[fin]) <= 5e-6


def test_leaf_ops_empty_batch(dev):
    """Zero rays through the leaf ops gives torch's empty outputs -- the oracle's (torch ops) shapes --
    instead of an error (the C ABI refuses n_rays == 0; the Python layer launches nothing)."""
    from oracle import codenerf_oracle as O
    from codenerf import ops
    from codenerf.nerf import PointSampler
    e3, e64 = torch.empty(0, 3), torch.empty(0, 64)
    ref = O.volume_render(torch.empty(0, 64, 4), e64, e3)
    got = ops.volume_render(torch.empty(0, 64, 4, device=dev), e64.to(dev), e3.to(dev))
    assert [tuple(t.shape) for t in got] == [tuple(t.shape) for t in ref]
    ps = PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    pts, z = ops.sample_uniform(e3.to(dev), e3.to(dev), ps.z_vals, ps.lower, ps.upper)
    pts_o, z_o = O.sample_uniform(e3, e3, O.Sampling(64, 64, 0.8, 1.8).bins)
    assert pts.shape == pts_o.shape and z.shape == z_o.shape
    pf, zf = ops.sample_pdf(e3.to(dev), e3.to(dev), torch.empty(0, 62, device=dev), e64.to(dev), 64,
                            u=ps.u_lin)
    assert pf.shape == (0, 128, 3) and zf.shape == (0, 128)
    enc = ops.posenc(e3.to(dev), [2.0 ** k for k in range(10)], True)
    assert enc.shape == O.posenc(e3, O.frequency_bands(10, True), True).shape
    assert ops.ray_points(e3.to(dev), e3.to(dev), e64.to(dev)).shape == (0, 64, 3)


@pytest.mark.parametrize("precision", ["f32", "bf16x3"])
def test_zero_ray_batch_backward(dev, precision):
    """A zero-ray batch through the differentiable path -- volume_render and the fused field forward /
    backward of both precisions, training (weights with gradients) and eval (frozen) -- returns empty
    or zero gradients instead of the C ABI's CN_EINVAL."""
    from codenerf.nerf import forward_pass, volume_render
    mdl, = models(dev, (0,), precision)
    mdl.train_precision = precision
    for frozen in (False, True):
        mdl.requires_grad_(not frozen)
        rd = torch.empty(0, 3, device=dev, requires_grad=True)
        pts = torch.empty(0, 64, 3, device=dev, requires_grad=True)
        zs = torch.randn(1, 256, device=dev).expand(0, -1).requires_grad_(True)
        zt = torch.randn(1, 256, device=dev).expand(0, -1).requires_grad_(True)
        raw = forward_pass(mdl, embedders(dev), rd, pts, (zs, zt))
        assert raw.shape == (0, 64, 4)
        z = torch.empty(0, 64, device=dev)
        rgb, disp, acc, w, depth = volume_render(raw, z, rd)
        (rgb.sum() + disp.sum() + acc.sum() + depth.sum()).backward()
        assert pts.grad is None or pts.grad.shape == (0, 64, 3)
        if not frozen:
            assert all(p.grad is None or not p.grad.any() for p in mdl.parameters())
            mdl.zero_grad()
    mdl.requires_grad_(True)


def test_volume_render_unaligned_inputs(dev):
    """raw / z as contiguous views at an odd element offset: the C ABI refuses them (CN_EINVAL, no
    launch: its 16-B vector accesses need aligned rows), the Python op realigns them and returns the
    aligned inputs' results bit for bit."""
    from codenerf import ops
    n, s = 256, 64
    g = torch.Generator().manual_seed(3)
    raw = (torch.randn(n, s, 4, generator=g) * 2).to(dev)
    z = torch.sort(1 + torch.rand(n, s, generator=g), -1).values.to(dev)
    rd = torch.randn(n, 3, generator=g).to(dev)
    rbuf = torch.empty(n * s * 4 + 1, device=dev)
    zbuf = torch.empty(n * s + 1, device=dev)
    raw_u, z_u = rbuf[1:].view(n, s, 4), zbuf[1:].view(n, s)
    raw_u.copy_(raw)
    z_u.copy_(z)
    assert raw_u.data_ptr() % 16 == 4 and z_u.is_contiguous()
    outs = [torch.empty(n, 3, device=dev)] + [torch.empty(n, device=dev) for _ in range(3)]
    rc = ops._lib_ready().cn_volume_render(ops.ptr(raw_u), ops.ptr(z_u), ops.ptr(rd), n, s, ops.ptr(outs[0]),
                                           ops.ptr(outs[1]), ops.ptr(outs[2]), None, ops.ptr(outs[3]),
                                           ops.stream_of(rd))
    assert rc != 0, "an unaligned raw row must be refused"
    for a, b in zip(ops.volume_render(raw_u, z_u, rd), ops.volume_render(raw, z, rd)):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0))


# ---------------------------------------------------------------- MLP


def test_mlp_forward_golden(dev, precision):
    g = load("mlp.npz", dev)
    m, = models(dev, (0,), precision)
    with torch.no_grad():
        raw = m(g["z_s"], g["z_t"], g["x"])
    assert maxdiff(raw, g["raw"]) <= 1e-4


@pytest.mark.parametrize("m_rows", [1, 127, 128, 1000])
def test_mlp_forward_rows(dev, precision, m_rows):
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    mdl, = models(dev, (0,), precision)
    torch.manual_seed(m_rows)
    x = torch.randn(m_rows, 90)
    zs, zt = synthetic.latent_codes(1, 1).expand(m_rows, -1), synthetic.latent_codes(2, 1).expand(m_rows, -1)
    ref = O.codenerf_mlp(synthetic.codenerf_params(0), zs, zt, x, 63)
    with torch.no_grad():
        got = mdl(zs.to(dev), zt.to(dev), x.to(dev))
    assert maxdiff(got, ref) <= 1e-4


@pytest.mark.parametrize("r,s", [(50, 8), (37, 64), (300, 3)])
def test_forward_pass_q1(dev, precision, r, s):
    """forward_pass with R not dividing anything: Q1 view-dir tiling (row k -> ray k mod R)."""
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    from codenerf.nerf import forward_pass
    torch.manual_seed(r * s)
    rd = torch.randn(r, 3)
    pts = torch.randn(r, s, 3)
    zs, zt = synthetic.latent_codes(3, r), synthetic.latent_codes(4, r)     # per-ray codes
    ref = O.forward_pass(synthetic.codenerf_params(0), O.EmbedCfg(), rd, pts, zs, zt)
    mdl, = models(dev, (0,), precision)
    with torch.no_grad():
        got = forward_pass(mdl, embedders(dev), rd.to(dev), pts.to(dev), (zs.to(dev), zt.to(dev)))
    assert maxdiff(got, ref) <= 1e-4


# The field kernels' encodings take the lazy fast_sincosf path only when every lane's largest
# argument |x| * 2^9 stays <= 2^14, i.e. |x| <= 32 at L = 10 (csrc/mlp_f32.hip, bound in
# mlp_common.h); past it the wave evaluates every pair with sincosf up front.  Raw outputs with
# |x| ~ 100 are larger, so the bound is relative to the largest |raw| (as test_trained_mlp's).
LARGE_ARG_RTOL = {"f32": 1e-5, "f32_v1": 1e-5, "bf16x3": 1.5e-5, "bf16x3_w16": 1.5e-5}
# the training forwards' first activation plane: h1 = relu(layer_xyz1(enc)) with the raw point among
# its inputs (|x| ~ 180 here), so 3xbf16's ~2^-17 relative error per product reaches 1.5e-5 of the
# plane's largest value (r04b: 1.52e-5 for bf16x3, 7.8e-7 for fp32)
LARGE_ARG_H1_RTOL = {"f32": 2e-6, "bf16x3": 3e-5}


def _large_arg_case(case, r, s, seed):
    g = torch.Generator().manual_seed(seed)
    rd = torch.randn(r, 3, generator=g)
    pts = torch.randn(r, s, 3, generator=g)
    if case == "far":
        pts = pts * 40.0                               # (almost) every lane past the 2^14 argument bound
    else:
        pts[37, 5] = torch.tensor([45.0, -38.0, 41.0])  # ONE sample of one wave far out: a mixed tile
    return rd, pts


@pytest.mark.parametrize("case", ["far", "mixed"])
def test_field_large_arguments_inference(dev, precision, case):
    """The inference field kernels past the fast-sincos argument bound, vs the oracle."""
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    from codenerf.nerf import forward_pass
    from conftest import margin
    r, s = 300, 64
    rd, pts = _large_arg_case(case, r, s, 11)
    zs, zt = synthetic.latent_codes(3, r), synthetic.latent_codes(4, r)
    ref = O.forward_pass(synthetic.codenerf_params(0), O.EmbedCfg(), rd, pts, zs, zt)
    mdl, = models(dev, (0,), precision)
    with torch.no_grad():
        got = forward_pass(mdl, embedders(dev), rd.to(dev), pts.to(dev), (zs.to(dev), zt.to(dev)))
    scale = ref.abs().max().item()
    margin(f"large_args_inference_{case}[{precision}]", "raw rel", maxdiff(got, ref) / scale, LARGE_ARG_RTOL[precision],
           max_abs_x=float(pts.abs().max()))


@pytest.mark.parametrize("case", ["far", "mixed"])
@pytest.mark.parametrize("train_precision", ["f32", "bf16x3"])
@pytest.mark.parametrize("mode", ["pts", "rayz"])
def test_field_large_arguments_training(dev, train_precision, case, mode):
    """The training forwards (fp32 w16 and 3xbf16: activation planes + ReLU masks) past the
    fast-sincos argument bound: raw and the saved post-activation planes vs the oracle's."""
    from oracle import codenerf_oracle as O
    from codenerf import ops, synthetic
    from conftest import margin
    r, s = 300, 64
    rd, pts = _large_arg_case(case, r, s, 12)
    geo = dict(pts=pts.to(dev))
    if mode == "rayz":       # pts = ro + rd z formed in the kernel: far rays from far origins
        z = torch.sort(0.8 + torch.rand(r, s, generator=torch.Generator().manual_seed(3)), dim=-1).values
        ro = pts[:, 0, :].clone()
        pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
        geo = dict(ro=ro.to(dev), z=z.to(dev))
    params_d = synthetic.codenerf_params(0)
    mdl, = models(dev, (0,), "f32")
    params = [p.detach() for p in mdl.param_list()]
    zs, zt = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    cb = ops.code_bias(params, zs.to(dev), zt.to(dev))
    fx, fd = [2.0 ** k for k in range(10)], [2.0 ** k for k in range(4)]
    x3 = train_precision == "bf16x3"
    raw, saved, _ = ops.radiance_field_train_w16(ops.mlp_pack(params, "bf16x3" if x3 else "f32_w16"), cb,
                                                 rd.to(dev), s, r, fx, fd, precision=train_precision, **geo)
    pre = {}
    ref = O.forward_pass(params_d, O.EmbedCfg(), rd, pts, zs.expand(r, -1), zt.expand(r, -1), pre_out=pre)
    tag = f"large_args_training_{case}_{mode}[{train_precision}]"
    rt = LARGE_ARG_RTOL[train_precision]
    margin(tag, "raw rel", maxdiff(raw, ref) / ref.abs().max().item(), rt, max_abs_x=float(pts.abs().max()))
    # the first saved plane is h1 = relu(layer_xyz1(enc)): the encodings' own consumer
    h1 = torch.relu(pre["h1"]) if "h1" in pre else None
    if h1 is not None:
        margin(tag, "h1 plane rel", maxdiff(saved[0], h1) / h1.abs().max().item(), LARGE_ARG_H1_RTOL[train_precision])


# ---------------------------------------------------------------- rendering


def _image_rays(dev, g, h, w):
    from codenerf.nerf import RaySampler
    rs = RaySampler(h, w, g["intrinsics"].cpu(), sample_size=min(4096, h * w), device=dev, datatype=torch.float32)
    ro, rd = rs.get_bundle(g["pose"])
    return rs, ro.reshape(-1, 3), rd.reshape(-1, 3)


@pytest.mark.parametrize("nc,nf", [(8, 8), (32, 128)])
@pytest.mark.parametrize("n_ranks", [1, 2, 3])
def test_render_small_golden(dev, precision, nc, nf, n_ranks):
    """parallel_image_render of the reference, rank slices rendered one by one (chunk 50, Q1 + Q5)."""
    from codenerf.nerf import PointSampler, render_rays
    from codenerf.utils import split_sizes
    g = load("render_small.npz", dev)
    _, ro, rd = _image_rays(dev, g, 12, 16)
    ps = PointSampler(nc, nf, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    mc, mf = models(dev, precision=precision)
    n = ro.shape[0]
    per, _ = split_sizes(n, n_ranks)
    outs, start = [], 0
    with torch.no_grad():
        for r in range(n_ranks):
            sl = slice(start, start + per[r])
            start += per[r]
            o = render_rays(ro[sl], rd[sl], g["z_s"].expand(n, -1)[sl], g["z_t"].expand(n, -1)[sl], ps, embedders(dev),
                            mc, mf, chunk_rows=50)
            outs.append(o["rgb_fine"])
    assert maxdiff(torch.cat(outs), g[f"nc{nc}_n{n_ranks}_rgb"]) <= TOL_RENDER


def test_render_small_perturbed_golden(dev, precision):
    from codenerf.nerf import PointSampler, render_rays
    g = load("render_small.npz", dev)
    _, ro, rd = _image_rays(dev, g, 12, 16)
    ps = PointSampler(8, 8, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    mc, mf = models(dev, precision=precision)
    n = ro.shape[0]
    with torch.no_grad():
        o = render_rays(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), ps, embedders(dev), mc, mf,
                        chunk_rows=50, t_rand=g["p_t_rand"], u=g["p_u"])
    assert maxdiff(o["rgb_coarse"], g["p_rgb_coarse"]) <= TOL_RENDER
    assert maxdiff(o["rgb_fine"], g["p_rgb_fine"]) <= TOL_RENDER


def test_render_full_golden(dev, precision):
    """C2 (128x128, 64 coarse) and C3 (64+64) at full size against the reference."""
    from codenerf.nerf import PointSampler, render_rays
    g = load("render_full.npz", dev)
    _, ro, rd = _image_rays(dev, g, 128, 128)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    mc, mf = models(dev, precision=precision)
    n = ro.shape[0]
    with torch.no_grad():
        o = render_rays(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), ps, embedders(dev), mc, mf,
                        chunk_rows=4096)
    d = {k: maxdiff(o[a], g[k]) for a, k in [("rgb_coarse", "rgb_c"), ("depth_coarse", "depth_c"),
                                             ("acc_coarse", "acc_c"), ("rgb_fine", "rgb_f"),
                                             ("depth_fine", "depth_f"), ("acc_fine", "acc_f")]}
    from conftest import margin
    for k, v in d.items():
        margin(f"render_full_c2c3[{precision}]", k, v, TOL_RENDER)
    # size-independent properties at full size
    assert bool((o["acc_fine"] <= 1.0 + 1e-6).all())
    assert bool((o["z_fine"][:, 1:] >= o["z_fine"][:, :-1]).all())
    with torch.no_grad():
        o2 = render_rays(ro, rd, g["z_s"].expand(n, -1), g["z_t"].expand(n, -1), ps, embedders(dev), mc, mf,
                         chunk_rows=4096)
    assert torch.equal(o["rgb_fine"], o2["rgb_fine"])       # deterministic


def test_chunking_is_semantics_not_tiling(dev, precision):
    """Q1: chunk_rows changes results exactly as the reference's chunking does (vs oracle)."""
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    from codenerf.nerf import PointSampler, render_rays
    g = load("render_small.npz", dev)
    _, ro, rd = _image_rays(dev, g, 12, 16)
    n = ro.shape[0]
    zs, zt = g["z_s"].expand(n, -1), g["z_t"].expand(n, -1)
    ps = PointSampler(8, 8, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    mc, mf = models(dev, precision=precision)
    for chunk in (64, 100, 192):
        with torch.no_grad():
            o = render_rays(ro, rd, zs, zt, ps, embedders(dev), mc, mf, chunk_rows=chunk)
            ref = O.render_image(ro.cpu(), rd.cpu(), zs.cpu(), zt.cpu(), O.Sampling(8, 8, 0.8, 1.8), O.EmbedCfg(),
                                 synthetic.codenerf_params(0), synthetic.codenerf_params(1), chunk)
        assert maxdiff(o["rgb_fine"], ref["rgb_fine"]) <= TOL_RENDER


def test_errors_are_loud(dev):
    from codenerf import ops
    from codenerf._lib import CodeNerfError
    with pytest.raises(ValueError):
        ops.posenc(torch.zeros(4, 3), [1.0], True)              # CPU tensor: no fallback
    with pytest.raises(AssertionError):
        ops.volume_render(torch.zeros(4, 5, 4, device=dev), torch.zeros(4, 6, device=dev), torch.zeros(4, 3, device=dev))
    with pytest.raises(CodeNerfError):
        ops.sample_pdf(torch.zeros(2, 3, device=dev), torch.zeros(2, 3, device=dev), torch.zeros(2, 300, device=dev),
                       torch.zeros(2, 302, device=dev), 8)       # nc > 256 rejected by the C ABI
