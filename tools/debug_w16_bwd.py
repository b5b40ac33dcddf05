"""Stage-by-stage check of the fp32 fused backward (csrc/mlp_f32.hip field_w16_bwd_kernel).

Runs the masks forward + fused backward with the debug dump on (cn_debug_set_buffer) and compares
each stage's gradient rows with torch fp32 math on the same ReLU decisions:
  0 d v2, 1 d v1, 2 d feat, 3 d h2, 4 d h1, 5 d enc / d dir (per lane group, kernel order).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402


def main():
    import codenerf
    from codenerf import _lib, ops, synthetic
    from codenerf.models import CodeNeRFModel
    from test_gpu_grad import decode_relu_masks_w16
    lib = codenerf.load_library() if hasattr(codenerf, "load_library") else _lib.load()
    lib = _lib.load()
    lib.cn_debug_set_buffer.argtypes = [ctypes.c_void_p]
    lib.cn_debug_set_buffer.restype = None
    dev = torch.device("cuda", 0)
    m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
    m.load_state_dict(synthetic.codenerf_params(0))
    m = m.to(dev)
    params = [p.detach() for p in m.param_list()]
    r, s = 16, 16
    g = torch.Generator().manual_seed(1)
    ro = (torch.randn(r, 3, generator=g) * 0.3 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = torch.randn(r, 3, generator=g).to(dev)
    z = torch.sort(0.8 + torch.rand(r, s, generator=g), dim=-1).values.to(dev)
    zs, zt = synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)
    gout = torch.randn(r, s, 4, generator=g).to(dev)
    fx = [2.0 ** k for k in range(10)]
    fd = [2.0 ** k for k in range(4)]
    cb = ops.code_bias(params, zs, zt)
    raw, masks = ops.radiance_field_masks(ops.mlp_pack(params, "f32_w16"), cb, rd, s, r, fx, fd, ro=ro, z=z,
                                          precision="f32")
    M = r * s
    dbg = torch.zeros(6, M, 256, device=dev)
    lib.cn_debug_set_buffer(dbg.data_ptr())
    out = ops.field_backward_x3(ops.mlp_pack(params, "f32_w16_t"), masks, gout.contiguous(), r, s, r, 1, fx, fd,
                                rd=rd, ro=ro, z=z, want_ro=True, want_rd=True, precision="f32")
    torch.cuda.synchronize()
    lib.cn_debug_set_buffer(None)
    mk = {k: v.to(dev) for k, v in decode_relu_masks_w16(masks, M).items()}
    P = {n: t.detach() for n, t in m.state_dict().items()}
    d = gout.reshape(M, 4)
    Wr, Wd2, Wd1 = P["fc_rgb.weight"], P["layer_dir2.weight"], P["layer_dir1.weight"]
    Wo, Wx2, Wx1 = P["fc_out.weight"], P["layer_xyz2.weight"], P["layer_xyz1.weight"]
    ref = {}
    ref[0] = d[:, :3] @ Wr[:, :256]
    ref[1] = (ref[0] * mk["v2"]) @ Wd2
    dv1 = ref[1] * mk["v1"]
    ref[2] = dv1 @ Wd1[:, :256]
    ddir = dv1 @ Wd1[:, 256:]
    ref[3] = ref[2] @ Wo[1:, :256] + d[:, 3:4] * Wo[0:1, :256]
    ref[4] = (ref[3] * mk["h2"]) @ Wx2[:, :256]
    denc = (ref[4] * mk["h1"]) @ Wx1
    for k in range(5):
        err = (dbg[k] - ref[k]).abs().max().item()
        print(f"stage {k}: max|d| {err:.3e}  (scale {ref[k].abs().max().item():.3e})")
        if err > 1e-3 * ref[k].abs().max().item():
            bad = (dbg[k] - ref[k]).abs()
            i = torch.argmax(bad).item()
            print(f"   worst at row {i // 256} feature {i % 256}: got {dbg[k].view(-1)[i].item():.5e} "
                  f"ref {ref[k].view(-1)[i].item():.5e}")
            print("   got row0[:8]", dbg[k][0, :8].tolist())
            print("   ref row0[:8]", ref[k][0, :8].tolist())
    # stage 5: genc[16] at 16 g + t (t: enc k-step of lane group g), gdir[8] at 64 + 8 g + s
    from codenerf.nerf import __init__ as _  # noqa: F401
    import importlib
    fcol = importlib.import_module("codenerf").__dict__
    del fcol

    def col_enc_xyz(t, gg):
        i = t & 7
        p = 4 * i + gg
        if p < 30:
            return (3 if t < 8 else 6) + 6 * (p // 3) + p % 3
        return (0 if gg == 2 else 2) if t < 8 else (1 if gg == 2 else -1)

    def col_enc_dir(sx, gg):
        if sx < 6:
            p = 4 * (sx % 3) + gg
            return (3 if sx < 3 else 6) + 6 * (p // 3) + p % 3
        return gg if (sx == 6 and gg < 3) else -1
    e1 = e2 = 0.0
    for gg in range(4):
        for t in range(16):
            c = col_enc_xyz(t, gg)
            if c >= 0:
                e1 = max(e1, (dbg[5][:, 16 * gg + t] - denc[:, c]).abs().max().item())
        for sx in range(8):
            c = col_enc_dir(sx, gg)
            if c >= 0:
                e2 = max(e2, (dbg[5][:, 64 + 8 * gg + sx] - ddir[:, c]).abs().max().item())
    print(f"stage 5: d enc max|d| {e1:.3e} (scale {denc.abs().max().item():.3e}); d dir max|d| {e2:.3e} "
          f"(scale {ddir.abs().max().item():.3e})")
    print("d_ro[0]", out["d_ro"][0].tolist())
    gc = out["g_code"][0]
    dh2m = ref[3] * mk["h2"]
    print("g_code xyz2 vs sum(dh2 * m_h2):", (gc[:256] - dh2m.sum(0)).abs().max().item(),
          " vs sum(dh2):", (gc[:256] - ref[3].sum(0)).abs().max().item(), " scale", dh2m.sum(0).abs().max().item())
    print("g_code feat vs sum(dfeat):", (gc[256:512] - ref[2].sum(0)).abs().max().item())
    print("g_code sigma/rgb:", (gc[512:516] - torch.cat([d[:, 3:4], d[:, :3]], 1).sum(0)).abs().max().item())
    for name in ("h1", "h2", "v1", "v2", None):
        alt = ref[3] * mk[name] if name else ref[3]
        print(f"stage4 with mask {name}: {((dbg[4] - alt @ Wx2[:, :256]).abs().max().item()):.3e}")
    print("stage4 = d feat @ Wx2 (stale act):", (dbg[4] - ref[2] @ Wx2[:, :256]).abs().max().item())
    print("stage4 = dh2 + correct (acc not zeroed):", (dbg[4] - ref[3] - ref[4]).abs().max().item())
    print("stage4 = dh2m @ Wx2 code half:", (dbg[4] - (ref[3] * mk["h2"]) @ Wx2[:, 256:]).abs().max().item())
    # the transposed pack itself, every wide chunk, vs a host reconstruction
    pk = ops.mlp_pack(params, "f32_w16_t").cpu()
    import numpy as np
    col_acc = lambda t, gg: 16 * (t >> 2) + 4 * gg + (t & 3)  # noqa: E731
    Wc = {k: v.cpu() for k, v in P.items()}
    firsts = [(1, "layer_dir2.weight", 0, 256), (9, "layer_dir1.weight", 0, 283), (18, "fc_out.weight", 1, 512),
              (26, "layer_xyz2.weight", 0, 512)]
    for first, name, roff, ld in firsts:
        W = Wc[name].reshape(-1)
        worst = 0.0
        for c in range(first, first + 8):
            blk = pk[c * 8192:(c + 1) * 8192].view(8, 4, 64, 4)
            for st in range(8):
                for q in range(4):
                    lane = torch.arange(64)
                    i, gg = lane & 15, lane >> 4
                    for j in range(4):
                        row = 16 * (4 * q + j) + i
                        kin = 16 * ((8 * (c - first) + st) >> 2) + 4 * gg + ((8 * (c - first) + st) & 3)
                        exp = W[(roff + kin) * ld + row]
                        worst = max(worst, (blk[st, q, :, j] - exp).abs().max().item())
        print(f"pack {name} chunks {first}..{first + 7}: max|d| {worst:.3e}")
    blk = pk[26 * 8192:27 * 8192].view(8, 4, 64, 4)
    for st, q, lane, j in [(0, 0, 0, 0), (0, 0, 1, 0), (0, 0, 16, 0), (0, 1, 0, 0), (1, 0, 0, 0), (0, 0, 0, 1)]:
        val = blk[st, q, lane, j].item()
        hits = []
        for name, t in Wc.items():
            idx = (t.reshape(-1) == val).nonzero().flatten().tolist()
            for ix in idx[:3]:
                hits.append((name, divmod(ix, t.shape[-1]) if t.dim() == 2 else ix))
        print(f"xyz2 chunk26 st{st} q{q} lane{lane} j{j} = {val:.6f} found at {hits}")
    print("stage4 vs out^T-pack-as-W:", (dbg[4] - (ref[3] * mk["h2"]) @ Wo[1:, :256]).abs().max().item())


if __name__ == "__main__":
    main()
