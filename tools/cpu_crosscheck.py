"""SURVEY §8(d) cross-check of the CPU baseline: the reference itself (imported from
/root/reference with tests/golden/make_golden.py's harness-side shims, in THIS container only --
it does not exist on the GPU box) against the oracle restatement bench.py times as
`cpu_baseline`, on the same host threads and the same workloads: C3 = one 4096-ray chunk at
64 + 64 samples (predict_radiance_and_render), C2 = the coarse pass of the same chunk.
Median of 3 each; writes profiles/r02/cpu_crosscheck.json.

    python tools/cpu_crosscheck.py [threads]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import torch  # noqa: E402


def median3(fn):
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[1], ts


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    torch.set_num_threads(threads)
    import make_golden as MG
    from codenerf import synthetic
    from oracle import codenerf_oracle as O
    import bench
    nerf, model_mod, _, ev = MG.import_reference()
    torch.set_num_threads(threads)
    k = synthetic.srn_intrinsics(bench.H, bench.FOCAL)
    pose = ev.pose_spherical(torch.tensor([0.5]), torch.tensor([0.3]), torch.tensor([1.3]))
    d = O.ray_directions(bench.H, bench.W, k)
    ro, rd = O.ray_bundle(d, pose.reshape(1, 4, 4))
    ro, rd = ro.reshape(-1, 3)[:bench.CHUNK].contiguous(), rd.reshape(-1, 3)[:bench.CHUNK].contiguous()
    n = ro.shape[0]
    zs1, zt1 = synthetic.latent_codes(5, 1), synthetic.latent_codes(6, 1)
    zs, zt = zs1.expand(n, -1), zt1.expand(n, -1)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    models = {"nerf_coarse": MG.make_model(model_mod, 0), "nerf_fine": MG.make_model(model_mod, 1)}
    emb = (nerf.PositionalEmbedder(10, True, True, torch.float32, "cpu"),
           nerf.PositionalEmbedder(4, True, True, torch.float32, "cpu"))
    out = {"threads": threads, "host": bench.host_cpu(), "rays": n}
    with torch.no_grad():
        for tag, nf, coarse_only in (("C2_coarse_64", 0, True), ("C3_64_64", bench.NF, False)):
            ps = nerf.PointSampler(bench.NC, max(nf, 1), bench.NEAR, bench.FAR, spacing_mode="lindepth", perturb=False,
                                   dtype=torch.float32, device="cpu")
            if coarse_only:
                def ref_fn():
                    pts, z = ps.sample_uniform(ro, rd)
                    raw = nerf.forward_pass(models["nerf_coarse"], emb, rd, pts, (zs, zt))
                    nerf.volume_render(raw, z, rd)
            else:
                def ref_fn():
                    nerf.predict_radiance_and_render((ro, rd), ps, emb, models["nerf_coarse"], models["nerf_fine"],
                                                     (zs, zt))

            def port_fn():
                O.render_image(ro, rd, zs, zt, O.Sampling(bench.NC, bench.NF, bench.NEAR, bench.FAR), O.EmbedCfg(),
                               pc, pf, bench.CHUNK, coarse_only=coarse_only)
            ref_fn()
            port_fn()
            m_ref, t_ref = median3(ref_fn)
            m_port, t_port = median3(port_fn)
            out[tag] = {"reference_s": m_ref, "port_s": m_port, "ratio_port_over_ref": m_port / m_ref,
                        "reference_rays_per_s": n / m_ref, "port_rays_per_s": n / m_port,
                        "reference_samples_s": t_ref, "port_samples_s": t_port}
            print(tag, json.dumps(out[tag]), flush=True)
    path = os.path.join(ROOT, "profiles", "r02", "cpu_crosscheck.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
