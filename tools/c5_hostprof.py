"""Host-side profile of the C5 eval iteration (cProfile over N iterations after warm-up) and its
wall time per iteration, to see where the Python/launch overhead goes (kernel-development tool)."""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(precision="bf16x3", iters=40):
    import codenerf
    from codenerf import synthetic
    from codenerf.evaluate import eval_step_loss, step_psnr
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler
    from codenerf.optim import AdamW
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", True, torch.float32, dev)
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    mods = {}
    for k, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        m = m.to(dev)
        m.requires_grad_(False)
        m.precision = precision
        mods[k] = m
    target = torch.rand(128 * 128, 4, generator=torch.Generator().manual_seed(3)).to(dev)
    zs = (torch.randn(1, 256) * 0.3).to(dev).requires_grad_(True)
    zt = (torch.randn(1, 256) * 0.3).to(dev).requires_grad_(True)
    th = torch.tensor([1.57], device=dev).requires_grad_(True)
    ph = torch.tensor([0.0], device=dev).requires_grad_(True)
    rh = torch.tensor([1.3], device=dev).requires_grad_(True)
    opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(0)

    def it():
        loss, logs = eval_step_loss(th, ph, rh, zs, zt, target, (rs, ps), emb, mods, 1e-5)
        opt.zero_grad()
        loss.backward()
        opt.step()
        step_psnr(logs)

    for _ in range(3):
        it()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        it()
    torch.cuda.synchronize()
    print(f"{precision}: {(time.perf_counter() - t0) / iters * 1e3:.3f} ms/iter")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(iters):
        it()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["bf16x3"]))
