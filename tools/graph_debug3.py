"""GraphedEvalStep (optimiser outside) with the pose / codes moved in place between replays vs the
eager step at the same values: which gradients go stale (debug tool)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main(which):
    import codenerf
    from codenerf import synthetic
    from codenerf.evaluate import GraphedEvalStep, eval_step_loss
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler
    from codenerf.optim import AdamW
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    g = {k: torch.from_numpy(v).to(dev) for k, v in np.load(os.path.join(ROOT, "tests/golden/eval_c5.npz")).items()}
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    ms = {}
    for k, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        m = m.to(dev).train()
        m.requires_grad_(False)
        ms[k] = m
    rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
    ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    names = ("theta", "phi", "rho", "z_s", "z_t")
    init = [torch.tensor([1.57], device=dev), torch.tensor([0.0], device=dev), torch.tensor([1.3], device=dev),
            synthetic.latent_codes(5, 1).to(dev), synthetic.latent_codes(6, 1).to(dev)]
    lv = [t.clone().requires_grad_(True) for t in init]
    th, ph, rh, zs, zt = lv
    opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(23)
    gs = GraphedEvalStep(th, ph, rh, zs, zt, g["target"], (rs, ps), emb, ms, opt, 1e-5, optimizer_in_graph=False)
    for it in range(3):
        with torch.no_grad():  # move the values in place (the optimiser would)
            if it > 0:
                for t in lv[:3] if which == "pose" else lv[3:]:
                    t.add_(0.01)
        state = np.random.get_state()
        loss, _ = gs.step()
        torch.cuda.synchronize()
        gg = [t.grad.clone() for t in lv]
        np.random.set_state(state)
        ref = [t.detach().clone().requires_grad_(True) for t in lv]
        le, _ = eval_step_loss(*ref, g["target"], (rs, ps), emb, ms, 1e-5)
        le.backward()
        print(which, it, "loss", loss.item(), le.item(),
              {n: "%.2e" % ((a - r.grad).abs().max().item() / r.grad.abs().max().item()) for n, a, r in zip(names, gg, ref)})


if __name__ == "__main__":
    main(sys.argv[1])
