"""Per-iteration pose: eager loop vs GraphedEvalStep with the AdamW update inside (debug tool)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main():
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
    dumps = {}
    for mode in ("eager", "graph"):
        rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
        ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", False, torch.float32, dev)
        zs = synthetic.latent_codes(5, 1).to(dev).requires_grad_(True)
        zt = synthetic.latent_codes(6, 1).to(dev).requires_grad_(True)
        th = torch.tensor([1.57], device=dev).requires_grad_(True)
        ph = torch.tensor([0.0], device=dev).requires_grad_(True)
        rh = torch.tensor([1.3], device=dev).requires_grad_(True)
        opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
        np.random.seed(23)
        gs = GraphedEvalStep(th, ph, rh, zs, zt, g["target"], (rs, ps), emb, ms, opt, 1e-5) if mode == "graph" else None
        for it in range(5):
            if gs is not None:
                loss, logs = gs.step()
            else:
                loss, logs = eval_step_loss(th, ph, rh, zs, zt, g["target"], (rs, ps), emb, ms, 1e-5)
                opt.zero_grad()
                loss.backward()
                opt.step()
            torch.cuda.synchronize()
            f = opt.flat_buffers()
            dumps[(mode, it)] = {k: f[k][:524].clone() for k in ("param", "grad", "exp_avg", "exp_avg_sq")}
            print(mode, it, "loss %.9f" % loss.item(), "pose", ["%.7f" % float(t) for t in (th, ph, rh)],
                  "grad th %.4e" % float(th.grad), "step", float(opt.state[th]["step"]),
                  "m_th %.4e" % float(opt.state[th]["exp_avg"]))
    for it in range(5):
        e, q = dumps[("eager", it)], dumps[("graph", it)]
        print(it, {k: "%.3e" % (e[k] - q[k]).abs().max().item() for k in e},
              "grad argmax", int((e["grad"] - q["grad"]).abs().argmax()))





if __name__ == "__main__":
    main()
