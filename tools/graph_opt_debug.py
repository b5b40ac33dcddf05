"""test_time_optimize: eager vs graph (optimiser outside) vs graph (optimiser inside), per-iteration
pose and codes (debug tool)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main():
    import codenerf
    from codenerf import synthetic
    from codenerf import evaluate as E
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    g = {k: torch.from_numpy(v).to(dev) for k, v in np.load(os.path.join(ROOT, "tests/golden/eval_c5.npz")).items()}
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))

    def models():
        ms = {}
        for k, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
            m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
            m.load_state_dict(synthetic.codenerf_params(seed))
            ms[k] = m.to(dev).train()
        return ms
    res = {}
    for mode in ("eager", "graph_out", "graph_in"):
        rs = RaySampler(128, 128, synthetic.srn_intrinsics(128), sample_size=2048, device=dev, datatype=torch.float32)
        ps = PointSampler(64, 64, 0.8, 1.8, "lindepth", False, torch.float32, dev)
        codes = (synthetic.latent_codes(5, 4).to(dev), synthetic.latent_codes(6, 4).to(dev))
        np.random.seed(23)
        if mode == "graph_out":
            orig = E.GraphedEvalStep.__init__

            def init(self, *a, **k):
                k["optimizer_in_graph"] = False
                orig(self, *a, **k)
            E.GraphedEvalStep.__init__ = init
            # the loop must then run opt.step() itself
        zs, zt, pose, hist, cam = E.test_time_optimize(g["target"], (rs, ps), emb, models(), codes, iterations=5,
                                                       graph=(mode != "eager"))
        if mode == "graph_out":
            E.GraphedEvalStep.__init__ = orig
        res[mode] = (torch.stack([p.detach() for p in pose]).cpu(), zs.detach().cpu(), [h["total_loss"] for h in hist])
        print(mode, "pose", res[mode][0].flatten().tolist(), "loss", res[mode][2])
    for m in ("graph_out", "graph_in"):
        print(m, "vs eager: pose", (res[m][0] - res["eager"][0]).abs().max().item(), "z_s",
              (res[m][1] - res["eager"][1]).abs().max().item())


if __name__ == "__main__":
    main()
