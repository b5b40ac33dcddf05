"""Run only the C5 eval step or the C3 training iteration of bench.py (for rocprofv3 kernel stats).

    python tools/step_prof.py eval f32 20      # 20 eval iterations, fp32 field kernels
    python tools/step_prof.py train f32 3      # 3 training iterations
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    what, prec, iters = sys.argv[1], sys.argv[2], int(sys.argv[3])
    import codenerf
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PositionalEmbedder, RaySampler
    codenerf.load_library()
    dev = torch.device("cuda", 0)
    k = synthetic.srn_intrinsics(bench.H, bench.FOCAL)
    if what == "eval":
        rs = RaySampler(bench.H, bench.W, k, sample_size=2048, device=dev, datatype=torch.float32)
        emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
        models = []
        for seed in (0, 1):
            m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
            m.load_state_dict(synthetic.codenerf_params(seed))
            models.append(m.to(dev).eval())
        print(bench.eval_bench(dev, rs, emb, models, iters, prec))
    else:
        os.environ["CODENERF_PRECISION"] = prec
        os.environ["CODENERF_TRAIN_PRECISION"] = prec
        print(bench.train_bench(dev, k, iters, 1, prec))


if __name__ == "__main__":
    main()
