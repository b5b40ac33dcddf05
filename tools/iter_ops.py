"""Which torch (aten) ops one eval / training iteration runs besides the HIP library's launches, per
iteration: torch.profiler (CPU activity only: the op names and counts, no device tracing) over N
iterations of bench.eval_bench's eager C5 loop (MODE=c5) or bench.train_bench's C3 loop (MODE=c3).
    python tools/iter_ops.py            # prints one JSON line: {op: calls per iteration}"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main():
    import torch
    from torch.profiler import ProfilerActivity, profile
    import bench
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PositionalEmbedder, RaySampler
    import codenerf
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    codenerf.load_library()
    mode = os.environ.get("MODE", "c5")
    iters = int(os.environ.get("ITERS", "10"))
    k = synthetic.srn_intrinsics(bench.H, bench.FOCAL)
    out = {}
    if mode == "c5":
        rs = RaySampler(bench.H, bench.W, k, sample_size=2048, device=dev, datatype=torch.float32)
        emb = (PositionalEmbedder(10, True, True, torch.float32, dev),
               PositionalEmbedder(4, True, True, torch.float32, dev))
        models = []
        for seed in (0, 1):
            m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
            m.load_state_dict(synthetic.codenerf_params(seed))
            models.append(m.to(dev).eval())
        bench.eval_bench(dev, rs, emb, models, 2, "f32")            # warm-up
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            bench.eval_bench(dev, rs, emb, models, iters, "f32")
        per = iters + 2                                                # eval_bench runs 2 untimed iterations
    else:
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            bench.train_bench(dev, k, iters, 1, "f32")
        per = iters + 1
    for ev in prof.key_averages():
        if ev.key.startswith("aten::") or ev.key.startswith("cudaMemcpy") or "Memcpy" in ev.key:
            out[ev.key] = round(ev.count / per, 2)
    print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]))), flush=True)


if __name__ == "__main__":
    main()
