"""C5 eval iteration, eager vs HIP graph (bench.eval_bench), for a rocprofv3 kernel / HIP-API timeline:
    rocprofv3 --kernel-trace --hip-runtime-trace -d <dir> -o run --output-format csv -- python tools/c5_timeline.py
Prints one JSON line per mode; tools/trace_gaps.py then splits the trace into the two timed windows
(marked by the roctx-free gap between them: the modes run 1 s apart)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))


def main():
    import torch
    import bench
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PositionalEmbedder, RaySampler
    import codenerf
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    codenerf.load_library()
    k = synthetic.srn_intrinsics(bench.H, bench.FOCAL)
    rs = RaySampler(bench.H, bench.W, k, sample_size=2048, device=dev, datatype=torch.float32)
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    models = []
    for seed in (0, 1):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        models.append(m.to(dev).eval())
    iters = int(os.environ.get("C5_ITERS", "40"))
    for prec in os.environ.get("C5_PRECISIONS", "f32 bf16x3").split():
        for graph in [g == "1" for g in os.environ.get("C5_GRAPH", "0 1").split()]:
            r = bench.eval_bench(dev, rs, emb, models, iters, prec, graph=graph)
            print(json.dumps({"precision": prec, "graph": graph, "ms_per_iter": r["ms_per_iter"],
                              "t_end": time.perf_counter()}), flush=True)
            time.sleep(1.0)


if __name__ == "__main__":
    main()
