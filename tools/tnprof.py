"""Where the whole-tile dW GEMM's waves spend their clocks (library built with -DCN_PROBE_TN_WAITPROF,
optionally with TN_NODMA): per stage, the clocks at the counted-vmcnt barrier and in the DMA issue,
against the whole loop.   CODENERF_LIB=.../lib_TN_WAITPROF.so python tools/tnprof.py [--m 393216]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-nerf_amd"))
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=393216)
    args = ap.parse_args()
    from codenerf import ops
    fn = ops._lib_ready().cn_debug_tnprof
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(args.m, 256, generator=g).to(dev)
    b = torch.relu(torch.randn(args.m, 256, generator=g)).to(dev)
    c = torch.zeros(256, 256, device=dev)
    for _ in range(4):
        ops.gemm_tn(a, b, c, deterministic=True)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 8, 4), dtype=np.int64)
    assert fn(buf.ctypes.data, 1024) == 0
    nb = int((buf[:, 0, 3] > 0).sum())
    p = buf[:nb].astype(np.float64)
    st = p[:, :, 3]
    out = {"tag": os.path.basename(os.environ.get("CODENERF_LIB", "default")), "blocks": nb,
           "stages": float(st.mean()),
           "barrier_clk_per_stage": float((p[:, :, 0] / st).mean()),
           "dma_clk_per_stage": float((p[:, :, 1] / st).mean()),
           "loop_clk_per_stage": float((p[:, :, 2] / st).mean()),
           "barrier_frac": float((p[:, :, 0] / p[:, :, 2]).mean()),
           "barrier_frac_by_wave": [float((p[:, w, 0] / p[:, w, 2]).mean()) for w in range(8)]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
