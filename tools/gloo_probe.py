"""Which collectives this torch build's gloo backend accepts on device (HIP) tensors: two spawned
ranks on cuda:0.  Prints one JSON line per collective (ok / the exact error)."""
import json
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tests = {
        "broadcast": lambda: dist.broadcast(torch.ones(8, device=dev) * rank, 0),
        "all_reduce_sum": lambda: dist.all_reduce(torch.ones(8, device=dev)),
        "all_reduce_max_f64": lambda: dist.all_reduce(torch.ones(1, device=dev, dtype=torch.float64),
                                                      op=dist.ReduceOp.MAX),
        "all_reduce_int32": lambda: dist.all_reduce(torch.ones(8, device=dev, dtype=torch.int32)),
        "all_gather": lambda: dist.all_gather([torch.zeros(8, device=dev) for _ in range(2)],
                                              torch.ones(8, device=dev)),
        "all_gather_into_tensor": lambda: dist.all_gather_into_tensor(torch.zeros(16, device=dev),
                                                                      torch.ones(8, device=dev)),
        "all_gather_object": lambda: dist.all_gather_object([None, None], {"r": rank}),
        "barrier": lambda: dist.barrier(),
    }
    for name, fn in tests.items():
        try:
            fn()
            torch.cuda.synchronize()
            res = "ok"
        except Exception as e:  # noqa: BLE001 - the probe records whatever the backend raises
            res = f"{type(e).__name__}: {str(e).splitlines()[0][:300]}"
        if rank == 0:
            print(json.dumps({"collective": name, "result": res}), flush=True)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(worker, args=(port,), nprocs=2, join=True, start_method="spawn")
    sys.exit(0)
