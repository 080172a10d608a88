"""Which gloo collectives take CUDA tensors on this torch build (two ranks on one GPU)?
usage: python tools/debug/gloo_cuda_probe.py   (spawns its two ranks itself)"""
import os
import socket
import subprocess
import sys


def rank_main():
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    res = {}

    def tryit(name, fn):
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {str(e)[:120]}"

    t = torch.arange(4, dtype=torch.int64, device="cuda") + 10 * r
    tryit("all_reduce", lambda: dist.all_reduce(t.clone()))
    tryit("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(torch.empty(4 * w, dtype=torch.int64, device="cuda"), t))
    tryit("all_gather_into_tensor_async",
          lambda: dist.all_gather_into_tensor(torch.empty(4 * w, dtype=torch.int64, device="cuda"), t, async_op=True).wait())
    tryit("all_gather", lambda: dist.all_gather([torch.empty(4, dtype=torch.int64, device="cuda") for _ in range(w)], t))
    tryit("all_to_all_single", lambda: dist.all_to_all_single(torch.empty(4, dtype=torch.int64, device="cuda"), t,
                                                              [2, 2], [2, 2]))
    tryit("all_to_all", lambda: dist.all_to_all([torch.empty(2, dtype=torch.int64, device="cuda") for _ in range(w)],
                                                [t[:2], t[2:]]))
    tryit("all_reduce_max", lambda: dist.all_reduce(t.clone(), op=dist.ReduceOp.MAX))
    print(f"rank {r}: {res}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if os.environ.get("RANK") is not None:
        rank_main()
        sys.exit(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__], env=dict(os.environ, RANK=str(q), WORLD_SIZE="2",
                                                                  MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for q in range(2)]
    sys.exit(max(p.wait(timeout=300) for p in procs))
