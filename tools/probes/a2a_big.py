"""Debug: RCCL collectives with world 1 over growing buffers (a self-send that loses data)."""
import os, sys
import torch
import torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for n in [1 << 16, 1 << 20, 1 << 22, 1 << 23, 1 << 24, 1 << 25, 1 << 26, 100_000_000]:
    a = torch.arange(n, dtype=torch.float64, device="cuda") + 1
    out = torch.empty_like(a)
    dist.all_to_all_single(out, a, output_split_sizes=[n], input_split_sizes=[n])
    torch.cuda.synchronize()
    bad = (out != a).nonzero()
    first = int(bad[0].item()) if bad.numel() else -1
    g = torch.empty_like(a)
    dist.all_gather_into_tensor(g, a)
    torch.cuda.synchronize()
    b2 = (g != a).sum().item()
    s = torch.empty_like(a)
    torch.cuda.synchronize()
    out3 = torch.empty_like(a)
    dist.all_to_all_single(out3, a, output_split_sizes=[n], input_split_sizes=[n])
    dist.barrier()
    torch.cuda.synchronize()
    print(f"n={n} bytes={n*8} a2a_mismatch={bad.numel()} first_bad={first} allgather_mismatch={b2} "
          f"a2a_after_barrier_mismatch={(out3 != a).sum().item()}", flush=True)
dist.destroy_process_group()
