"""Probe: can two RCCL ranks share one GPU (for rehearsing the nccl p2p path)?"""
import os
import torch
import torch.distributed as dist
rank = int(os.environ["RANK"])
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.arange(8, dtype=torch.int64, device="cuda") + 100 * rank
out = torch.empty_like(t)
dist.all_to_all_single(out, t)
torch.cuda.synchronize()
print(rank, "a2a", out.tolist(), flush=True)
peer = 1 - rank
r = torch.empty(4, dtype=torch.int64, device="cuda")
ops = [dist.P2POp(dist.isend, t[:4].contiguous(), peer), dist.P2POp(dist.irecv, r, peer)]
for w in dist.batch_isend_irecv(ops):
    w.wait()
torch.cuda.synchronize()
print(rank, "p2p", r.tolist(), flush=True)
dist.destroy_process_group()
