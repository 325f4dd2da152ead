"""Can two ranks share one GPU over RCCL (backend "nccl")?  Each rank puts a
tensor on cuda:0 and all-gathers it; prints the result or the error.  Run as
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
--master-port P tools/diag/rccl_two_ranks_one_gpu.py"""
import os
import sys
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank + 1), device="cuda")
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_gather ok {[o.tolist() for o in out]}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: {type(e).__name__}: {str(e)[:400]}", flush=True)
    sys.exit(3)
