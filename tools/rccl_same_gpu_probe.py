"""Probe (tool, not product): can two ranks share one GPU through RCCL on this box?  Under
``torchrun --nproc-per-node 2``, both ranks on cuda:0: a torch.distributed (nccl = RCCL)
all-reduce, then rccl.RcclComm's own communicator and ncclAllReduce of a uint64 count vector.
Prints one JSON line per rank with what worked.  RCCL may refuse a duplicate GPU; that is a
result too."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
out = {"rank": rank, "world": world}
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((24,), rank + 1, dtype=torch.int64, device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    out["torch_nccl_allreduce"] = int(t[0].item()) == world * (world + 1) // 2
except Exception as err:  # the result is what failed
    out["torch_nccl_error"] = repr(err)[:300]
if dist.is_initialized():
    try:
        from rss_simulator_nvidia_amd.rccl import RcclComm
        t0 = time.perf_counter()
        comm = RcclComm("cuda:0", timeout_s=60)
        out["rcclcomm_init_s"] = round(time.perf_counter() - t0, 2)
        c = torch.full((24,), 1 << 40 | (rank + 1), dtype=torch.int64, device="cuda:0")
        comm.all_reduce_counts(c)
        torch.cuda.synchronize()
        want = world * (1 << 40) + world * (world + 1) // 2
        out["rcclcomm_allreduce"] = int(c[0].item()) == want
        comm.destroy()
    except Exception as err:
        out["rcclcomm_error"] = repr(err)[:300]
    dist.destroy_process_group()
print(json.dumps(out), flush=True)
