"""PCIe probe (tool, not product): pinned H2D alone, D2H alone, and both at once on two
streams -- the ceiling for rss_hash_host's direct-DMA pipeline.  Prints one JSON line."""
import json
import time

import torch

MB = 1 << 20
size = 512 * MB
dev = torch.device("cuda:0")
h_up = torch.empty(size, dtype=torch.uint8).pin_memory()
h_dn = torch.empty(size, dtype=torch.uint8).pin_memory()
d_up = torch.empty(size, dtype=torch.uint8, device=dev)
d_dn = torch.empty(size, dtype=torch.uint8, device=dev)
s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def up():
    with torch.cuda.stream(s_up):
        d_up.copy_(h_up, non_blocking=True)


def dn():
    with torch.cuda.stream(s_dn):
        h_dn.copy_(d_dn, non_blocking=True)


def both():
    up()
    dn()


t_up, t_dn, t_both = timed(up), timed(dn), timed(both)
print(json.dumps({"bytes_each": size, "h2d_GBs": size / t_up / 1e9, "d2h_GBs": size / t_dn / 1e9,
                  "concurrent_total_GBs": 2 * size / t_both / 1e9,
                  "concurrent_s": t_both, "serial_s": t_up + t_dn}))
