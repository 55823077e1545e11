"""Fixed launch sequence for rocprofv3 --pmc passes (tool, not product).

Launches, on 2**28 resident tuples (H=128, Q=24): 3 x full outputs with u8 queues
(the bench's step: rss_hash_device_ws, single-pass counts with the balanced tail),
3 x counts-only (single-pass), 3 x full outputs with u32 queues, in that order, so that
dispatches can be attributed by position.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n, H, Q = 1 << 28, 128, 24
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
hashes = torch.empty(n, dtype=torch.int32, device=dev)
queues = torch.empty(n, dtype=torch.int32, device=dev)
counts = torch.zeros(Q, dtype=torch.int64, device=dev)
ws = torch.zeros(_native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)
_native.generate_device(SEED, 0, n, tuples.data_ptr(), s)
torch.cuda.synchronize()
modes = [("full_u8", hashes.data_ptr(), queues.data_ptr(), _native.FLAG_QUEUE_U8, ws.data_ptr()),
         ("counts_only", None, None, 0, ws.data_ptr()),
         ("full_u32", hashes.data_ptr(), queues.data_ptr(), _native.FLAG_ACCUMULATE, None)]
for name, hp, qp, fl, wsp in modes:
    for _ in range(3):
        _native.hash_device(key, tuples.data_ptr(), n, H, Q, hp, qp, counts.data_ptr(), fl, s, wsp)
    torch.cuda.synchronize()
    print("mode", name, flush=True)
