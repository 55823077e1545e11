"""A few many-queues launches for a rocprofv3 kernel trace (tool, not product): 2^28 tuples,
H = 2^30, Q in {20000, 65536, 131072}, full outputs and counts only, wide then narrow
(RSS_WIDE_HIST=0) -- the per-kernel split of the hash pass, the range passes and the reduce.

    rocprofv3 --kernel-trace --stats -- python tools/many_queues_prof.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), s)
h = torch.empty(n, dtype=torch.int32, device=dev)
q = torch.empty(n, dtype=torch.int32, device=dev)
for wide in ("1", "0"):
    os.environ["RSS_WIDE_HIST"] = wide
    for Q in (20000, 65536, 131072):
        c = torch.zeros(Q, dtype=torch.int64, device=dev)
        fl = _native.FLAG_QUEUE_U16 if Q <= 65536 else 0
        for _ in range(5):
            _native.hash_device(key, tup.data_ptr(), n, 1 << 30, Q, h.data_ptr(), q.data_ptr(),
                                c.data_ptr(), fl, s)
            _native.hash_device(key, tup.data_ptr(), n, 1 << 30, Q, None, None, c.data_ptr(), 0, s)
        torch.cuda.synchronize()
        print("Q", Q, "wide", wide, "sum", int(c.sum()), flush=True)
