"""A/B timing of two builds of the library on one box (tool, not product): the bench's
launch (2^28 resident tuples, u32 hash + u8 queue + counts, H=128, Q=24) and the
counts-only launch, 40 timed launches after 20 warm ones, in a process whose library is
chosen by RSS_TOEPLITZ_LIB.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
hashes = torch.empty(n, dtype=torch.int32, device=dev)
queues = torch.empty(n, dtype=torch.uint8, device=dev)
counts = torch.zeros(24, dtype=torch.int64, device=dev)
_native.generate_device(SEED, 0, n, tuples.data_ptr(), s.cuda_stream)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
out = {"lib": os.path.basename(_native.LIB_PATH)}
for mode, hp, qp, fl in (("full_u8", hashes.data_ptr(), queues.data_ptr(), _native.FLAG_QUEUE_U8),
                         ("counts_only", None, None, 0)):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(40)]
    for i in range(-20, 40):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tuples.data_ptr(), n, 128, 24, hp, qp, counts.data_ptr(),
                            fl | _native.FLAG_ACCUMULATE, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    out[mode] = {"median_ms": t[20], "mean_ms": sum(t) / 40, "min_ms": t[0]}
print(json.dumps(out))
