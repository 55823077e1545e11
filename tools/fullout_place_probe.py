"""Placement spread of the many-queues full-output launch (tool, not product): the same
launch (2^28 uniform tuples, H = 2^30, Q = 131072, hash u32 + queue u32 + counts) timed on
8 successive output allocations (the earlier ones kept alive, so each lands elsewhere) and
2 input copies -- DESIGN.md §3 "Placement": the rate depends on where the streams' allocations
land in HBM.  Medians of 10 launches after 5 warm ones.  One JSON line.

usage: python tools/fullout_place_probe.py [Q]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
n, H = 1 << 28, 1 << 30
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
inputs = []
for _ in range(2):
    t = torch.empty(3 * n, dtype=torch.int32, device=dev)
    _native.generate_device(SEED, 0, n, t.data_ptr(), s.cuda_stream)
    inputs.append(t)
c = torch.zeros(Q, dtype=torch.int64, device=dev)


def timed(tup, h, q, reps=10, warm=5):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(), c.data_ptr(),
                            0, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    assert int(c.sum()) == n
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return round(x[len(x) // 2], 4)


outs, rec = [], {"Q": Q, "tuples": n, "ms": []}
for k in range(8):
    outs.append((torch.empty(n, dtype=torch.int32, device=dev),
                 torch.empty(n, dtype=torch.int32, device=dev)))
    h, q = outs[-1]
    rec["ms"].append([timed(tup, h, q) for tup in inputs])
flat = sorted(x for row in rec["ms"] for x in row)
rec.update(first_ms=rec["ms"][0][0], min_ms=flat[0], median_ms=flat[len(flat) // 2], max_ms=flat[-1])
print(json.dumps(rec), flush=True)
