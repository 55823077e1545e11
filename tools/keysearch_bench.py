"""Key-search throughput (tool, not product): K random keys x n resident flows, one launch.
Prints key-tuple evaluations per second.
usage: python tools/keysearch_bench.py [K] [n] [uniform|flow] [H] [Q]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rss_simulator_nvidia_amd import _native, keysearch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
dist = sys.argv[3] if len(sys.argv) > 3 else "uniform"
H = int(sys.argv[4]) if len(sys.argv) > 4 else 128
Q = int(sys.argv[5]) if len(sys.argv) > 5 else 24
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
keys = keysearch.random_keys(K, seed=0)
win = np.stack([np.ctypeslib.as_array(_native.prepare_key(k).window) for k in keys])
windows = torch.from_numpy(win.astype(np.uint32).view(np.int32)).to(dev)
tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
counts = torch.empty((K, Q), dtype=torch.int64, device=dev)
if dist == "flow":
    import bench  # noqa: E402
    bench.flow_device(torch, tuples, 0, n, dev)
else:
    _native.generate_device(1, 0, n, tuples.data_ptr(), s)
run = lambda: _native.key_search_device(windows.data_ptr(), K, tuples.data_ptr(), n, H, Q,  # noqa
                                        counts.data_ptr(), s)
run()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
a.record()
for _ in range(reps):
    run()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / reps
assert int(counts.sum()) == K * n
print(json.dumps({"distribution": dist, "keys": K, "flows": n, "htable": H, "queues": Q, "ms": ms,
                  "key_tuple_evals_per_s": K * n / (ms / 1e3),
                  "keys_per_s": K / (ms / 1e3)}))
