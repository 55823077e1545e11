"""Counts-only launch time per input allocation (tool, not product): does the read-only
stream of the counts-only kernel depend on where its input lands, as the 12 R + 5 W stream
does?  Four torch-allocated inputs of 2^28 tuples, counts-only (rss_counts_perm_kernel)
timed on each in two interleaved rounds; prints one JSON line per round."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
counts = torch.zeros(24, dtype=torch.int64, device=dev)
inputs = []
for _ in range(4):
    t = torch.empty(3 * n, dtype=torch.int32, device=dev)
    _native.generate_device(SEED, 0, n, t.data_ptr(), s.cuda_stream)
    inputs.append(t)
torch.cuda.synchronize()


def timed(t, reps=20, warm=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, t.data_ptr(), n, 128, 24, None, None, counts.data_ptr(),
                            _native.FLAG_ACCUMULATE, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return round(x[len(x) // 2], 4)


for r in range(2):
    print(json.dumps({"round": r, "counts_only_median_ms": [timed(t) for t in inputs]}), flush=True)

# after a burst of full-output launches (the bench's order): counts-only at once, after an
# idle pause, and after more counts-only warm launches
import time  # noqa: E402
hashes = torch.empty(n, dtype=torch.int32, device=dev)
queues = torch.empty(n, dtype=torch.uint8, device=dev)


def full_burst(k=200):
    for _ in range(k):
        _native.hash_device(key, inputs[1].data_ptr(), n, 128, 24, hashes.data_ptr(),
                            queues.data_ptr(), counts.data_ptr(),
                            _native.FLAG_ACCUMULATE | _native.FLAG_QUEUE_U8, s.cuda_stream)
    torch.cuda.synchronize()


out = {}
full_burst()
out["after_full_burst"] = timed(inputs[1], warm=30)
full_burst()
time.sleep(0.1)
out["after_full_burst_sleep100ms"] = timed(inputs[1], warm=30)
full_burst()
time.sleep(1.0)
out["after_full_burst_sleep1s"] = timed(inputs[1], warm=30)
full_burst()
out["after_full_burst_warm300"] = timed(inputs[1], warm=300)
print(json.dumps(out), flush=True)
