"""Mode-switch probe (tool, not product): per-launch times of the counts-only kernel
(12 B/tuple) right after a run of full-output launches, and vice versa, at 2^28 tuples.
Prints one JSON line of per-launch microseconds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rss_simulator_nvidia_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
N = 1 << 28
tuples = torch.empty(3 * N, dtype=torch.int32, device=dev)
hashes = torch.empty(N, dtype=torch.int32, device=dev)
queues = torch.empty(N, dtype=torch.uint8, device=dev)
counts = torch.zeros(24, dtype=torch.int64, device=dev)
_native.generate_device(0x5EED, 0, N, tuples.data_ptr(), s.cuda_stream)
key = _native.prepare_key([int(x, 16) for x in open(os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
    "tests/golden/example_input/hash_key.txt")).read().split(":")])
acc = _native.FLAG_ACCUMULATE


def series(mode, k):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for a, b in ev:
        a.record(s)
        if mode == "full":
            _native.hash_device(key, tuples.data_ptr(), N, 128, 24, hashes.data_ptr(),
                                queues.data_ptr(), counts.data_ptr(), acc | _native.FLAG_QUEUE_U8,
                                s.cuda_stream)
        else:
            _native.hash_device(key, tuples.data_ptr(), N, 128, 24, None, None, counts.data_ptr(),
                                acc, s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    return [round(1e3 * a.elapsed_time(b), 1) for a, b in ev]


out = {}
order = [("counts", 30), ("full", 30), ("counts", 30), ("full", 30), ("counts", 30)]
if len(sys.argv) > 1 and sys.argv[1] == "full-first":
    order = [("full", 60), ("counts", 30), ("full", 30)]
for i, (mode, k) in enumerate(order):
    out["%d_%s" % (i, mode)] = series(mode, k)
print(json.dumps(out))
