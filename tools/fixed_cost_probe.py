"""Fixed-cost probe (tool, not product): rss_toeplitz_kernel time vs n at the bench's
outputs (u32 hash + u8 queue + counts), from one lane-iteration (2^20 tuples on 256 CUs)
to the bench size, so the per-launch constant (launch, LUT build, epilogue) separates
from the per-tuple stream time.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from rss_simulator_nvidia_amd import _native

dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
N = 1 << 28
tuples = torch.empty(3 * N, dtype=torch.int32, device=dev)
hashes = torch.empty(N, dtype=torch.int32, device=dev)
queues = torch.empty(N, dtype=torch.uint8, device=dev)
counts = torch.zeros(24, dtype=torch.int64, device=dev)
_native.generate_device(0x5EED, 0, N, tuples.data_ptr(), s.cuda_stream)
key = _native.prepare_key([int(x, 16) for x in open("tests/golden/example_input/hash_key.txt").read().split(":")])
flags = _native.FLAG_QUEUE_U8 | _native.FLAG_ACCUMULATE
out = {}
for n in (1 << 20, 1 << 22, 1 << 24, 1 << 26, 1 << 28):
    def run():
        _native.hash_device(key, tuples.data_ptr(), n, 128, 24, hashes.data_ptr(), queues.data_ptr(),
                            counts.data_ptr(), flags, s.cuda_stream)
    for _ in range(3):
        run()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record(s)
        run()
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    out[str(n)] = {"median_us": 1e3 * t[len(t) // 2], "min_us": 1e3 * t[0]}

# the bench's step shape at the full size: zero the counts, then the hash launch, with the
# events around the hash launch only; and the same with counts zeroed on a side stream
n = N
side = torch.cuda.Stream(dev)
cb = [counts, torch.zeros(24, dtype=torch.int64, device=dev)]
for shape in ("zero_then_hash", "back_to_back", "zero_then_hash"):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record(s)
    for i, (a, b) in enumerate(ev):
        c = cb[i & 1]
        if shape == "zero_then_hash":
            c.zero_()
        a.record(s)
        _native.hash_device(key, tuples.data_ptr(), n, 128, 24, hashes.data_ptr(), queues.data_ptr(),
                            c.data_ptr(), flags, s.cuda_stream)
        b.record(s)
    t1.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    out["full_" + shape + "_%d" % len(out)] = {"median_us": 1e3 * t[len(t) // 2], "min_us": 1e3 * t[0],
                                  "mean_us": 1e3 * sum(t) / len(t), "wall_per_step_us": 1e3 * t0.elapsed_time(t1) / 20}
print(json.dumps(out))
