"""Counts-only launch time on the bench's placed input vs fresh inputs (tool, not product):
a ResidentBatch placed as bench.py places it (2 x 12 candidates, full-output probe), then
counts-only timed on its input and on two freshly allocated copies, interleaved."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402
from rss_simulator_nvidia_amd.resident import ResidentBatch  # noqa: E402

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
batch = ResidentBatch(n, key, 128, 24, device=dev, placement=(2, 12),
                      fill=lambda t: _native.generate_device(SEED, 0, n, t.data_ptr(), s.cuda_stream))
counts = torch.zeros(24, dtype=torch.int64, device=dev)
fresh = []
for _ in range(2):
    t = torch.empty(3 * n, dtype=torch.int32, device=dev)
    t.copy_(batch.tuples)
    fresh.append(t)
torch.cuda.synchronize()


def timed(t, flags=0, hq=(None, None), reps=20, warm=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, t.data_ptr(), n, 128, 24, hq[0], hq[1], counts.data_ptr(),
                            flags | _native.FLAG_ACCUMULATE, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return round(x[len(x) // 2], 4)


full = (batch.hashes.data_ptr(), batch.queues.data_ptr())
for r in range(3):
    print(json.dumps({
        "round": r, "placed_counts": timed(batch.tuples), "fresh0_counts": timed(fresh[0]),
        "fresh1_counts": timed(fresh[1]),
        "placed_full": timed(batch.tuples, _native.FLAG_QUEUE_U8, full),
        "fresh0_full_on_placed_outputs": timed(fresh[0], _native.FLAG_QUEUE_U8, full)}), flush=True)
print(json.dumps({"placement": batch.report["chosen"], "chosen_ms": batch.report["chosen_ms"]}))
