"""Per-step wall time around the hash kernel (tool, not product): 2^28 tuples, H=128, Q=24,
u8 queues, 60 steps after 10 warm ones, for (a) torch zero_ + accumulate launch with HIP
events around each launch (the bench's step), (b) the same without events, (c) a
non-accumulate launch (the library's hipMemsetAsync of the counts) with events, (d) (c)
without events.  Prints one JSON line per round."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), sp)
h = torch.empty(n, dtype=torch.int32, device=dev)
q = torch.empty(n, dtype=torch.uint8, device=dev)
c = torch.zeros(24, dtype=torch.int64, device=dev)


def run(zero_in_torch, events, steps=60, warm=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    flags = _native.FLAG_QUEUE_U8 | (_native.FLAG_ACCUMULATE if zero_in_torch else 0)
    for i in range(-warm, steps):
        if i == 0:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if zero_in_torch:
            c.zero_()
        if events and i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tup.data_ptr(), n, 128, 24, h.data_ptr(), q.data_ptr(),
                            c.data_ptr(), flags, sp)
        if events and i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    k = sum(a.elapsed_time(b) for a, b in ev) / steps if events else None
    return round(wall, 4), (round(k, 4) if k else None)


for r in range(3):
    print(json.dumps({"round": r, "torch_zero_events": run(True, True),
                      "torch_zero_no_events": run(True, False),
                      "lib_memset_events": run(False, True),
                      "lib_memset_no_events": run(False, False)}), flush=True)
