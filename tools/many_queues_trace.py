"""One many-queues launch shape repeated, for a per-kernel breakdown under
`rocprofv3 --kernel-trace --stats` (tool, not product): 2^28 uniform tuples, H = 2^30,
Q queues, `full` (hash u32 + queue u32 + counts) or `counts` (counts only), `reps` launches
after 3 warm ones.  Prints the launches' median wall time per launch (HIP events).
Trailing ``option=value`` arguments run the launches on the tests' hooks build with those
path options (tests/hooks.py: e.g. ``wide=0``, ``alloc_fail=2``); the product library reads
no environment switches.

usage: python tools/many_queues_trace.py Q full|counts [reps] [option=value ...]"""
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

Q = int(sys.argv[1])
outputs = sys.argv[2] == "full"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
opts = dict(a.split("=", 1) for a in sys.argv[4:])
if opts:
    from hooks import hooks  # noqa: E402
    scope = hooks(**{k: int(v) for k, v in opts.items()})
else:
    scope = contextlib.nullcontext()
n, H = 1 << 28, 1 << 30
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), s.cuda_stream)
h = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
q = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
c = torch.zeros(Q, dtype=torch.int64, device=dev)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
      for _ in range(reps)]
with scope:
    for i in range(-3, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr() if outputs else None,
                            q.data_ptr() if outputs else None, c.data_ptr(), 0, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
assert int(c.sum()) == n
x = sorted(a.elapsed_time(b) for a, b in ev)
print(json.dumps({"Q": Q, "mode": sys.argv[2], "reps": reps, "median_ms": round(x[len(x) // 2], 4),
                  "hooks": opts}),
      flush=True)
