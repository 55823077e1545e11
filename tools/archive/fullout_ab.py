"""Full-output many-queues launches on the small tables, walk variants (tool, not product):
2^28 uniform tuples, H = 2^30, hash u32 + queue u32 + counts; the balanced tail (default),
the static walk (RSS_BALANCE=0) and the load prefetch (RSS_PREFETCH=1); medians of 10
launches after 5 warm ones, three alternating rounds, best kept.  Run it once per library
(RSS_TOEPLITZ_LIB) to compare builds on one box.  One JSON line per Q.

usage: python tools/fullout_ab.py [Q ...]"""
raise SystemExit("archived (round 5): this A/B probe set RSS_* environment switches that the "
                 "product library no longer reads, so every variant would time the default "
                 "path; the alternatives are reachable through tests/hooks.py only")

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n, H = 1 << 28, 1 << 30
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), s.cuda_stream)
h = torch.empty(n, dtype=torch.int32, device=dev)
q = torch.empty(n, dtype=torch.int32, device=dev)
VARIANTS = {"tail": {}, "static": {"RSS_BALANCE": "0", "RSS_PREFETCH": "0"},
            "prefetch": {"RSS_PREFETCH": "1"}}


def timed(Q, env, reps=10, warm=5):
    os.environ.update(env)
    try:
        c = torch.zeros(Q, dtype=torch.int64, device=dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for i in range(-warm, reps):
            if i >= 0:
                ev[i][0].record(s)
            _native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(),
                                c.data_ptr(), 0, s.cuda_stream)
            if i >= 0:
                ev[i][1].record(s)
        torch.cuda.synchronize()
        assert int(c.sum()) == n
        x = sorted(a.elapsed_time(b) for a, b in ev)
        return x[len(x) // 2]
    finally:
        for k in env:
            os.environ.pop(k, None)


for Q in [int(x) for x in sys.argv[1:]] or [131072, 161144]:
    rec = {"Q": Q, "tuples": n, "lib": os.path.basename(_native.LIB_PATH)}
    for rnd in range(3):
        for name, env in VARIANTS.items():
            k = name + "_full_ms"
            t = round(timed(Q, env), 4)
            rec[k] = min(t, rec.get(k, t))
    print(json.dumps(rec), flush=True)
