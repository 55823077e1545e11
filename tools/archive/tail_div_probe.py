"""Balanced-tail share A/B (tool, not product): the last rows / div of a single-pass or u8
launch's rows handed out per workgroup slot (RSS_TAIL_DIV, default 10) -- the bench's step
shape (H = 128, Q = 24, hash u32 + queue u8, single-pass counts on a zeroed workspace) and
the many-queues full-output launch (H = 2^30, Q = 131072, hash u32 + queue u32); 2^28
uniform tuples, medians of 10 launches after 5 warm ones, three alternating rounds, best kept.

usage: python tools/tail_div_probe.py [div ...]"""
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

n = 1 << 28
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), s.cuda_stream)
h = torch.empty(n, dtype=torch.int32, device=dev)
q32 = torch.empty(n, dtype=torch.int32, device=dev)
q8 = torch.empty(n, dtype=torch.uint8, device=dev)
ws = torch.zeros(_native.counts_workspace_bytes(128, 24) // 8 + 1, dtype=torch.int64, device=dev)


def timed(shape, div, reps=10, warm=5):
    os.environ["RSS_TAIL_DIV"] = str(div)
    try:
        Q = 24 if shape == "step" else 131072
        c = torch.zeros(Q, dtype=torch.int64, device=dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for i in range(-warm, reps):
            if i >= 0:
                ev[i][0].record(s)
            if shape == "step":
                _native.hash_device(key, tup.data_ptr(), n, 128, 24, h.data_ptr(), q8.data_ptr(),
                                    c.data_ptr(), _native.FLAG_QUEUE_U8, s.cuda_stream,
                                    workspace_ptr=ws.data_ptr())
            else:
                _native.hash_device(key, tup.data_ptr(), n, 1 << 30, Q, h.data_ptr(), q32.data_ptr(),
                                    c.data_ptr(), 0, s.cuda_stream)
            if i >= 0:
                ev[i][1].record(s)
        torch.cuda.synchronize()
        assert int(c.sum()) == n
        x = sorted(a.elapsed_time(b) for a, b in ev)
        return x[len(x) // 2]
    finally:
        os.environ.pop("RSS_TAIL_DIV", None)


divs = [int(x) for x in sys.argv[1:]] or [10, 5, 3, 20]
rec = {"tuples": n}
for rnd in range(3):
    for shape in ("step", "q131072_full"):
        for d in divs:
            k = "%s_div%d_ms" % (shape, d)
            t = round(timed(shape, d), 4)
            rec[k] = min(t, rec.get(k, t))
print(json.dumps(rec), flush=True)
