"""Same-buffer A/B/C of the small-table passes' walk: static grid-stride (RSS_BALANCE=0), the
same with a load prefetch (RSS_PREFETCH=1: the next group's three 16-B loads issued before
this group's LDS work) and the balanced tail (the default; HIST_RANGE8 launches) (tool, not
product): 2^28 uniform tuples, H = 2^30, full outputs (hash u32 + queue u32) and counts only,
three alternating rounds, medians of 10 launches after 5 warm ones.  One JSON line per Q.

usage: python tools/prefetch_ab.py [Q ...]"""
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


VARIANTS = {"static": {"RSS_BALANCE": "0", "RSS_PREFETCH": "0"},
            "prefetch": {"RSS_BALANCE": "0", "RSS_PREFETCH": "1"},
            "tail": {"RSS_BALANCE": "1", "RSS_PREFETCH": "0"}}


def timed(Q, outputs, variant, reps=10, warm=5):
    os.environ.update(VARIANTS[variant])
    c = torch.zeros(Q, dtype=torch.int64, device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    hp, qp = (h.data_ptr(), q.data_ptr()) if outputs else (None, None)
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tup.data_ptr(), n, H, Q, hp, qp, c.data_ptr(), 0, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    assert int(c.sum()) == n
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return x[len(x) // 2]


for Q in [int(x) for x in sys.argv[1:]] or [20000, 65536, 131072, 161144]:
    rec = {"Q": Q, "tuples": n}
    for rnd in range(3):
        for v in VARIANTS:
            for outputs in (True, False):
                k = "%s_%s_ms" % (v, "full" if outputs else "counts")
                rec.setdefault(k, []).append(round(timed(Q, outputs, v), 4))
    os.environ.pop("RSS_PREFETCH", None)
    os.environ.pop("RSS_BALANCE", None)
    for k in [k for k in rec if k.endswith("_ms")]:
        rec[k + "_best"] = min(rec[k])
    print(json.dumps(rec), flush=True)
