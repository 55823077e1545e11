"""Many-queues launches with u8 bins (HIST_RANGE8) against the u16 path (RSS_RANGE8=0) on the
same buffers (tool, not product): 2^28 uniform tuples, H = 2^30, full outputs (hash u32 +
queue u32) and counts only; medians of 10 launches after 5 warm ones, alternating variants in
two rounds.  `force` = the poison-gated recount on every launch (RSS_RANGE8_DEBUG=force: what
a batch that wraps a u8 bin costs); `column` = counts only through a scratch queue column
instead of residual lists (RSS_RESID=0).  Prints one JSON line per Q.

usage: python tools/range8_probe.py [Q ...]"""
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
VARIANTS = {"u8": {}, "u16": {"RSS_RANGE8": "0"}, "force": {"RSS_RANGE8_DEBUG": "force"},
            "column": {"RSS_RESID": "0"}}


def timed(Q, outputs, env, reps=10, warm=5):
    for k, v in env.items():
        os.environ[k] = v
    try:
        c = torch.zeros(Q, dtype=torch.int64, device=dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        hp, qp = (h.data_ptr(), q.data_ptr()) if outputs else (None, None)
        for i in range(-warm, reps):
            if i >= 0:
                ev[i][0].record(s)
            _native.hash_device(key, tup.data_ptr(), n, H, Q, hp, qp, c.data_ptr(), 0,
                                s.cuda_stream)
            if i >= 0:
                ev[i][1].record(s)
        torch.cuda.synchronize()
        assert int(c.sum()) == n
        x = sorted(a.elapsed_time(b) for a, b in ev)
        return x[len(x) // 2]
    finally:
        for k in env:
            os.environ.pop(k, None)


qs = [int(x) for x in sys.argv[1:]] or [65536, 80577, 100000, 131072, 161144, 200000, 262144,
                                        1000000]
# the bench's step shape on the same input for scale: H=128, Q=24, u8 queues, counts
c24 = torch.zeros(24, dtype=torch.int64, device=dev)
for Q in qs:
    rec = {"Q": Q, "tuples": n}
    for rnd in range(2):
        for name, env in VARIANTS.items():
            if name == "force" and rnd:
                continue
            for outputs in (True, False):
                k = "%s_%s_ms" % (name, "full" if outputs else "counts")
                t = timed(Q, outputs, env)
                rec[k] = round(min(t, rec.get(k, t)), 4)
    rec["u8_full_GBs"] = round(n * 20 / (rec["u8_full_ms"] / 1e3) / 1e9)
    rec["u8_counts_read_GBs"] = round(n * 12 / (rec["u8_counts_ms"] / 1e3) / 1e9)
    print(json.dumps(rec), flush=True)
