"""Counts-only load shape A/B in one process (tool, not product): rss_counts_perm_kernel with
its product loads (a lane's 4 tuples as 3 x 16 B at a 48-B stride) vs whole-tuple dwordx3
loads (RSS_COUNTS_WHOLE=1: a wave's instruction j reads tuples 64j + lane), alternating, on
three input allocations of 2^28 tuples; counts checked equal.  One JSON line per input."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n, H, Q = 1 << 28, 128, 24
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
inputs = []
for _ in range(3):
    t = torch.empty(3 * n, dtype=torch.int32, device=dev)
    _native.generate_device(SEED, 0, n, t.data_ptr(), s.cuda_stream)
    inputs.append(t)
counts = {m: torch.zeros(Q, dtype=torch.int64, device=dev) for m in ("0", "1")}


def run(t, mode, reps, c=None):
    os.environ["RSS_COUNTS_WHOLE"] = mode
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e in ev:
        e[0].record(s)
        _native.hash_device(key, t.data_ptr(), n, H, Q, None, None, (c if c is not None else counts[mode]).data_ptr(), 0, s.cuda_stream)
        e[1].record(s)
    torch.cuda.synchronize()
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return x[len(x) // 2]


for k, t in enumerate(inputs):
    for m in ("0", "1"):
        run(t, m, 30)  # warm / settle
    res = {"0": [], "1": []}
    for _ in range(6):
        for m in ("0", "1"):
            res[m].append(round(run(t, m, 20), 4))
    same = bool(torch.equal(counts["0"], counts["1"]))
    print(json.dumps({"input": k, "product_ms": res["0"], "whole_tuple_ms": res["1"],
                      "product_median": sorted(res["0"])[3], "whole_median": sorted(res["1"])[3],
                      "counts_equal": same}), flush=True)
