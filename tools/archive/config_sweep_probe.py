"""Kernel time across (H, Q) configurations on fixed buffers (tool, not product): full
output (hash u32 + the narrowest queue width) and counts only, 2^28 tuples, medians of 10
launches after 5 warm ones, against the same buffers' 12 R + 5 W / 12 R + 6 W / 12 R + 8 W
byte counts.  Count vectors are min(H, Q) long (``_native.queue_modulus``): rows with Q >= H
run the Q <= H kernel.  For Q > 8192 the round-2 narrow range passes (RSS_WIDE_HIST=0) are
timed beside the wide pass; the 12-bit tables (RSS_SMALL_LUT=0: 16384 queues in the
hash pass) beside the small tables (up to 80572 in u16 bins, 161144 in u8) for Q > 8192.  ``many`` as the argument: the Q > 8192 rows
only.  Prints one JSON line per configuration."""
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
q = torch.empty(n, dtype=torch.int32, device=dev)


def timed(H, Q, outputs, flags, reps=10, warm=5):
    c = torch.zeros(_native.queue_modulus(H, Q)[1], dtype=torch.int64, device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    hp, qp = (h.data_ptr(), q.data_ptr()) if outputs else (None, None)
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, tup.data_ptr(), n, H, Q, hp, qp, c.data_ptr(),
                            flags | _native.FLAG_ACCUMULATE, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return round(x[len(x) // 2], 4)


ROWS = [(128, 24), (128, 16), (512, 64), (100, 7), (1000, 24), (65536, 24),
        (128, 129), (128, 20000), (128, 300000), (128, 4 * 10 ** 9),
        (65536, 4096), (1 << 20, 1000), (1 << 20, 8193), (1 << 20, 16384), (1 << 20, 20000),
        (1 << 20, 40000),
        (4294967295, 65536), (1 << 30, 80572), (1 << 30, 131072), (1 << 30, 131073),
        (1 << 30, 262144)]
many = sys.argv[1:] == ["many"]
for H, Q in ROWS:
    qn = _native.queue_modulus(H, Q)[1]
    if many and qn <= 8192:
        continue
    width = 1 if qn <= 256 else (2 if qn <= 65536 else 4)
    fl = {1: _native.FLAG_QUEUE_U8, 2: _native.FLAG_QUEUE_U16, 4: 0}[width]
    full = timed(H, Q, True, fl)
    co = timed(H, Q, False, 0)
    rec = {"H": H, "Q": Q, "queues_counted": qn, "queue_bytes": width, "full_ms": full,
           "full_GBs": round(n * (16 + width) / (full / 1e3) / 1e9),
           "counts_ms": co, "counts_read_GBs": round(n * 12 / (co / 1e3) / 1e9)}
    if qn > 8192:  # the round-2 narrow passes beside the wide one
        os.environ["RSS_WIDE_HIST"] = "0"
        rec["narrow_full_ms"] = timed(H, Q, True, fl)
        rec["narrow_counts_ms"] = timed(H, Q, False, 0)
        os.environ.pop("RSS_WIDE_HIST", None)
    if qn > 8192:  # the 12-bit tables: 16384 queues in the hash pass, the rest from the column
        os.environ["RSS_SMALL_LUT"] = "0"
        rec["tables12_full_ms"] = timed(H, Q, True, fl)
        rec["tables12_counts_ms"] = timed(H, Q, False, 0)
        os.environ.pop("RSS_SMALL_LUT", None)
    print(json.dumps(rec), flush=True)
