"""HBM placement of the bench's three streams (tool, not product): the same full-output
launch (2^28 resident tuples, u32 hash + u8 queue + counts, H=128, Q=24) timed with the
tuple / hash / queue arrays carved from one allocation at different relative offsets,
interleaved in rounds so that clock / thermal drift shows up as drift across rounds and
placement as a stable difference between layouts.  Prints one JSON line per round and a
summary line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 28
MiB = 1 << 20
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
counts = torch.zeros(24, dtype=torch.int64, device=dev)
IN, HB, QB = 12 * n, 4 * n, n
GiB = 1 << 30
slack = int(os.environ.get("SLACK_MIB", "64")) * MiB
buf = torch.empty(IN + HB + QB + 3 * slack, dtype=torch.uint8, device=dev)
base = buf.data_ptr()

# (name, tuples offset, hash offset, queue offset) in bytes from the buffer start
BIG = os.environ.get("BIG") == "1"
layouts = [
    ("gap0", 0, IN, IN + HB),
    ("gap256M", 0, IN + 256 * MiB, IN + HB + 512 * MiB),
    ("gap512M", 0, IN + 512 * MiB, IN + HB + 1024 * MiB),
    ("gap1G", 0, IN + GiB, IN + HB + 2 * GiB),
    ("hgap1G_q0", 0, IN + GiB, IN + HB + GiB),
    ("hgap0_q1G", 0, IN, IN + HB + GiB),
    ("gap768M", 0, IN + 768 * MiB, IN + HB + 1536 * MiB),
] if BIG else [
    ("packed", 0, IN, IN + HB),
    ("hash+2M", 0, IN + 2 * MiB, IN + HB + 4 * MiB),
    ("hash+1M+64K", 0, IN + MiB + 65536, IN + HB + 2 * MiB + 131072),
    ("hash+8M+4K", 0, IN + 8 * MiB + 4096, IN + HB + 16 * MiB + 8192),
    ("hash+32M", 0, IN + 32 * MiB, IN + HB + 64 * MiB),
    ("in+16M", 16 * MiB, IN + 32 * MiB, IN + HB + 48 * MiB),
]
for name, a, b, c in layouts:
    assert a % 16 == 0 and b % 16 == 0 and c % 16 == 0 and c + QB <= buf.numel(), name
_native.generate_device(SEED, 0, n, base + layouts[0][1], sp)
torch.cuda.synchronize()


def run(layout, reps=20, warm=5):
    _, a, b, c = layout
    if a != layouts[0][1]:
        _native.generate_device(SEED, 0, n, base + a, sp)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, base + a, n, 128, 24, base + b, base + c, counts.data_ptr(),
                            _native.FLAG_QUEUE_U8 | _native.FLAG_ACCUMULATE, sp)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    t = sorted(x.elapsed_time(y) for x, y in ev)
    return t[len(t) // 2]


# separately allocated tensors, as bench.py does
sep_t = torch.empty(3 * n, dtype=torch.int32, device=dev)
sep_h = torch.empty(n, dtype=torch.int32, device=dev)
sep_q = torch.empty(n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, sep_t.data_ptr(), sp)


def run_sep(reps=20, warm=5):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash_device(key, sep_t.data_ptr(), n, 128, 24, sep_h.data_ptr(), sep_q.data_ptr(),
                            counts.data_ptr(), _native.FLAG_QUEUE_U8 | _native.FLAG_ACCUMULATE, sp)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    t = sorted(x.elapsed_time(y) for x, y in ev)
    return t[len(t) // 2]


rounds = int(os.environ.get("ROUNDS", "4"))
table = {name: [] for name, *_ in layouts}
table["bench_tensors"] = []
for r in range(rounds):
    row = {"round": r, "bench_tensors": run_sep()}
    table["bench_tensors"].append(row["bench_tensors"])
    for lay in (layouts if r % 2 == 0 else layouts[::-1]):
        row[lay[0]] = run(lay)
        table[lay[0]].append(row[lay[0]])
    print(json.dumps(row), flush=True)
print(json.dumps({"summary_median_ms": {k: sorted(v)[len(v) // 2] for k, v in table.items()},
                  "addresses": {"buf": hex(base), "sep_tuples": hex(sep_t.data_ptr()),
                                "sep_hash": hex(sep_h.data_ptr()),
                                "sep_queue": hex(sep_q.data_ptr())}}), flush=True)
