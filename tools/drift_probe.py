"""Per-launch time over a long run of back-to-back launches (tool, not product): is the bench's
timed region slower than the placement probe's short bursts because the clocks settle lower
under sustained load, and what do per-launch HIP events cost per step?  2^28 tuples, H=128,
Q=24, u8 queues, placed ResidentBatch buffers (2 x 12 candidates), single-pass counts.
Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402
from rss_simulator_nvidia_amd.resident import ResidentBatch  # noqa: E402

n, H, Q = 1 << 28, 128, 24
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
batch = ResidentBatch(n, key, H, Q, device=dev, placement=(2, 12),
                      fill=lambda t: _native.generate_device(SEED, 0, n, t.data_ptr(), s.cuda_stream))
counts = torch.zeros(Q, dtype=torch.int64, device=dev)
out = {"chosen_ms": batch.report["chosen_ms"]}

W = 100  # launches per window
windows = []
for w in range(12):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(W)]
    for e in ev:
        e[0].record(s)
        batch.hash(counts)
        e[1].record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    windows.append([round(sum(t) / W, 4), round(t[W // 2], 4), round(t[0], 4), round(t[-1], 4)])
out["events_windows_mean_median_min_max_ms"] = windows

walls = {}
for mode in ("events", "no_events", "events_every_other"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(400)]
    for i in range(400):
        rec = mode == "events" or (mode == "events_every_other" and i % 2 == 0)
        if rec:
            ev[i][0].record(s)
        batch.hash(counts)
        if rec:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    walls[mode] = round((time.perf_counter() - t0) * 1e3 / 400, 4)
out["wall_ms_per_launch"] = walls

# short bursts with a pause between them (the probe's pattern)
bursts = []
for b in range(6):
    time.sleep(0.3)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for e in ev:
        e[0].record(s)
        batch.hash(counts)
        e[1].record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(c) for a, c in ev)
    bursts.append([round(t[0], 4), round(t[5], 4), round(t[-1], 4)])
out["bursts_after_pause_min_median_max_ms"] = bursts
print(json.dumps(out))
