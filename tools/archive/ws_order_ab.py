"""Same-process A/B of single-pass launch variants, alternating in blocks of launches on the
same buffers: the default (release/acquire hand-off, balanced tail) against
RSS_WS_ORDER=relaxed (no release ticket / acquire fence; round 2's form) and RSS_BALANCE=0
(static grid-stride to the end) and RSS_OFF32=0 (64-bit addressing); DESIGN.md §3 "Single-pass counts", "Balanced tail".  The bench's step:
rss_hash_device_ws over 2^28 tuples, H=128, Q=24, u8 queues.

    python tools/ws_order_ab.py [rounds]
"""
raise SystemExit("archived (round 5): this A/B probe set RSS_* environment switches that the "
                 "product library no longer reads, so every variant would time the default "
                 "path; the alternatives are reachable through tests/hooks.py only")

import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rss_simulator_nvidia_amd import _native  # noqa: E402
from rss_simulator_nvidia_amd.resident import ResidentBatch  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    placement = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n, H, Q = 1 << 28, 128, 24
    key_bytes = [int(x, 16) for x in open(os.path.join(ROOT, "tests", "golden", "example_input",
                                                       "hash_key.txt")).read().split(":")]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    key = _native.prepare_key(key_bytes)
    batch = ResidentBatch(n, key, H, Q, device=dev, queue_width="u8", placement=(1, placement),
                          fill=lambda t: _native.generate_device(0x5EED, 0, n, t.data_ptr(),
                                                                 stream.cuda_stream),
                          stream=stream)
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    modes = {"default": {}, "relaxed": {"RSS_WS_ORDER": "relaxed"}, "static": {"RSS_BALANCE": "0"},
             "off64": {"RSS_OFF32": "0"},
             "counts_default": {}, "counts_static": {"RSS_BALANCE": "0"}}
    res = {m: [] for m in modes}
    for _ in range(200):  # clock settle
        batch.hash(counts=counts)
    for r in range(rounds):
        order = list(modes) if r % 2 == 0 else list(modes)[::-1]
        for mode in order:
            for var in ("RSS_WS_ORDER", "RSS_BALANCE", "RSS_OFF32"):
                os.environ.pop(var, None)
            os.environ.update(modes[mode])
            outputs = not mode.startswith("counts")  # counts only: the register-table kernel
            for _ in range(10):
                batch.hash(counts=counts, outputs=outputs)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(50):
                batch.hash(counts=counts, outputs=outputs)
            b.record(stream)
            torch.cuda.synchronize()
            res[mode].append(a.elapsed_time(b) / 50)
            assert int(counts.sum()) == n
    for var in ("RSS_WS_ORDER", "RSS_BALANCE", "RSS_OFF32"):
        os.environ.pop(var, None)
    out = {m: {"ms_per_launch": v, "median": statistics.median(v)} for m, v in res.items()}
    out["default_minus_relaxed_us"] = 1e3 * (out["default"]["median"] - out["relaxed"]["median"])
    out["static_minus_default_us"] = 1e3 * (out["static"]["median"] - out["default"]["median"])
    out["off64_minus_default_us"] = 1e3 * (out["off64"]["median"] - out["default"]["median"])
    out["counts_static_minus_default_us"] = 1e3 * (out["counts_static"]["median"] -
                                                   out["counts_default"]["median"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
