"""Same-buffer A/B of the single-pass fold (tool, not product; DESIGN.md §3 "Single-pass
counts"): the arrival fold (default: every workgroup's add carries an arrival count, the last
add per queue writes that queue's count -- one atomic round trip on the last workgroup's
path) against RSS_FOLD=ticket (sums, a ticket, the last workgroup's exchanges -- three), with
the balanced tail and with the static walk (RSS_BALANCE=0), beside the plain accumulating
launch (no workspace).  The bench's step (2^28 tuples, H=128, Q=24, u8 queues) and its
counts-only form; variants alternate in blocks of 50 launches.

    python tools/ws_fold_ab.py [rounds]
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
    n, H, Q = 1 << 28, 128, 24
    key_bytes = [int(x, 16) for x in open(os.path.join(ROOT, "tests", "golden", "example_input",
                                                       "hash_key.txt")).read().split(":")]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    key = _native.prepare_key(key_bytes)
    batch = ResidentBatch(n, key, H, Q, device=dev, queue_width="u8", placement=(1, 1),
                          fill=lambda t: _native.generate_device(0x5EED, 0, n, t.data_ptr(), sp),
                          stream=stream)
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    ws = torch.zeros(_native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)

    def launch(fold, outputs, balance="1"):
        h = batch.hashes.data_ptr() if outputs else None
        q = batch.queues.data_ptr() if outputs else None
        flags = _native.FLAG_QUEUE_U8 if outputs else 0
        os.environ["RSS_BALANCE"] = balance
        if fold is None:  # plain: accumulate into the counts, no workspace
            _native.hash_device(key, batch.tuples.data_ptr(), n, H, Q, h, q, counts.data_ptr(),
                                flags | _native.FLAG_ACCUMULATE, sp)
        else:
            os.environ["RSS_FOLD"] = fold
            _native.hash_device(key, batch.tuples.data_ptr(), n, H, Q, h, q, counts.data_ptr(),
                                flags, sp, ws.data_ptr())

    modes = {"arrival": ("arrival", True, "1"), "ticket": ("ticket", True, "1"),
             "arrival_static": ("arrival", True, "0"), "ticket_static": ("ticket", True, "0"),
             "plain": (None, True, "1"),
             "counts_arrival": ("arrival", False, "1"), "counts_ticket": ("ticket", False, "1"),
             "counts_plain": (None, False, "1")}
    res = {m: [] for m in modes}
    for _ in range(200):  # clock settle
        launch("arrival", True)
    for r in range(rounds):
        order = list(modes) if r % 2 == 0 else list(modes)[::-1]
        for mode in order:
            fold, outputs, balance = modes[mode]
            for _ in range(10):
                launch(fold, outputs, balance)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(50):
                launch(fold, outputs, balance)
            b.record(stream)
            torch.cuda.synchronize()
            res[mode].append(a.elapsed_time(b) / 50)
            if fold is not None:
                assert int(counts.sum()) == n and int(ws.abs().sum()) == 0
    for var in ("RSS_FOLD", "RSS_BALANCE"):
        os.environ.pop(var, None)
    out = {m: {"ms_per_launch": v, "median": statistics.median(v)} for m, v in res.items()}
    for m in ("ticket", "arrival_static", "ticket_static", "plain"):
        out[m + "_minus_arrival_us"] = 1e3 * (out[m]["median"] - out["arrival"]["median"])
    for m in ("counts_ticket", "counts_plain"):
        out[m + "_minus_arrival_us"] = 1e3 * (out[m]["median"] - out["counts_arrival"]["median"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
