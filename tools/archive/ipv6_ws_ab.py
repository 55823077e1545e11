"""Same-buffer A/B of the IPv6 step (tool, not product): the plain launch
(``rss_hash6_device``, static grid-stride, accumulating counts) against the single-pass
launch (``rss_hash6_device_ws``) with the balanced tail and with ``RSS_BALANCE=0``.

2^28 / 3 uniform 36-byte tuples (the size of ``profiles/r02/ipv6_vs_stream_floor.log``),
hash u32 + queue u8 + counts = 41 B per tuple.  Each variant: 20 warm launches, then one HIP
event pair around 40 launches; the variants alternate for ``ROUNDS`` rounds.  Prints one JSON
line.  usage: python tools/ipv6_ws_ab.py [ROUNDS]
"""
raise SystemExit("archived (round 5): this A/B probe set RSS_* environment switches that the "
                 "product library no longer reads, so every variant would time the default "
                 "path; the alternatives are reachable through tests/hooks.py only")

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rss_simulator_nvidia_amd import _native  # noqa: E402


def main(rounds):
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    n = ((1 << 28) // 3) & ~3
    words = torch.randint(-2**31, 2**31 - 1, (9 * n,), dtype=torch.int32, device=dev)
    h = torch.empty(n, dtype=torch.int32, device=dev)
    q = torch.empty(n, dtype=torch.uint8, device=dev)
    c = torch.zeros(24, dtype=torch.int64, device=dev)
    ws = torch.zeros(_native.counts_workspace_bytes(128, 24) // 8, dtype=torch.int64, device=dev)
    k6 = _native.prepare_key6(list(range(3, 43)))

    def plain():
        _native.hash6_device(k6, words.data_ptr(), n, 128, 24, h.data_ptr(), q.data_ptr(),
                             c.data_ptr(), _native.FLAG_QUEUE_U8 | _native.FLAG_ACCUMULATE, sp)

    def single_pass():
        _native.hash6_device(k6, words.data_ptr(), n, 128, 24, h.data_ptr(), q.data_ptr(),
                             c.data_ptr(), _native.FLAG_QUEUE_U8, sp, ws.data_ptr())

    variants = {"plain": (plain, "1"), "ws_balanced": (single_pass, "1"),
                "ws_static": (single_pass, "0")}
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, (fn, bal) in variants.items():
            os.environ["RSS_BALANCE"] = bal
            for _ in range(20):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(40):
                fn()
            b.record(stream)
            torch.cuda.synchronize()
            res[name].append(round(a.elapsed_time(b) / 40, 4))
    os.environ.pop("RSS_BALANCE", None)
    best = {k: min(v) for k, v in res.items()}
    print(json.dumps({"tuples": n, "bytes_per_tuple": 41, "ms_per_launch": res, "best_ms": best,
                      "best_TBs": {k: round(n * 41 / (v / 1e3) / 1e12, 3) for k, v in best.items()}}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
