"""IPv6 counts-only launch time, register-table kernel vs LDS-table kernel (tool, not
product): 2^26 uniform 36-byte tuples, H=128, Q=24, RSS_COUNTS_PERM toggled per launch
group, interleaved rounds.  Prints one JSON line per round."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = 1 << 26
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev)
key6 = _native.prepare_key6([int(x, 16) for x in EXAMPLE_KEY.split(":")])
words = torch.randint(-2**31, 2**31 - 1, (9 * n,), dtype=torch.int32, device=dev)
counts = torch.zeros(24, dtype=torch.int64, device=dev)


def timed(perm, reps=20, warm=10):
    os.environ["RSS_COUNTS_PERM"] = "1" if perm else "0"
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for i in range(-warm, reps):
        if i >= 0:
            ev[i][0].record(s)
        _native.hash6_device(key6, words.data_ptr(), n, 128, 24, None, None, counts.data_ptr(),
                             _native.FLAG_ACCUMULATE, s.cuda_stream)
        if i >= 0:
            ev[i][1].record(s)
    torch.cuda.synchronize()
    x = sorted(a.elapsed_time(b) for a, b in ev)
    return round(x[len(x) // 2], 4)


for r in range(3):
    lut, perm = timed(False), timed(True)
    print(json.dumps({"round": r, "lut_ms": lut, "perm_ms": perm,
                      "perm_read_TBs": round(36 * n / (perm / 1e3) / 1e12, 3),
                      "lut_read_TBs": round(36 * n / (lut / 1e3) / 1e12, 3)}), flush=True)
