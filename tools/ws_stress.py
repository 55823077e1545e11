"""Single-pass counts stress (tool, not product): 6000 back-to-back rss_hash_device_ws
launches on ONE workspace over three batches of different sizes (incl. grids of one and of
256 workgroups), overwrite and accumulate, every result checked against the oracle's counts
for that batch.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from oracle.oracle import OracleLib  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

H, Q = 128, 24
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
kb = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
key = _native.prepare_key(kb)
ora = OracleLib()
batches = []
for seed, n in ((1, 1000), (2, (1 << 20) + 3), (3, 1 << 22)):
    host = ora.generate(seed, 0, n)
    want = ora.run(kb, host, H, Q, want_hash=False, want_queue=False)[2]
    batches.append((n, torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev), want))
ws = torch.zeros(_native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)
outs = torch.zeros((600, Q), dtype=torch.int64, device=dev)
h = torch.empty(1 << 22, dtype=torch.int32, device=dev)
bad = 0
launches = 0
for rnd in range(10):
    for i in range(600):
        n, t, _ = batches[i % 3]
        _native.hash_device(key, t.data_ptr(), n, H, Q, h.data_ptr() if i % 2 else None, None,
                            outs[i].data_ptr(), 0, s, ws.data_ptr())
        launches += 1
    torch.cuda.synchronize()
    got = outs.cpu().numpy().view(np.uint64)
    for i in range(600):
        bad += int(not np.array_equal(got[i], batches[i % 3][2]))
    outs.zero_()
acc = torch.zeros(Q, dtype=torch.int64, device=dev)
for i in range(300):
    n, t, _ = batches[i % 3]
    _native.hash_device(key, t.data_ptr(), n, H, Q, None, None, acc.data_ptr(),
                        _native.FLAG_ACCUMULATE, s, ws.data_ptr())
    launches += 1
torch.cuda.synchronize()
acc_ok = bool(np.array_equal(acc.cpu().numpy().view(np.uint64), 100 * sum(b[2] for b in batches)))
print(json.dumps({"launches": launches, "mismatched_batches": bad, "accumulate_ok": acc_ok,
                  "workspace_zero": int(ws.abs().sum()) == 0}))
sys.exit(0 if bad == 0 and acc_ok else 1)
