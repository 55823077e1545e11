"""IPv6 kernel throughput (tool, not product): 2**26 resident 36-byte tuples, H=128, Q=24."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
key = _native.prepare_key6([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tuples = torch.randint(-2**31, 2**31 - 1, (9 * n,), dtype=torch.int32, device=dev)
hashes = torch.empty(n, dtype=torch.int32, device=dev)
queues = torch.empty(n, dtype=torch.int32, device=dev)
counts = torch.empty(24, dtype=torch.int64, device=dev)
res = {"tuples": n}
for name, hp, qp, fl, qbytes in (
        ("full", hashes.data_ptr(), queues.data_ptr(), 0, 4),
        ("full_u8", hashes.data_ptr(), queues.data_ptr(), _native.FLAG_QUEUE_U8, 1),
        ("counts_only", None, None, 0, 0)):
    run = lambda: _native.hash6_device(key, tuples.data_ptr(), n, 128, 24, hp, qp,  # noqa: E731
                                       counts.data_ptr(), fl, s)
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    nbytes = 36 + (4 + qbytes if hp else 0)
    res[name] = {"ms": ms, "tuples_per_s": n / ms * 1e3, "GB_per_s": n * nbytes / ms / 1e6}
print(json.dumps(res))
