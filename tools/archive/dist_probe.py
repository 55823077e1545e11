"""Uniform vs flow-like input on one box (tool, not product).

For each distribution (bench.py's generators, 2**28 resident tuples, H=128, Q=24) launches
counts-only x3 then full-u8 x3 and prints their HIP-event times; under rocprofv3 --pmc the
dispatch order is: uniform counts, uniform full, flow counts, flow full (3 each).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

n, H, Q = 1 << 28, int(os.environ.get("PROBE_H", 128)), int(os.environ.get("PROBE_Q", 24))
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
s = stream.cuda_stream
key = _native.prepare_key([int(x, 16) for x in bench.EXAMPLE_KEY.split(":")])
tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
hashes = torch.empty(n, dtype=torch.int32, device=dev)
queues = torch.empty(n, dtype=torch.int32, device=dev)
counts = torch.zeros(Q, dtype=torch.int64, device=dev)
for dist in ("uniform", "flow"):
    if dist == "uniform":
        _native.generate_device(bench.SEED, 0, n, tuples.data_ptr(), s)
    else:
        bench.flow_device(torch, tuples, 0, n, dev)
    torch.cuda.synchronize()
    for mode, hp, qp, fl in (("counts", None, None, 0),
                             ("full_u8", hashes.data_ptr(), queues.data_ptr(),
                              _native.FLAG_QUEUE_U8)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(3):
            _native.hash_device(key, tuples.data_ptr(), n, H, Q, hp, qp, counts.data_ptr(),
                                fl | _native.FLAG_ACCUMULATE, s)
        b.record(stream)
        torch.cuda.synchronize()
        print("%-8s %-8s %.4f ms" % (dist, mode, a.elapsed_time(b) / 3), flush=True)
