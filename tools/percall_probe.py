"""Latency of the reference-style per-tuple call (tool, not product): the reference's
``Simulator.__calc_entry_hash`` (simulator.py:80-92) calls ``Toeplitz.compute_hash`` once per
row; here that call goes to the GPU through ``HostContext.hash``.  Prints one JSON line:
per-call latency of ``compute_hash`` and of ``compute_hash_batch`` at several batch sizes,
plus the host CPU share the bench's CPU baseline would use."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bench import EXAMPLE_KEY, cpu_share  # noqa: E402
from rss_simulator_nvidia_amd.toeplitz import Toeplitz  # noqa: E402

key = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
tz = Toeplitz(key)
out = {"cpu_share": cpu_share(), "os_cpu_count": os.cpu_count(),
       "affinity": len(os.sched_getaffinity(0)), "omp": os.environ.get("OMP_NUM_THREADS")}
assert tz.compute_hash("3.3.3.1", "3.3.3.2", 5201, 5001) == 3151101778
for _ in range(200):
    tz.compute_hash("3.3.3.1", "3.3.3.2", 5201, 5001)
reps = 2000
t0 = time.perf_counter()
for i in range(reps):
    tz.compute_hash("10.0.%d.%d" % (i >> 8 & 255, i & 255), "3.3.3.2", 1024 + i, 80)
dt = time.perf_counter() - t0
out["compute_hash_us"] = dt / reps * 1e6
# the Python share of that call: string parsing + packing, no native call
from rss_simulator_nvidia_amd.ingest import ip_to_u32, pack_columns  # noqa: E402
t0 = time.perf_counter()
for i in range(reps):
    pack_columns([ip_to_u32("10.0.%d.%d" % (i >> 8 & 255, i & 255))], [ip_to_u32("3.3.3.2")],
                 [(1024 + i) & 0xFFFF], [80])
out["python_pack_us"] = (time.perf_counter() - t0) / reps * 1e6
rng = np.random.default_rng(1)
batch = {}
for n in (1, 16, 256, 4096, 65536, 1 << 20):
    tup = rng.integers(0, 2**32, (n, 3), dtype=np.uint64).astype(np.uint32)
    for _ in range(5):
        tz.compute_hash_batch(tup)
    r = max(5, min(500, (1 << 22) // n))
    t0 = time.perf_counter()
    for _ in range(r):
        tz.compute_hash_batch(tup)
    dt = (time.perf_counter() - t0) / r
    batch[str(n)] = {"us_per_call": dt * 1e6, "tuples_per_s": n / dt}
out["compute_hash_batch"] = batch
print(json.dumps(out), flush=True)
