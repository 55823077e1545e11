"""Process start-up costs of the CLI (tool, not product): library load, first HIP call
(device count), context creation, and a tiny hash, each timed from a fresh process."""
import json
import os
import sys
import time

t0 = time.perf_counter()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rss_simulator_nvidia_amd import _native  # noqa: E402
t1 = time.perf_counter()
lib = _native.load()
t2 = time.perf_counter()
n = _native.device_count()
t3 = time.perf_counter()
ctx = _native.HostContext(0)
t4 = time.perf_counter()
import numpy as np  # noqa: E402
key = _native.prepare_key(list(range(40)))
ctx.hash(key, np.zeros((1024, 3), np.uint32), 128, 24)
t5 = time.perf_counter()
ctx.hash(key, np.zeros((1024, 3), np.uint32), 128, 24)
t6 = time.perf_counter()
print(json.dumps({"import_s": t1 - t0, "dlopen_s": t2 - t1, "device_count_s": t3 - t2,
                  "ctx_create_s": t4 - t3, "first_hash_s": t5 - t4, "second_hash_s": t6 - t5,
                  "devices": n}))
