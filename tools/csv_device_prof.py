"""Fixed workload for rocprofv3 --kernel-trace --stats of the device CSV kernels (tool).

Generates a 2^24-row canonical CSV (tools/gen_csv.c), then runs rss_csv_hash_text on the
in-memory image 5 times (H=128, Q=24).  usage: python tools/csv_device_prof.py [ROWS] [DIR]
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
work = sys.argv[2] if len(sys.argv) > 2 else "/tmp/rss_csvprof"
os.makedirs(work, exist_ok=True)
gen, path = os.path.join(work, "gen_csv"), os.path.join(work, "in.csv")
subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(ROOT, "tools", "gen_csv.c")], check=True)
subprocess.run([gen, str(rows), "12345", path], check=True)

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

data = np.fromfile(path, dtype=np.uint8)
ctx = _native.default_context()
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
for i in range(5):
    t0 = time.perf_counter()
    image, counts, n = ctx.csv_hash_text(key, data, 128, 24)
    print("run %d: %d rows, %d B in, %d B out, %.4f s" % (i, n, len(data), len(image),
                                                          time.perf_counter() - t0), flush=True)
