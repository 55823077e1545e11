"""CSV -> CSV above 4 GiB (tool, not product): a generated canonical file of ROWS rows
through the device file path (rss_csv_hash_file, line-aligned segments) and through the
host text path (RSS_CSV_DEVICE=0); the two output files must be identical.  Prints one
JSON object.  usage: python tools/e2e_big.py [ROWS] [WORKDIR]"""
import filecmp
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native, fastcsv  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 120_000_000
work = sys.argv[2] if len(sys.argv) > 2 else "/tmp/rss_big"
os.makedirs(work, exist_ok=True)
gen = os.path.join(work, "gen_csv")
subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(ROOT, "tools", "gen_csv.c")], check=True)
src = os.path.join(work, "big.csv")
t0 = time.perf_counter()
subprocess.run([gen, str(rows), "4242", src], check=True)
print("generated %d rows, %.2f GB in %.1f s" % (rows, os.path.getsize(src) / 1e9,
                                               time.perf_counter() - t0), file=sys.stderr, flush=True)
key = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
_native.default_context()
result = {"rows": rows, "bytes_in": os.path.getsize(src)}
for path in ("device", "host"):
    os.environ["RSS_CSV_DEVICE"] = "1" if path == "device" else "0"
    out = os.path.join(work, "out_%s.csv" % path)
    if os.path.exists(out):
        os.unlink(out)
    t = {}
    t0 = time.perf_counter()
    assert fastcsv.run_csv(key, src, 128, 24, out, timings=t)
    wall = time.perf_counter() - t0
    result[path] = {"wall_s": wall, "rows_per_s": rows / wall, "path_taken": t.get("path"),
                    "bytes_out": os.path.getsize(out)}
    print(path, result[path], file=sys.stderr, flush=True)
result["outputs_identical"] = filecmp.cmp(os.path.join(work, "out_device.csv"),
                                          os.path.join(work, "out_host.csv"), shallow=False)
print(json.dumps(result))
