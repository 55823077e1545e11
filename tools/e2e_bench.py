"""End-to-end (host memory) rates for DESIGN.md §6 (tool, not product).

1. CSV -> CSV through the CLI fast path, per stage: the device text path
   (rss_csv_hash_text: parse / hash / format on the GPU) and the host text path
   (RSS_CSV_DEVICE=0: native parse, rss_hash_host = pinned chunked H2D -> kernel -> D2H,
   native format); both outputs must be identical;
2. rss_hash_host alone on host-resident packed tuples (the PCIe-inclusive rate);
3. the pandas CLI path (RSS_CSV_FASTPATH=0) on a smaller file, for comparison.
Prints one JSON object.
usage: python tools/e2e_bench.py [ROWS] [PANDAS_ROWS] [WORKDIR]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native, fastcsv  # noqa: E402
from rss_simulator_nvidia_amd.main import main as cli_main  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
pandas_rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
work = sys.argv[3] if len(sys.argv) > 3 else "/tmp/rss_e2e"
os.makedirs(work, exist_ok=True)
gen = os.path.join(work, "gen_csv")
subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(ROOT, "tools", "gen_csv.c")], check=True)
big, small = os.path.join(work, "big.csv"), os.path.join(work, "small.csv")
subprocess.run([gen, str(rows), "12345", big], check=True)
subprocess.run([gen, str(pandas_rows), "777", small], check=True)
key = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
H, Q = 128, 24
result = {"rows": rows, "htable": H, "queues": Q}

# CSV -> CSV on each path: the first call (cold: staging allocation, page cache state
# as left by the generator) and a second call (warm); the outputs must be identical
_native.default_context()
for path in ("device", "host"):
    os.environ["RSS_CSV_DEVICE"] = "1" if path == "device" else "0"
    runs = []
    for _ in range(2):
        out_path = os.path.join(work, "out_big_%s.csv" % path)
        if os.path.exists(out_path):
            os.unlink(out_path)  # truncating an 898 MB page-cached file costs ~0.1 s itself
        t = {}
        t0 = time.perf_counter()
        assert fastcsv.run_csv(key, big, H, Q, out_path, timings=t)
        runs.append((time.perf_counter() - t0, t))
    assert runs[-1][1]["path"] == path
    wall, t = runs[-1]
    result["csv_fastpath_" + path] = {
        "wall_s": wall, "rows_per_s": rows / wall, "first_call_wall_s": runs[0][0],
        "stages_s": {k: v for k, v in t.items() if k in
                     ("read", "parse", "gpu", "format", "write", "device_file")},
        "bytes_in": t["bytes_in"], "bytes_out": t["bytes_out"]}
os.environ["RSS_CSV_DEVICE"] = "1"
result["device_host_outputs_identical"] = \
    open(os.path.join(work, "out_big_device.csv"), "rb").read() == \
    open(os.path.join(work, "out_big_host.csv"), "rb").read()

# the device text path from a host file image (rss_csv_hash_text, file already in memory)
data = np.fromfile(big, dtype=np.uint8)
k0 = _native.prepare_key(key)
ctx = _native.default_context()
ctx.csv_hash_text(k0, data, H, Q, copy=False)
for copy in (False, True):  # the context-owned image (zero-copy view) / the default copy
    t0 = time.perf_counter()
    img, _, _ = ctx.csv_hash_text(k0, data, H, Q, copy=copy)
    wall = time.perf_counter() - t0
    result["csv_hash_text_in_memory" + ("_copy" if copy else "")] = {
        "wall_s": wall, "rows_per_s": rows / wall,
        "note": "file image in host memory -> statistics image in host memory (PCIe-inclusive, "
                "no file I/O)" + ("; plus the copy of the output image out of the context "
                                  "(csv_hash_text's default copy=True)" if copy else
                                  "; the image as a view of the context's buffer (copy=False)")}
    del img
del data

# the CLI as a user runs it: a fresh process (interpreter start, imports, GPU init)
cli = [sys.executable, "-m", "rss_simulator_nvidia_amd", "--key-file",
       os.path.join(ROOT, "tests", "golden", "example_input", "hash_key.txt"), "--ips-file", big,
       "--htable-size", str(H), "--num-queues", str(Q), "--csv", os.path.join(work, "out_cli.csv")]
walls = []
for _ in range(2):
    if os.path.exists(os.path.join(work, "out_cli.csv")):
        os.unlink(os.path.join(work, "out_cli.csv"))
    t0 = time.perf_counter()
    subprocess.run(cli, check=True, cwd=ROOT, stdout=subprocess.DEVNULL)
    walls.append(time.perf_counter() - t0)
result["cli_process"] = {"wall_s": min(walls), "rows_per_s": rows / min(walls), "walls_s": walls,
                         "note": "python -m rss_simulator_nvidia_amd --csv, whole process"}
result["cli_output_identical"] = open(os.path.join(work, "out_cli.csv"), "rb").read() == \
    open(os.path.join(work, "out_big_device.csv"), "rb").read()

# rss_hash_host alone (PCIe-inclusive): packed tuples in host memory -> host outputs
tuples = _native.csv_parse(np.fromfile(big, dtype=np.uint8))[0]
ctx = _native.default_context()
k = _native.prepare_key(key)
ctx.hash(k, tuples[:1 << 20], H, Q)
t0 = time.perf_counter()
h, q, c = ctx.hash(k, tuples, H, Q)
dt = time.perf_counter() - t0
result["host_path"] = {"wall_s": dt, "tuples_per_s": rows / dt,
                       "bytes_moved": rows * 20, "GB_per_s": rows * 20 / dt / 1e9,
                       "note": "12 B/tuple H2D + 8 B/tuple D2H through pinned staging"}
assert int(c.sum()) == rows

# the same on page-locked buffers (pinned once, reused): the copy engines move the caller's
# tuples and outputs directly, no staging copies; also at 4x the size (16 pipeline chunks)
for reps, name in ((1, "host_path_pinned"), (4, "host_path_pinned_4x")):
    src = np.tile(tuples, reps) if reps > 1 else tuples
    m = len(src)
    pin_t = _native.pinned_empty(m, _native.TUPLE_DTYPE)
    pin_t[:] = src
    out = (_native.pinned_empty(m, np.uint32), _native.pinned_empty(m, np.uint32))
    ctx.hash(k, pin_t, H, Q, out=out)
    walls = []
    for _ in range(3):
        t0 = time.perf_counter()
        _, _, c2 = ctx.hash(k, pin_t, H, Q, out=out)
        walls.append(time.perf_counter() - t0)
    dt = min(walls)
    same = bool(np.array_equal(out[0][:rows], h) and np.array_equal(out[1][:rows], q))
    result[name] = {"tuples": m, "wall_s": dt, "walls_s": walls, "tuples_per_s": m / dt,
                    "bytes_moved": m * 20, "GB_per_s": m * 20 / dt / 1e9,
                    "outputs_equal_staged": same,
                    "note": "tuples, hash and queue arrays in rss_host_alloc memory: direct DMA, "
                            "12 B/tuple H2D + 8 B/tuple D2H"}
    assert int(c2.sum()) == m and same
    del pin_t, out, src

# pandas path on the small file
os.environ["RSS_CSV_FASTPATH"] = "0"
t0 = time.perf_counter()
cli_main(["--key-file", os.path.join(ROOT, "tests", "golden", "example_input", "hash_key.txt"),
          "--ips-file", small, "--htable-size", str(H), "--num-queues", str(Q),
          "--csv", os.path.join(work, "out_small_pandas.csv")])
dt = time.perf_counter() - t0
os.environ["RSS_CSV_FASTPATH"] = "1"
cli_main(["--key-file", os.path.join(ROOT, "tests", "golden", "example_input", "hash_key.txt"),
          "--ips-file", small, "--htable-size", str(H), "--num-queues", str(Q),
          "--csv", os.path.join(work, "out_small_fast.csv")])
same = open(os.path.join(work, "out_small_pandas.csv"), "rb").read() == \
    open(os.path.join(work, "out_small_fast.csv"), "rb").read()
result["csv_pandas_path"] = {"rows": pandas_rows, "wall_s": dt, "rows_per_s": pandas_rows / dt,
                             "fast_path_output_identical": same}
print(json.dumps(result))
