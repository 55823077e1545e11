"""IPv6 CSV -> CSV rates (tool, not product): the device text path (rss_csv6_hash_file)
and the host text path (RSS_CSV_DEVICE=0: rss_csv_parse6 -> IPv6 kernel ->
rss_csv_format6) on the big file -- outputs must be identical -- and the pandas path
(RSS_CSV_FASTPATH=0) on a smaller file.  Prints one JSON object.
usage: python tools/e2e_ipv6_bench.py [ROWS] [PANDAS_ROWS] [WORKDIR]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native, fastcsv  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
pandas_rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 17
work = sys.argv[3] if len(sys.argv) > 3 else "/tmp/rss_e2e6"
os.makedirs(work, exist_ok=True)


def write_file(path, n, seed):
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 1 << 16, (n, 16))
    g[:, 2:6] = 0  # a zero run: every address takes the '::' form for its groups 2..5
    p = rng.integers(0, 1 << 16, (n, 2))
    with open(path, "w") as f:
        f.write("src_ip,dst_ip,src_port,dst_port\n")
        for i in range(n):
            a, b = g[i, :8], g[i, 8:]
            f.write("%x:%x::%x:%x,%x:%x:%x:%x:%x:%x:%x:%x,%d,%d\n" % (
                a[0], a[1], a[6], a[7], *b, p[i, 0], p[i, 1]))


big, small = os.path.join(work, "big6.csv"), os.path.join(work, "small6.csv")
t0 = time.perf_counter()
write_file(big, rows, 1)
write_file(small, pandas_rows, 2)
gen_s = time.perf_counter() - t0
key = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
H, Q = 128, 24
result = {"rows": rows, "htable": H, "queues": Q, "generate_s": gen_s}
_native.default_context()
outputs = {}
for dev, name in (("1", "csv6_device"), ("0", "csv6_fastpath")):
    os.environ["RSS_CSV_DEVICE"] = dev
    runs = []
    out = os.path.join(work, "out_big6_%s.csv" % dev)
    for _ in range(3):
        if os.path.exists(out):
            os.unlink(out)
        t = {}
        t0 = time.perf_counter()
        assert fastcsv.run_csv6(key, big, H, Q, out, timings=t)
        runs.append((time.perf_counter() - t0, t))
    wall, t = min(runs[1:], key=lambda r: r[0])
    result[name] = {"path": t["path"], "wall_s": wall, "rows_per_s": rows / wall,
                    "first_call_wall_s": runs[0][0],
                    "stages_s": {k: v for k, v in t.items()
                                 if k in ("read", "parse", "gpu", "format", "write")},
                    "bytes_in": t["bytes_in"], "bytes_out": t["bytes_out"]}
    with open(out, "rb") as f:
        outputs[dev] = hash(f.read())
os.environ["RSS_CSV_DEVICE"] = "1"
result["big_outputs_identical"] = outputs["1"] == outputs["0"]
assert result["big_outputs_identical"]
from rss_simulator_nvidia_amd.main import main as cli_main  # noqa: E402
outs = {}
for fast in ("1", "0"):
    os.environ["RSS_CSV_FASTPATH"] = fast
    out = os.path.join(work, "out_small6_%s.csv" % fast)
    t0 = time.perf_counter()
    cli_main(["--key-file", os.path.join(ROOT, "tests", "golden", "example_input", "hash_key.txt"),
              "--ips-file", small, "--ipv6", "--htable-size", str(H), "--num-queues", str(Q),
              "--csv", out])
    dt = time.perf_counter() - t0
    outs[fast] = open(out, "rb").read()
    result["cli_small_" + ("fast" if fast == "1" else "pandas")] = {
        "rows": pandas_rows, "wall_s": dt, "rows_per_s": pandas_rows / dt}
result["small_outputs_identical"] = outs["1"] == outs["0"]
assert result["small_outputs_identical"]
print(json.dumps(result))
