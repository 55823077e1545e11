"""The reference API end to end on one GPU (tool, not product): ``Simulator`` on an N-row
canonical CSV (``tools/gen_csv.c``) -- ``load_ips_from_csv`` (pandas), ``calc_hash``,
``calc_queue_number``, ``write_statistics`` -- each step timed, and the written file compared
with the CLI's device CSV path on the same input (the two must be byte-identical).

usage: python tools/simulator_e2e.py [N]        (prints one JSON line)"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rss_simulator_nvidia_amd import _native  # noqa: E402
from rss_simulator_nvidia_amd.hash_key import HashKey  # noqa: E402
from rss_simulator_nvidia_amd.simulator import Simulator  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    key = HashKey.from_file(os.path.join(ROOT, "tests", "golden", "example_input", "hash_key.txt"))
    with tempfile.TemporaryDirectory() as tmp:
        gen = os.path.join(tmp, "gen_csv")
        subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(ROOT, "tools", "gen_csv.c")], check=True)
        src = os.path.join(tmp, "in.csv")
        subprocess.run([gen, str(n), "7", src], check=True)
        _native.default_context()  # context creation is not a step of the flow
        t = {}
        t0 = time.perf_counter()
        sim = Simulator(key, 128, 24)
        sim.load_ips_from_csv(src)
        t["load_ips_from_csv"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        sim.calc_hash()
        t["calc_hash"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        sim.calc_queue_number()
        t["calc_queue_number"] = time.perf_counter() - t0
        out_api = os.path.join(tmp, "api.csv")
        t0 = time.perf_counter()
        sim.write_statistics(out_api)
        t["write_statistics"] = time.perf_counter() - t0
        out_cli = os.path.join(tmp, "cli.csv")
        t0 = time.perf_counter()
        counts, rows = _native.default_context().csv_hash_file(_native.prepare_key(key), src,
                                                               out_cli, 128, 24)
        t["device_csv_path_file_to_file"] = time.perf_counter() - t0
        same = open(out_api, "rb").read() == open(out_cli, "rb").read()
    total = sum(v for k, v in t.items() if k != "device_csv_path_file_to_file")
    print(json.dumps({"rows": n, "seconds": {k: round(v, 4) for k, v in t.items()},
                      "api_total_s": round(total, 4), "api_rows_per_s": n / total,
                      "device_csv_rows_per_s": n / t["device_csv_path_file_to_file"],
                      "api_file_equals_device_csv_file": same}), flush=True)


if __name__ == "__main__":
    main()
