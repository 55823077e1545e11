"""Calibrate the bench's CPU baseline against the REFERENCE itself.

The reference cannot travel to the GPU box, so ``bench.py``'s ``cpu_baseline`` times this
build's pure-Python restatement of its per-tuple path (``oracle.compute_hash_port``) on the
box's host cores.  This script runs in the build container only: on the first N tuples of
the bench stream, as dotted-quad strings and integer ports (exactly the rows
``bench.cpu_baseline`` feeds the port), it times the reference's
``Toeplitz(key).compute_hash`` (``toeplitz.py:46-69``) and the port on ONE core of this
host, checks that both give the same hash for every row, and writes the rate ratio to
``cpu_calibration.json`` -- data only.  ``bench.py`` reports
``cpu_baseline.reference_equivalent`` = the port's rate on the GPU box / that ratio.

Run:  PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_cpu_calibration.py [N]
"""
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main(n):
    sys.path.insert(0, HERE)
    import make_golden  # the shim and the tree guard of the fixture generator
    Toeplitz, _, _ = make_golden.import_reference()
    sys.path.insert(0, ROOT)
    from oracle.oracle import compute_hash_port, generate_np
    import bench
    key = [int(x, 16) for x in bench.EXAMPLE_KEY.split(":")]
    tup = generate_np(bench.SEED, 0, n)
    dotted = make_golden.ip_str
    rows = [(dotted(int(s)), dotted(int(d)), int(p) >> 16, int(p) & 0xFFFF) for s, d, p in tup]
    ref = Toeplitz(key)
    best = {}
    for name, fn in (("reference", lambda r: ref.compute_hash(*r)),
                     ("port", lambda r: compute_hash_port(key, *r))):
        out, times = None, []
        for _ in range(3):
            t0 = time.perf_counter()
            out = [fn(r) for r in rows]
            times.append(time.perf_counter() - t0)
        best[name] = (min(times), out)
    assert best["reference"][1] == best["port"][1], "port and reference hashes differ"
    ref_rate = n / best["reference"][0]
    port_rate = n / best["port"][0]
    rec = {"tuples": n, "sample": "first %d tuples of the bench stream (seed 0x%X), dotted-quad "
                                  "strings + integer ports, key example_input/hash_key.txt" % (n, bench.SEED),
           "cores": 1, "reference_tuples_per_s": ref_rate, "port_tuples_per_s": port_rate,
           "port_over_reference": port_rate / ref_rate, "hashes_equal": True,
           "timing": "best of 3 passes each, one process, perf_counter",
           "host": {"python": platform.python_version(), "machine": platform.machine(),
                    "processor": platform.processor() or None},
           "reference_call": "rss_simulator.toeplitz.Toeplitz(key).compute_hash(src_ip, dst_ip, "
                             "src_port, dst_port) (toeplitz.py:46-69)",
           "port_call": "oracle.oracle.compute_hash_port (the bench's cpu_baseline)"}
    with open(os.path.join(HERE, "cpu_calibration.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
