"""Host-memory IPv6 batches against IPv4 ones (tool, not product): seconds per call of
``HostContext.hash6`` (``rss_hash6_host``) and ``HostContext.hash`` (``rss_hash_host``) on
pageable numpy tuples at several batch sizes, best of a few calls after a warm-up call.
Prints one JSON line.

usage: python tools/host6_probe.py [LIBRARY]   (another build of librss_toeplitz.so, for A/B)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bench import EXAMPLE_KEY  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402


def best(fn, reps):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    if len(sys.argv) > 1:
        _native.LIB_PATH = sys.argv[1]  # read by _native.load() on first use
    key_bytes = [int(x, 16) for x in EXAMPLE_KEY.split(":")]
    k4, k6 = _native.prepare_key(key_bytes), _native.prepare_key6(key_bytes)
    ctx = _native.HostContext(0)
    rng = np.random.default_rng(3)
    out = {}
    for n in (1, 1024, 1 << 16, 1 << 20, 1 << 22, 1 << 24):
        t6 = rng.integers(0, 2**32, (n, 9), dtype=np.uint32)
        t4 = np.ascontiguousarray(t6[:, :3])
        reps = 200 if n <= 1024 else (20 if n <= 1 << 20 else 8)
        s6 = best(lambda: ctx.hash6(k6, t6, 128, 24), reps)
        s4 = best(lambda: ctx.hash(k4, t4, 128, 24), reps)
        out[str(n)] = {"ipv6_s": s6, "ipv4_s": s4, "ipv6_tuples_per_s": n / s6,
                       "ipv4_tuples_per_s": n / s4, "ipv6_GBps_in": n * 36 / s6 / 1e9}
        print("n=%d ipv6 %.3g s ipv4 %.3g s" % (n, s6, s4), file=sys.stderr, flush=True)
    # the reference-compatible per-row calls (one tuple each) on the default context
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    tz = Toeplitz(key_bytes)
    w6 = rng.integers(0, 2**32, (500, 9), dtype=np.uint32)
    w4 = np.ascontiguousarray(w6[:, :3])
    for name, fn in (("compute_queues6", lambda i: tz.compute_queues6(w6[i:i + 1], 128, 24)),
                     ("compute_queues", lambda i: tz.compute_queues(w4[i:i + 1], 128, 24)),
                     ("default_ctx_hash6", lambda i: _native.default_context().hash6(
                         k6, w6[i:i + 1], 128, 24)),
                     ("fresh_ctx_hash6", lambda i: ctx.hash6(k6, w6[i:i + 1], 128, 24))):
        fn(0)
        t0 = time.perf_counter()
        for i in range(len(w6)):
            fn(i)
        out[name + "_us_per_call"] = (time.perf_counter() - t0) / len(w6) * 1e6
        print("%s %.1f us per call" % (name, out[name + "_us_per_call"]), file=sys.stderr,
              flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
