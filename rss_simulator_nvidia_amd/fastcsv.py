"""CLI fast path for ``--csv`` runs.

canonical CSV file --rss_csv_hash_text (text up, newline index, parse, hash, format
on the device, file image down)--> statistics file, byte-identical to the reference's
``write_statistics`` output (``rss_simulator/simulator.py:100-116``).  When the device
text path declines (body of 4 GiB or more) the host path runs: native parse
(rss_csv_parse) --> rss_hash_host (pinned, chunked H2D -> kernel -> D2H) --> native
format (rss_csv_format).

Files outside the canonical form (see ``include/rss_toeplitz.h``) return False and
the CLI takes the pandas path of :class:`~rss_simulator_nvidia_amd.simulator.Simulator`,
which reproduces the reference's parsing rules and errors.  ``RSS_CSV_FASTPATH=0``
disables this module (the GPU computes the hashes either way); ``RSS_CSV_DEVICE=0``
keeps the text work on the host.
"""
import os
import time

import numpy as np

from rss_simulator_nvidia_amd import _native


def enabled():
    return os.environ.get("RSS_CSV_FASTPATH", "1") != "0"


def device_text_enabled():
    return os.environ.get("RSS_CSV_DEVICE", "1") != "0"


def run_csv(hash_key, ips_file, htable, nqueues, output, threads=0, timings=None,
            fields=_native.FIELDS_ALL, reta=None):
    """Process ``ips_file`` into ``output``; False if the file needs the pandas path."""
    t = [time.perf_counter()]
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return False
    t.append(time.perf_counter())
    key = _native.prepare_key(hash_key, fields)
    ctx = _native.default_context()
    done = ctx.csv_hash_text(key, data, htable, nqueues, reta=reta) \
        if device_text_enabled() else None
    if done is not None:
        image, _, n = done
        t.append(time.perf_counter())
        image.tofile(output)
        t.append(time.perf_counter())
        if timings is not None:
            for name, a, b in zip(("read", "device", "write"), t, t[1:]):
                timings[name] = b - a
            timings.update(rows=n, bytes_in=len(data), bytes_out=len(image), path="device")
        print("Wrote statistics to {csv}.".format(csv=output))
        return True
    parsed = _native.csv_parse(data, threads)
    if parsed is None:
        return False
    tuples, layout = parsed
    t.append(time.perf_counter())
    h, q, c = ctx.hash(key, tuples, htable, nqueues, reta=reta)
    t.append(time.perf_counter())
    out = _native.csv_format(tuples, h, q, c, layout, threads)
    t.append(time.perf_counter())
    out.tofile(output)
    t.append(time.perf_counter())
    if timings is not None:
        for name, a, b in zip(("read", "parse", "gpu", "format", "write"), t, t[1:]):
            timings[name] = b - a
        timings.update(rows=len(tuples), bytes_in=len(data), bytes_out=len(out), path="host")
    print("Wrote statistics to {csv}.".format(csv=output))
    return True


def run_counts(hash_key, ips_file, htable, nqueues, threads=0, fields=_native.FIELDS_ALL,
               reta=None):
    """Per-queue counts of a canonical file via the counts-only kernel (12 B/tuple);
    None if the file needs the pandas path."""
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return None
    key = _native.prepare_key(hash_key, fields)
    ctx = _native.default_context()
    if device_text_enabled():
        done = ctx.csv_hash_text(key, data, htable, nqueues, reta=reta, counts_only=True)
        if done is not None:
            return done[1]
    parsed = _native.csv_parse(data, threads)
    if parsed is None:
        return None
    _, _, counts = ctx.hash(key, parsed[0], htable, nqueues, want_hash=False, want_queue=False,
                            reta=reta)
    return counts
