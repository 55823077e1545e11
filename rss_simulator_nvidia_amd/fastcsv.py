"""CLI fast path for ``--csv`` runs.

canonical CSV file --rss_csv_hash_file (text streamed up through pinned staging,
newline index, parse, hash, format on the device, rows streamed down into the output
file)--> statistics file, byte-identical to the reference's
``write_statistics`` output (``rss_simulator/simulator.py:100-116``).  When the device
text path declines (RSS_CSV_DEVICE=0) the host path runs: native parse
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
    key = _native.prepare_key(hash_key, fields)
    ctx = _native.default_context()
    if device_text_enabled():
        done = ctx.csv_hash_file(key, ips_file, output, htable, nqueues, reta=reta)
        if done is not None:
            if timings is not None:
                timings.update(device_file=time.perf_counter() - t[0], rows=done[1],
                               bytes_in=os.path.getsize(ips_file),
                               bytes_out=os.path.getsize(output), path="device")
            print("Wrote statistics to {csv}.".format(csv=output))
            return True
    t = [time.perf_counter()]
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return False
    t.append(time.perf_counter())
    parsed = _native.csv_parse(data, threads)
    if parsed is None:
        return False
    tuples, layout = parsed
    t.append(time.perf_counter())
    h, q, c = ctx.hash(key, tuples, htable, nqueues, reta=reta)
    t.append(time.perf_counter())
    out = _native.csv_format(tuples, h, q, c, layout, threads)
    t.append(time.perf_counter())
    try:
        out.tofile(output)
    except OSError:
        return False  # the pandas path raises the reference's error for this path
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
    key = _native.prepare_key(hash_key, fields)
    ctx = _native.default_context()
    if device_text_enabled():
        done = ctx.csv_hash_file(key, ips_file, None, htable, nqueues, reta=reta)
        if done is not None:
            return done[0]
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return None
    parsed = _native.csv_parse(data, threads)
    if parsed is None:
        return None
    _, _, counts = ctx.hash(key, parsed[0], htable, nqueues, want_hash=False, want_queue=False,
                            reta=reta)
    return counts


def run_csv6(hash_key, ips_file, htable, nqueues, output, threads=0, timings=None,
             fields=_native.FIELDS_ALL, reta=None):
    """``--ipv6 --csv`` for a canonical IPv6 file: the whole job on the device
    (rss_csv6_hash_file: newline index, parse, rss_hash6_device, rows copied from the
    input text), or with RSS_CSV_DEVICE=0 native parse (rss_csv_parse6) -> the IPv6
    kernel (rss_hash6_host) -> native format (rss_csv_format6).  False if the file needs
    the pandas path."""
    t = [time.perf_counter()]
    key6 = _native.prepare_key6(hash_key, fields)
    ctx = _native.default_context()
    if device_text_enabled():
        done = ctx.csv_hash_file(key6, ips_file, output, htable, nqueues, reta=reta)
        if done is not None:
            if timings is not None:
                timings.update(device_file=time.perf_counter() - t[0], rows=done[1],
                               bytes_in=os.path.getsize(ips_file),
                               bytes_out=os.path.getsize(output), path="device6")
            print("Wrote statistics to {csv}.".format(csv=output))
            return True
    t = [time.perf_counter()]
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return False
    t.append(time.perf_counter())
    parsed = _native.csv_parse6(data, threads)
    if parsed is None:
        return False
    tuples, spans, layout = parsed
    t.append(time.perf_counter())
    h, q, c = ctx.hash6(key6, tuples, htable, nqueues, reta=reta)
    t.append(time.perf_counter())
    out = _native.csv_format6(data, spans, h, q, c, layout, threads)
    t.append(time.perf_counter())
    try:
        out.tofile(output)
    except OSError:
        return False  # the pandas path raises the reference's error for this path
    t.append(time.perf_counter())
    if timings is not None:
        for name, a, b in zip(("read", "parse", "gpu", "format", "write"), t, t[1:]):
            timings[name] = b - a
        timings.update(rows=len(tuples), bytes_in=len(data), bytes_out=len(out), path="host6")
    print("Wrote statistics to {csv}.".format(csv=output))
    return True


def run_counts6(hash_key, ips_file, htable, nqueues, threads=0, fields=_native.FIELDS_ALL,
                reta=None):
    """Per-queue counts of a canonical IPv6 file; None if it needs the pandas path."""
    key6 = _native.prepare_key6(hash_key, fields)
    ctx = _native.default_context()
    if device_text_enabled():
        done = ctx.csv_hash_file(key6, ips_file, None, htable, nqueues, reta=reta)
        if done is not None:
            return done[0]
    try:
        data = np.fromfile(ips_file, dtype=np.uint8)
    except (OSError, ValueError):
        return None
    parsed = _native.csv_parse6(data, threads)
    if parsed is None:
        return None
    _, _, counts = ctx.hash6(key6, parsed[0], htable, nqueues, want_hash=False,
                             want_queue=False, reta=reta)
    return counts
