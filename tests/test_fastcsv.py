"""Native CSV fast path (host code, no GPU): parse == pandas ingest, format == the
reference's write_statistics bytes, and every non-canonical input is refused."""
import os
import random

import numpy as np
import pandas as pd
import pytest

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.ingest import pack_frame


def parse(text, threads=0):
    return _native.csv_parse(np.frombuffer(text.encode("latin-1"), dtype=np.uint8), threads)


def reference_stats_bytes(df, hashes, htable, nqueues, tmp_path):
    """What simulator.py:96-115 writes, produced with pandas (df gets the new columns)."""
    df = df.copy()
    df["hash_result"] = hashes.astype(np.int64)
    df["queue_number"] = df.hash_result % htable % nqueues
    path = str(tmp_path / "ref_stats.csv")
    df["queue_number"].value_counts().sort_index().rename_axis("queue_number") \
        .to_frame("counts").to_csv(path)
    df.to_csv(path, mode="a", index=False)
    return open(path, "rb").read()


def native_stats_bytes(text, key, htable, nqueues, oracle_lib, threads=0):
    tuples, layout = parse(text, threads)
    arr = np.stack([tuples["sip"], tuples["dip"], tuples["ports"]], axis=1)
    h, q, c = oracle_lib.run(key, arr, htable, nqueues, threads=2)
    return _native.csv_format(tuples, h, q, c, layout, threads).tobytes(), tuples, h


def test_example_matches_pandas_and_golden(golden_dir, example_key, oracle_lib, tmp_path):
    path = os.path.join(golden_dir, "example_input", "ips.csv")
    text = open(path, "rb").read().decode("latin-1")
    tuples, layout = parse(text)
    np.testing.assert_array_equal(tuples, pack_frame(pd.read_csv(path)))
    assert list(layout.field_column) == [0, 1, 2, 3]
    for name in sorted(os.listdir(os.path.join(golden_dir, "example"))):
        if not name.endswith(".csv"):
            continue
        h, q = (int(x[1:]) for x in name[4:-4].split("_"))
        got, _, _ = native_stats_bytes(text, example_key, h, q, oracle_lib)
        assert got == open(os.path.join(golden_dir, "example", name), "rb").read(), name


def _random_canonical(rng, n, order, crlf, blank_lines, trailing_nl):
    nl = "\r\n" if crlf else "\n"
    names = ["src_ip", "dst_ip", "src_port", "dst_port"]
    lines = [",".join(names[c] for c in order)]
    for _ in range(n):
        vals = ["%d.%d.%d.%d" % tuple(rng.randrange(256) for _ in range(4)),
                "%d.%d.%d.%d" % tuple(rng.randrange(256) for _ in range(4)),
                str(rng.choice([0, 1, 9, 10, 80, 443, 65535, rng.randrange(65536)])),
                str(rng.randrange(65536))]
        lines.append(",".join(vals[c] for c in order))
        if blank_lines and rng.random() < 0.05:
            lines.append("")
    return nl.join(lines) + (nl if trailing_nl else "")


@pytest.mark.parametrize("seed", range(8))
def test_random_canonical_round_trip(seed, example_key, oracle_lib, tmp_path):
    rng = random.Random(seed)
    order = list(range(4))
    rng.shuffle(order)
    text = _random_canonical(rng, rng.choice([1, 7, 500, 3000]), order, crlf=seed % 2 == 1,
                             blank_lines=seed % 3 == 0, trailing_nl=seed % 4 != 2)
    path = tmp_path / "in.csv"
    path.write_bytes(text.encode())
    df = pd.read_csv(path)
    htable, nqueues = rng.choice([(128, 24), (100, 7), (512, 64), (1, 1)])
    got, tuples, h = native_stats_bytes(text, example_key, htable, nqueues, oracle_lib)
    np.testing.assert_array_equal(tuples, pack_frame(df))
    assert got == reference_stats_bytes(df, h, htable, nqueues, tmp_path)


def test_threads_do_not_change_output(example_key, oracle_lib):
    rng = random.Random(99)
    text = _random_canonical(rng, 300000, [2, 0, 3, 1], crlf=True, blank_lines=True,
                             trailing_nl=True)
    a = native_stats_bytes(text, example_key, 128, 24, oracle_lib, threads=1)[0]
    b = native_stats_bytes(text, example_key, 128, 24, oracle_lib, threads=8)[0]
    c = native_stats_bytes(text, example_key, 128, 24, oracle_lib, threads=16)[0]
    assert a == b == c


HEADER = "src_ip,dst_ip,src_port,dst_port\n"
NOT_CANONICAL = [
    HEADER,                                       # no rows (pandas path raises)
    "",                                           # empty file
    HEADER + "3.3.3.300,1.1.1.1,1,1\n",           # octet > 255
    HEADER + "03.3.3.1,1.1.1.1,1,1\n",            # leading zero
    HEADER + "3.3.3.1,1.1.1.1,65536,1\n",         # port > 65535
    HEADER + "3.3.3.1,1.1.1.1,01,1\n",            # leading zero port
    HEADER + "3.3.3.1,1.1.1.1,-1,1\n",            # sign
    HEADER + "3.3.3.1,1.1.1.1,+1,1\n",
    HEADER + " 3.3.3.1,1.1.1.1,1,1\n",            # whitespace
    HEADER + "3.3.3.1,1.1.1.1,1,1 \n",
    HEADER + "3.3.3.1,1.1.1.1,1\t,1\n",
    HEADER + "3.3.3.1.5,1.1.1.1,1,1\n",           # five octets
    HEADER + "3.3.3,1.1.1.1,1,1\n",               # three octets
    HEADER + "3.3.3.1,1.1.1.1,1,1,9\n",           # extra field
    HEADER + "3.3.3.1,1.1.1.1,1\n",               # missing field
    HEADER + "3.3.3.1,1.1.1.1,,1\n",              # empty field
    HEADER + '"3.3.3.1",1.1.1.1,1,1\n',           # quoted
    HEADER + "3.3.3.1,1.1.1.1,1.0,1\n",           # float port
    HEADER + "3.3.3.1,1.1.1.1,1,1\r5.5.5.5,1.1.1.1,1,1\n",  # bare CR = line break in pandas
    HEADER + "   \n3.3.3.1,1.1.1.1,1,1\n",        # whitespace-only line
    "﻿" + HEADER + "3.3.3.1,1.1.1.1,1,1\n",  # BOM
    "src_ip,dst_ip,src_port\n1.1.1.1,1.1.1.1,1\n",              # missing column
    "src_ip,dst_ip,src_port,dst_port,x\n1.1.1.1,1.1.1.1,1,1,a\n",  # extra column
    "src_ip,src_ip,src_port,dst_port\n1.1.1.1,1.1.1.1,1,1\n",      # duplicate column
    "Src_ip,dst_ip,src_port,dst_port\n1.1.1.1,1.1.1.1,1,1\n",      # case
    "\n" + HEADER + "1.1.1.1,1.1.1.1,1,1\n",      # leading blank line
    HEADER + "1.1.1.1,1.1.1.1,1,1\n\xe9\n",       # non-ASCII
]


@pytest.mark.parametrize("text", NOT_CANONICAL)
def test_non_canonical_inputs_are_refused(text):
    assert parse(text.encode("utf-8").decode("latin-1")) is None


def test_golden_edge_inputs_are_refused(golden_dir):
    for name in ["octet_overflow.csv", "whitespace.csv", "ports_wide.csv", "extra_reordered.csv",
                 "missing_col.csv", "header_only.csv", "not_csv.csv"]:
        data = np.fromfile(os.path.join(golden_dir, "edge", name), dtype=np.uint8)
        assert _native.csv_parse(data) is None, name


def test_accepted_mutations_agree_with_pandas(tmp_path):
    # light fuzz: random single-character edits of a canonical file; whenever the fast
    # path accepts the result, pandas must read exactly the same tuples.
    rng = random.Random(5)
    base = _random_canonical(rng, 40, [0, 1, 2, 3], crlf=False, blank_lines=False,
                             trailing_nl=True)
    alphabet = "0123456789.,\n\r -+\"a"
    accepted = 0
    for _ in range(400):
        s = list(base)
        i = rng.randrange(len(HEADER), len(s))
        op = rng.random()
        if op < 0.4:
            s[i] = rng.choice(alphabet)
        elif op < 0.7:
            s.insert(i, rng.choice(alphabet))
        else:
            del s[i]
        text = "".join(s)
        got = parse(text)
        if got is None:
            continue
        accepted += 1
        path = tmp_path / "m.csv"
        path.write_bytes(text.encode())
        np.testing.assert_array_equal(got[0], pack_frame(pd.read_csv(path)))
    assert accepted > 20


class _RoutingCtx:
    """Stands in for the device context: records which fast-path entry points ran."""

    def __init__(self, accept):
        self.accept, self.calls = accept, []

    def csv_hash_file(self, key, in_path, out_path, htable, nqueues, reta=None):
        self.calls.append(("file", out_path))
        if not self.accept:
            return None
        if out_path is not None:
            open(out_path, "wb").write(b"device\n")
        return np.arange(nqueues, dtype=np.uint64), 3

    def hash(self, key, tuples, htable, nqueues, **kwargs):
        self.calls.append(("hash", len(tuples)))
        n = len(tuples)
        return (np.zeros(n, np.uint32), np.zeros(n, np.uint32),
                np.bincount(np.zeros(n, np.int64), minlength=nqueues).astype(np.uint64))


def test_fast_path_routing(monkeypatch, tmp_path, golden_dir, example_key):
    from rss_simulator_nvidia_amd import fastcsv
    src = os.path.join(golden_dir, "example_input", "ips.csv")
    out = str(tmp_path / "o.csv")
    ctx = _RoutingCtx(accept=True)
    monkeypatch.setattr(_native, "default_context", lambda: ctx)
    assert fastcsv.run_csv(example_key, src, 128, 24, out)
    assert ctx.calls == [("file", out)] and open(out, "rb").read() == b"device\n"
    assert fastcsv.run_counts(example_key, src, 128, 24).tolist() == list(range(24))
    ctx = _RoutingCtx(accept=False)  # device declines -> host parse + rss_hash_host
    monkeypatch.setattr(_native, "default_context", lambda: ctx)
    assert fastcsv.run_csv(example_key, src, 128, 24, out)
    assert ctx.calls == [("file", out), ("hash", 100)]
    assert open(out, "rb").read().startswith(b"queue_number,counts\n0,100\n")
    monkeypatch.setenv("RSS_CSV_DEVICE", "0")  # host text path only
    ctx = _RoutingCtx(accept=True)
    monkeypatch.setattr(_native, "default_context", lambda: ctx)
    assert fastcsv.run_csv(example_key, src, 128, 24, out)
    assert ctx.calls == [("hash", 100)]
    assert not fastcsv.run_csv(example_key, str(tmp_path / "missing.csv"), 128, 24, out)
