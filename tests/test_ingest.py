"""Address-column ingest (``ingest.ip_column``) against the literal restatement of the
reference's ``__ip_to_int`` + byte masks (``ingest.ip_to_u32``, ``toeplitz.py:100-111`` /
``:127-137``) cell by cell: the native quad parser (``rss_parse_dotted``) must take exactly
the plain ``d.d.d.d`` cells and give their reference values, and every other cell -- which the
reference may still accept (whitespace, extra octets, octets > 255, signs, underscores,
non-ASCII digits) or reject -- must come out as the literal path gives it, exceptions
included.  CPU only (the library loads without a GPU)."""
import numpy as np
import pandas as pd
import pytest

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.ingest import ip_column, ip_to_u32, pack_frame

ACCEPTED = ["1.2.3.4", "0.0.0.0", "255.255.255.255", "999.999.999.999", "010.001.0.9",
            "1.2.3.4.5", "1.2.3.4.x", " 1.2.3.4", "1.2.3.4 ", "1.2.3.4\r", "+1.2.3.4",
            "1_0.2.3.4", "１.2.3.4", "1.2.3.0004", "4294.1.1.1", "1.2.3.-4", "-1.2.3.4"]
REJECTED = ["1.2.3", "", "a.b.c.d", "1..2.3", "1.2.3.", ".1.2.3", "1.2.3.4/24", "1,2,3,4",
            "1 .2.3.4x"]


def _literal(cell):
    try:
        return ip_to_u32(cell), None
    except Exception as err:  # the type the reference raises
        return None, type(err)


def test_native_parser_takes_exactly_the_plain_quads():
    cells = ACCEPTED + REJECTED + ["12.34.56.78", "1.22.333.4", "1234.1.1.1", "1.2.3.4\n5"]
    ok, val = _native.parse_dotted(["1.2.3.4", "9.8.7.6"])
    assert ok.tolist() == [True, True] and val.tolist() == [0x01020304, 0x09080706]
    assert _native.parse_dotted(["1.2.3.4\n5", "1.2.3.4"]) is None  # a cell holding '\n'
    got = _native.parse_dotted([c for c in cells if "\n" not in c])
    assert got is not None
    import re
    plain = re.compile(r"[0-9]{1,3}\.[0-9]{1,3}\.[0-9]{1,3}\.[0-9]{1,3}")
    for c, o, v in zip([c for c in cells if "\n" not in c], *got):
        assert bool(o) == bool(plain.fullmatch(c)), c
        if o:
            assert int(v) == ip_to_u32(c), c


def test_random_columns_equal_the_literal_path():
    rng = np.random.default_rng(12)
    pool = ACCEPTED + ["%d.%d.%d.%d" % tuple(rng.integers(0, 1000, 4)) for _ in range(200)]
    for trial in range(20):
        cells = [pool[i] for i in rng.integers(0, len(pool), 5000)]
        got = ip_column(pd.Series(cells, dtype=object))
        want = np.array([ip_to_u32(c) for c in cells], dtype=np.uint32)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("bad", REJECTED + [None, 1.5, float("nan"), b"1.2.3.4", 16909060])
def test_a_rejected_cell_raises_what_the_literal_path_raises(bad):
    cells = ["1.2.3.4"] * 10 + [bad] + ["5.6.7.8"] * 5
    _, err = _literal(bad)
    if err is None:  # (an int cell: the reference raises on .split too)
        pytest.skip("accepted by the literal path")
    with pytest.raises(err):
        ip_column(pd.Series(cells, dtype=object))


def test_string_dtype_and_ports_through_pack_frame():
    df = pd.DataFrame({"src_ip": pd.Series(["1.2.3.4", " 10.0.0.1"], dtype="string"),
                       "dst_ip": ["255.255.255.255", "1.2.3.4.5"],
                       "src_port": [65536 + 7, -1], "dst_port": [80, 443]})
    t = pack_frame(df)
    assert t["sip"].tolist() == [0x01020304, 0x0A000001]
    assert t["dip"].tolist() == [0xFFFFFFFF, 0x01020304]
    assert t["ports"].tolist() == [(7 << 16) | 80, (0xFFFF << 16) | 443]


def test_million_row_column_is_fast():
    import time
    rng = np.random.default_rng(3)
    v = rng.integers(0, 2**32, 1_000_000, dtype=np.uint64).tolist()
    cells = ["%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255) for x in v]
    s = pd.Series(cells, dtype=object)
    t0 = time.perf_counter()
    got = ip_column(s)
    dt = time.perf_counter() - t0
    np.testing.assert_array_equal(got, np.array(v, dtype=np.uint64).astype(np.uint32))
    assert dt < 2.0, dt  # native pass: ~0.1 s here; pandas' regex + split took ~4 s


def _v6_forms(rng, k):
    import ipaddress
    out = []
    for _ in range(k):
        hi = int(rng.integers(0, 2**63)) << 1 | int(rng.integers(0, 2))
        lo = int(rng.integers(0, 2**16)) if rng.random() < 0.4 else int(rng.integers(0, 2**63))
        a = ipaddress.IPv6Address((hi << 64 | lo) if rng.random() < 0.7 else lo)
        form = int(rng.integers(0, 4))
        out.append(str(a) if form == 0 else a.exploded if form == 1 else
                   str(a).upper() if form == 2 else a.exploded.replace(":0000", ":0"))
    return out


def test_ipv6_columns_equal_ipaddress():
    from rss_simulator_nvidia_amd.ingest import ipv6_column, ipv6_words
    rng = np.random.default_rng(6)
    odd = ["::", "::1", "1::", "::ffff:1.2.3.4", "fe80::1%eth0", " ::1 ", "::1\r", "0:0:0:0:0:0:0:0",
           "FFFF:ffff:FfFf:ffff:ffff:ffff:ffff:ffff"]
    cells = _v6_forms(rng, 3000) + odd
    rng.shuffle(cells)
    got = ipv6_column(pd.Series(cells, dtype=object))
    want = np.array([ipv6_words(c) for c in cells], dtype=np.uint32)
    np.testing.assert_array_equal(got, want)
    ok, _ = _native.parse_ipv6(["::ffff:1.2.3.4", "::1", " ::1", "1:2:3:4:5:6:7:8:9"])
    assert ok.tolist() == [False, True, False, False]  # the odd forms take ipaddress


@pytest.mark.parametrize("bad", [":::", "1:2:3:4:5:6:7:8:9", "12345::", "g::1", "1.2.3.4", ""])
def test_ipv6_bad_cells_raise_like_ipaddress(bad):
    from rss_simulator_nvidia_amd.ingest import ipv6_column
    with pytest.raises(ValueError):
        ipv6_column(pd.Series(["::1"] * 5 + [bad], dtype=object))


# ---------------------------------------------------------------- write_statistics ----
def _pandas_statistics(df, counts, path):
    """write_statistics' bytes the reference way (simulator.py:100-116)."""
    with open(path, "w") as f:
        f.write("queue_number,counts\n")
        for q in np.flatnonzero(counts):
            f.write("{},{}\n".format(int(q), int(counts[q])))
    df.to_csv(path, mode="a", index=False)
    with open(path, "rb") as f:
        return f.read()


def _simulator_with(df, counts):
    from rss_simulator_nvidia_amd.simulator import Simulator
    sim = Simulator([0] * 40, 128, 24)
    sim.load_frame(df)
    sim._Simulator__counts = counts  # (what calc_hash leaves)
    return sim


def _frame(rng, n, order):
    v = rng.integers(0, 2**32, (2, n), dtype=np.uint64)
    quad = lambda u: ["%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255)  # noqa: E731
                      for x in u.tolist()]
    cols = {"src_ip": quad(v[0]), "dst_ip": quad(v[1]),
            "src_port": rng.integers(0, 65536, n), "dst_port": rng.integers(0, 65536, n)}
    df = pd.DataFrame({c: cols[c] for c in order})
    df["hash_result"] = rng.integers(0, 2**32, n).astype(np.int64)
    df["queue_number"] = (df["hash_result"] % 128 % 24).astype(np.int64)
    counts = np.bincount(df["queue_number"], minlength=24).astype(np.uint64)
    return df, counts


@pytest.mark.parametrize("order", [["src_ip", "dst_ip", "src_port", "dst_port"],
                                   ["dst_port", "src_ip", "src_port", "dst_ip"]])
def test_write_statistics_native_bytes_equal_pandas(tmp_path, capsys, order):
    """A canonical frame takes the native formatter: the file is byte for byte what the
    reference's to_csv writes, the stdout line unchanged."""
    df, counts = _frame(np.random.default_rng(len(order[0])), 50000, order)
    want = _pandas_statistics(df, counts, tmp_path / "ref.csv")
    sim = _simulator_with(df, counts)
    calls = []
    orig = _native.csv_format
    try:
        _native.csv_format = lambda *a, **k: calls.append(1) or orig(*a, **k)
        sim.write_statistics(str(tmp_path / "out.csv"))
    finally:
        _native.csv_format = orig
    assert calls, "the canonical frame did not take the native formatter"
    assert (tmp_path / "out.csv").read_bytes() == want
    assert capsys.readouterr().out == "Wrote statistics to %s.\n" % (tmp_path / "out.csv")


@pytest.mark.parametrize("spoil", ["leading_zero", "octet_256", "extra_column", "no_queue",
                                   "negative_port", "float_port", "space"])
def test_write_statistics_non_canonical_frames_take_pandas(tmp_path, capsys, spoil):
    df, counts = _frame(np.random.default_rng(3), 2000, ["src_ip", "dst_ip", "src_port",
                                                         "dst_port"])
    if spoil == "leading_zero":
        df.loc[7, "src_ip"] = "01.2.3.4"
    elif spoil == "octet_256":
        df.loc[7, "dst_ip"] = "1.2.3.256"
    elif spoil == "extra_column":
        df["note"] = "x"
    elif spoil == "no_queue":
        df = df.drop(columns=["queue_number"])
    elif spoil == "negative_port":
        df.loc[7, "src_port"] = -1
    elif spoil == "float_port":
        df["dst_port"] = df["dst_port"].astype(float)
    else:
        df.loc[7, "src_ip"] = " 1.2.3.4"
    want = _pandas_statistics(df, counts, tmp_path / "ref.csv")
    _simulator_with(df, counts).write_statistics(str(tmp_path / "out.csv"))
    assert (tmp_path / "out.csv").read_bytes() == want


# ---------------------------------------------------------------- load_ips_from_csv ----
@pytest.mark.parametrize("variant", ["plain", "reordered", "crlf", "blank_lines", "no_final_newline"])
def test_canonical_csv_frame_equals_pandas(tmp_path, variant):
    """load_ips_from_csv of a canonical file (pyarrow reader) builds exactly pd.read_csv's
    DataFrame: values, dtypes, column order."""
    from rss_simulator_nvidia_amd.simulator import Simulator
    rng = np.random.default_rng(len(variant))
    df, _ = _frame(rng, 3000, ["dst_port", "src_ip", "dst_ip", "src_port"] if variant == "reordered"
                   else ["src_ip", "dst_ip", "src_port", "dst_port"])
    text = df.drop(columns=["hash_result", "queue_number"]).to_csv(index=False)
    if variant == "crlf":
        text = text.replace("\n", "\r\n")
    elif variant == "blank_lines":
        lines = text.split("\n")
        text = "\n".join(lines[:10] + [""] + lines[10:20] + ["", ""] + lines[20:])
    elif variant == "no_final_newline":
        text = text.rstrip("\n")
    path = tmp_path / "in.csv"
    path.write_bytes(text.encode())
    want = pd.read_csv(path)
    sim = Simulator([0] * 40, 128, 24)
    calls = []
    import rss_simulator_nvidia_amd.simulator as simmod
    orig = simmod._read_canonical_csv
    simmod._read_canonical_csv = lambda p: calls.append(1) or orig(p)
    try:
        sim.load_ips_from_csv(str(path))
    finally:
        simmod._read_canonical_csv = orig
    got = sim.data_frame
    assert calls and orig(str(path)) is not None, "the canonical file did not take pyarrow"
    assert list(got.columns) == list(want.columns)
    assert got.dtypes.tolist() == want.dtypes.tolist()
    assert got.equals(want)


def test_non_canonical_csv_keeps_pandas(tmp_path):
    from rss_simulator_nvidia_amd.simulator import _read_canonical_csv
    path = tmp_path / "in.csv"
    path.write_text("src_ip,dst_ip,src_port,dst_port\n01.2.3.4,1.2.3.4,1,2\n")
    assert _read_canonical_csv(str(path)) is None  # leading zero: not canonical
    path.write_text("src_ip,dst_ip,src_port,dst_port,extra\n1.2.3.4,1.2.3.4,1,2,x\n")
    assert _read_canonical_csv(str(path)) is None
    assert _read_canonical_csv(str(tmp_path / "missing.csv")) is None
