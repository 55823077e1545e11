"""IPv6 CSV fast path (host code, no GPU): rss_csv_parse6 reads exactly what the pandas
path's ``ipaddress`` parse reads, refuses every text form it does not handle, and
rss_csv_format6 writes the bytes pandas' ``write_statistics`` writes for the same
frame (hashes from the oracle's closed form over the 288 IPv6 windows)."""
import io
import ipaddress

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as o
from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.ingest import pack_frame6


def parse6(text, threads=0):
    return _native.csv_parse6(np.frombuffer(text.encode("latin-1"), dtype=np.uint8), threads)


def random_ipv6_text(rng):
    """One address in a random RFC 4291 text form (no IPv4 suffix, no zone)."""
    groups = [int(x) for x in rng.integers(0, 1 << 16, 8)]
    for k in range(8):  # runs of zero groups make '::' likely
        if rng.random() < 0.3:
            groups[k] = 0
    style = rng.integers(0, 4)
    if style == 0:
        return str(ipaddress.IPv6Address(b"".join(g.to_bytes(2, "big") for g in groups)))
    if style == 1:  # full form, upper case, leading zeros
        return ":".join("%04X" % g for g in groups)
    if style == 2:  # no compression, minimal digits
        return ":".join("%x" % g for g in groups)
    # compress a random (possibly non-zero-preserving) zero run
    a = int(rng.integers(0, 8))
    b = int(rng.integers(a + 1, 9))
    for k in range(a, b):
        groups[k] = 0
    left = ":".join("%x" % g for g in groups[:a])
    right = ":".join("%x" % g for g in groups[b:])
    return left + "::" + right


def words_of(text):
    packed = ipaddress.IPv6Address(text).packed
    return [int.from_bytes(packed[i:i + 4], "big") for i in range(0, 16, 4)]


def test_address_forms_match_ipaddress():
    rng = np.random.default_rng(6)
    addrs = [random_ipv6_text(rng) for _ in range(4000)] + [
        "::", "::1", "1::", "1:2:3:4:5:6:7::", "::2:3:4:5:6:7:8", "0:0:0:0:0:0:0:0",
        "FFFF:ffff:FfFf:0:0:0:0:1", "fe80::abcd:0:0:1"]
    text = "src_ip,dst_ip,src_port,dst_port\n" + "".join(
        "%s,%s,%d,%d\n" % (a, addrs[-1 - i], i % 65536, 65535 - i % 65536)
        for i, a in enumerate(addrs))
    tuples, spans, layout = parse6(text, threads=4)
    assert len(tuples) == len(addrs)
    want_s = np.array([words_of(a) for a in addrs], dtype=np.uint32)
    want_d = np.array([words_of(addrs[-1 - i]) for i in range(len(addrs))], dtype=np.uint32)
    np.testing.assert_array_equal(tuples["sip"], want_s)
    np.testing.assert_array_equal(tuples["dip"], want_d)
    lines = text.encode().split(b"\n")[1:-1]
    raw = text.encode()
    assert [raw[int(b):int(e)] for b, e in spans] == lines


NOT_CANONICAL6 = [
    "::ffff:1.2.3.4", "fe80::1%eth0", ":::", "1:2:3:4:5:6:7:8:9", "12345::", "1::2::3",
    " ::1", "::1 ", '"::1"', "", ":1::", "1:", ":1:2:3:4:5:6:7", "1:2:3:4:5:6:7:8::",
    "::1:2:3:4:5:6:7:8", "g::1", "1.2.3.4", "1:2:3:4:5:6:7", "::-1",
]


@pytest.mark.parametrize("addr", NOT_CANONICAL6)
def test_non_canonical_addresses_are_refused(addr):
    assert parse6("src_ip,dst_ip,src_port,dst_port\n%s,::1,1,2\n" % addr) is None


@pytest.mark.parametrize("row", ["::1,::2,65536,1", "::1,::2,01,2", "::1,::2,-1,2", "::1,::2,1",
                                 "::1,::2,1,2,3", "::1;::2;1;2"])
def test_non_canonical_rows_are_refused(row):
    assert parse6("src_ip,dst_ip,src_port,dst_port\n%s\n" % row) is None


def reference_stats_bytes6(text, hashes, htable, nqueues, tmp_path):
    """What simulator.py:96-115 writes for this frame, produced with pandas."""
    df = pd.read_csv(io.StringIO(text))
    df["hash_result"] = hashes.astype(np.int64)
    df["queue_number"] = df.hash_result % htable % nqueues
    path = str(tmp_path / "ref6.csv")
    df["queue_number"].value_counts().sort_index().rename_axis("queue_number") \
        .to_frame("counts").to_csv(path)
    df.to_csv(path, mode="a", index=False)
    return open(path, "rb").read(), df


@pytest.mark.parametrize("seed", range(6))
def test_random_files_match_pandas_bytes(seed, oracle_lib, tmp_path):
    rng = np.random.default_rng(100 + seed)
    cols = ["src_ip", "dst_ip", "src_port", "dst_port"]
    order = list(rng.permutation(4))
    n = int(rng.integers(1, 3000))
    eol = "\r\n" if seed % 2 else "\n"
    rows = []
    for i in range(n):
        vals = {"src_ip": random_ipv6_text(rng), "dst_ip": random_ipv6_text(rng),
                "src_port": str(int(rng.integers(0, 65536))),
                "dst_port": str(int(rng.integers(0, 65536)))}
        rows.append(",".join(vals[cols[k]] for k in order))
        if seed % 3 == 0 and rng.random() < 0.05:
            rows.append("")  # blank lines are skipped by both paths
    text = ",".join(cols[k] for k in order) + eol + eol.join(rows) + (eol if seed != 4 else "")
    key = [int(x) for x in rng.integers(0, 256, 40)]
    H, Q = [(128, 24), (100, 7), (512, 64)][seed % 3]
    parsed = parse6(text, threads=3)
    assert parsed is not None
    tuples, spans, layout = parsed
    words = np.ascontiguousarray(tuples).view(np.uint32).reshape(-1, 9)
    h = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    q, c = o.queue_and_counts(h, H, Q)
    got = _native.csv_format6(text.encode("latin-1"), spans, h, q, c, layout, threads=3).tobytes()
    want, df = reference_stats_bytes6(text, h, H, Q, tmp_path)
    # the pandas path packs the same frame to the same words
    np.testing.assert_array_equal(np.ascontiguousarray(pack_frame6(df)).view(np.uint32).reshape(-1, 9),
                                  words)
    assert got == want


def test_accepted_mutations_agree_with_pandas():
    """Random single-byte mutations of a canonical file: whenever the native scanner still
    accepts the text, pandas + ipaddress (the pandas path) read the same tuples."""
    rng = np.random.default_rng(77)
    base_rows = ["%s,%s,%d,%d" % (random_ipv6_text(rng), random_ipv6_text(rng),
                                  int(rng.integers(0, 65536)), int(rng.integers(0, 65536)))
                 for _ in range(6)]
    base = "src_ip,dst_ip,src_port,dst_port\n" + "\n".join(base_rows) + "\n"
    alphabet = "0123456789abcdefABCDEF:,.\r\n %g-"
    accepted = 0
    for _ in range(400):
        chars = list(base)
        pos = int(rng.integers(0, len(chars)))
        op = rng.integers(0, 3)
        c = alphabet[int(rng.integers(0, len(alphabet)))]
        if op == 0:
            chars[pos] = c
        elif op == 1:
            chars.insert(pos, c)
        else:
            del chars[pos]
        text = "".join(chars)
        parsed = parse6(text)
        if parsed is None:
            continue
        accepted += 1
        df = pd.read_csv(io.StringIO(text))
        want = np.ascontiguousarray(pack_frame6(df)).view(np.uint32).reshape(-1, 9)
        np.testing.assert_array_equal(np.ascontiguousarray(parsed[0]).view(np.uint32).reshape(-1, 9),
                                      want)
        assert list(df.columns[:4]) == [["src_ip", "dst_ip", "src_port", "dst_port"][k]
                                        for k in parsed[2].field_column]
    assert accepted > 50
