"""GPU parity of the IPv6 device CSV path (``rss_csv6_hash_text`` / ``rss_csv6_hash_file``):
the statistics file it builds on the device must be byte-identical to the host path
(rss_csv_parse6 + the oracle's closed form over the 288 IPv6 windows + rss_csv_format6,
itself pinned to pandas + ipaddress by tests/test_fastcsv6.py), and it must refuse
exactly what the host scanner refuses."""
import random

import numpy as np
import pytest

from oracle import oracle as o
from test_fastcsv6 import NOT_CANONICAL6, parse6, random_ipv6_text, reference_stats_bytes6

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

COLS = ["src_ip", "dst_ip", "src_port", "dst_port"]


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


@pytest.fixture(scope="module")
def ctx(native):
    return native.HostContext(0)


def _bytes(text):
    return np.frombuffer(text.encode("latin-1"), dtype=np.uint8)


def random_file6(seed, n, order, crlf=False, blank_lines=False, trailing_nl=True, pool=4096):
    """n canonical IPv6 rows in the given column order; addresses drawn from a pool of
    random RFC 4291 text forms (every style of random_ipv6_text)."""
    rng = np.random.default_rng(seed)
    addrs = [random_ipv6_text(rng) for _ in range(min(pool, 2 * n))]
    a = rng.integers(0, len(addrs), (n, 2))
    p = rng.integers(0, 65536, (n, 2))
    r = random.Random(seed)
    rows = []
    for i in range(n):
        vals = (addrs[a[i, 0]], addrs[a[i, 1]], str(p[i, 0]), str(p[i, 1]))
        rows.append(",".join(vals[k] for k in order))
        if blank_lines and r.random() < 0.02:
            rows.append("")
    eol = "\r\n" if crlf else "\n"
    return ",".join(COLS[k] for k in order) + eol + eol.join(rows) + (eol if trailing_nl else "")


def device_image6(native, ctx, text, key, H, Q, reta=None):
    got = ctx.csv_hash_text(native.prepare_key6(key), _bytes(text), H, Q, reta=reta)
    return None if got is None else (got[0].tobytes(), got[1].copy(), got[2])


def host_image6(native, oracle_lib, text, key, H, Q, reta=None):
    parsed = parse6(text)
    if parsed is None:
        return None
    tuples, spans, layout = parsed
    words = np.ascontiguousarray(tuples).view(np.uint32).reshape(-1, 9)
    h = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    if reta is None:
        q, c = o.queue_and_counts(h, H, Q)
    else:
        q = np.asarray(reta, dtype=np.uint32)[h % H]
        c = np.bincount(q, minlength=Q).astype(np.uint64)
    return native.csv_format6(text.encode("latin-1"), spans, h, q, c, layout).tobytes(), c, len(h)


@pytest.mark.parametrize("seed", range(8))
def test_random_canonical_equals_host_path(native, ctx, oracle_lib, example_key, seed):
    rng = random.Random(600 + seed)
    order = list(range(4))
    rng.shuffle(order)
    n = rng.choice([1, 2, 255, 256, 257, 5000, 40000])
    text = random_file6(seed, n, order, crlf=seed % 2 == 1, blank_lines=seed % 3 == 0,
                        trailing_nl=seed % 4 != 2)
    H, Q = rng.choice([(128, 24), (100, 7), (512, 64), (1, 1), (65536, 1000)])
    got = device_image6(native, ctx, text, example_key, H, Q)
    want = host_image6(native, oracle_lib, text, example_key, H, Q)
    assert got[2] == want[2] == n
    np.testing.assert_array_equal(got[1], want[1])
    assert got[0] == want[0]


def test_matches_pandas_bytes(native, ctx, oracle_lib, example_key, tmp_path):
    """The device image against what the pandas path writes (simulator.py:96-115)."""
    text = random_file6(5, 3000, [2, 0, 3, 1], crlf=True)
    got = device_image6(native, ctx, text, example_key, 128, 24)
    words = np.ascontiguousarray(parse6(text)[0]).view(np.uint32).reshape(-1, 9)
    h = o.hash_words_np(oracle_lib.windows_n(example_key, 288), words)
    want, _ = reference_stats_bytes6(text, h, 128, 24, tmp_path)
    assert got[0] == want


def test_address_forms_and_line_ends(native, ctx, oracle_lib, example_key):
    addrs = ["::", "::1", "1::", "1:2:3:4:5:6:7::", "::2:3:4:5:6:7:8", "0:0:0:0:0:0:0:0",
             "FFFF:ffff:FfFf:0:0:0:0:1", "fe80::abcd:0:0:1", "ffff:ffff:ffff:ffff:ffff:ffff:ffff:ffff",
             "2001:db8::", "0000:0000:0000:0000:0000:0000:0000:0001"]
    rows = ["%s,%s,%d,%d" % (a, addrs[-1 - i], i, 65535 - i) for i, a in enumerate(addrs)]
    head = "src_ip,dst_ip,src_port,dst_port\n"
    for text in [head + "\n".join(rows), head + "\n\n" + "\n\n".join(rows) + "\n\n",
                 head.replace("\n", "\r\n") + "\r\n".join(rows) + "\r\n\r\n",
                 head + "\n".join(rows) + "\r", head + "\n".join(rows) + "\n\r",
                 "dst_port,src_ip,src_port,dst_ip\n" + "\n".join(
                     "1,%s,2,%s" % (a, addrs[-1 - i]) for i, a in enumerate(addrs))]:
        got = device_image6(native, ctx, text, example_key, 128, 24)
        want = host_image6(native, oracle_lib, text, example_key, 128, 24)
        assert got is not None and got[0] == want[0], repr(text)


@pytest.mark.parametrize("addr", NOT_CANONICAL6)
def test_non_canonical_addresses_refused(native, ctx, example_key, addr):
    text = "src_ip,dst_ip,src_port,dst_port\n::1,::2,3,4\n%s,::1,1,2\n" % addr
    assert ctx.csv_hash_text(native.prepare_key6(example_key), _bytes(text), 128, 24) is None


@pytest.mark.parametrize("row", ["::1,::2,65536,1", "::1,::2,01,2", "::1,::2,-1,2", "::1,::2,1",
                                 "::1,::2,1,2,3", "::1;::2;1;2", "::1,::2,1,2\r\r"])
def test_non_canonical_rows_refused(native, ctx, example_key, row):
    text = "src_ip,dst_ip,src_port,dst_port\n%s\n" % row
    assert ctx.csv_hash_text(native.prepare_key6(example_key), _bytes(text), 128, 24) is None


def test_mutations_accepted_exactly_when_host_accepts(native, ctx, oracle_lib, example_key):
    rng = random.Random(13)
    base = random_file6(13, 40, [1, 0, 3, 2], blank_lines=True)
    head_len = base.index("\n") + 1
    alphabet = "0123456789abcdefABCDEF:,.\r\n %g-"
    accepted = 0
    for _ in range(300):
        s = list(base)
        i = rng.randrange(head_len, len(s))
        op = rng.random()
        if op < 0.4:
            s[i] = rng.choice(alphabet)
        elif op < 0.7:
            s.insert(i, rng.choice(alphabet))
        else:
            del s[i]
        text = "".join(s)
        want = host_image6(native, oracle_lib, text, example_key, 128, 24)
        got = device_image6(native, ctx, text, example_key, 128, 24)
        assert (want is None) == (got is None), repr(text)
        if got is not None:
            accepted += 1
            assert got[0] == want[0]
    assert accepted > 20


def test_counts_only_and_reta(native, ctx, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import reta as rt
    text = random_file6(3, 30000, [0, 1, 2, 3])
    key6 = native.prepare_key6(example_key)
    image, counts, n = ctx.csv_hash_text(key6, _bytes(text), 512, 16, counts_only=True)
    want = host_image6(native, oracle_lib, text, example_key, 512, 16)
    assert image is None and n == 30000
    np.testing.assert_array_equal(counts, want[1])
    table = rt.weights(512, [1, 3, 0, 2] * 4)
    got = device_image6(native, ctx, text, example_key, 512, 16, reta=table)
    assert got[0] == host_image6(native, oracle_lib, text, example_key, 512, 16, reta=table)[0]


def test_field_selection_key(native, ctx, oracle_lib, example_key):
    """A 2-tuple key (addresses only) through the device path equals the host path's
    rss_hash6_host with the same prepared key."""
    text = random_file6(8, 2000, [0, 1, 2, 3])
    key6 = native.prepare_key6(example_key, native.FIELDS_IP)
    image, counts, n = ctx.csv_hash_text(key6, _bytes(text), 128, 24)
    tuples, spans, layout = parse6(text)
    h, q, c = ctx.hash6(key6, tuples, 128, 24)
    assert image.tobytes() == native.csv_format6(text.encode(), spans, h, q, c, layout).tobytes()


@pytest.mark.parametrize("segment", [None, (64 << 20) + 4096])
def test_file_to_file(native, ctx, oracle_lib, example_key, tmp_path, monkeypatch, segment):
    """rss_csv6_hash_file: > 2 pinned staging buffers of input and output; with the
    segment floor the body is cut into 2 line-aligned segments."""
    if segment:
        monkeypatch.setenv("RSS_CSV_SEGMENT_BYTES", str(segment))
    text = random_file6(21, 1_300_000, [0, 2, 1, 3], crlf=segment is None, blank_lines=True,
                        trailing_nl=segment is None)
    src, dst = tmp_path / "in6.csv", tmp_path / "out6.csv"
    src.write_bytes(text.encode())
    assert src.stat().st_size > (64 << 20) + 4096
    key6 = native.prepare_key6(example_key)
    counts, n = ctx.csv_hash_file(key6, str(src), str(dst), 128, 24)
    want = host_image6(native, oracle_lib, text, example_key, 128, 24)
    assert n == want[2] == 1_300_000
    np.testing.assert_array_equal(counts, want[1])
    assert dst.read_bytes() == want[0]
    c2, n2 = ctx.csv_hash_file(key6, str(src), None, 128, 24)
    np.testing.assert_array_equal(c2, want[1])
    assert n2 == n


def test_cli_ipv6_csv_takes_the_device_path(native, example_key, tmp_path, monkeypatch):
    """fastcsv.run_csv6 routes a canonical file through rss_csv6_hash_file and writes the
    same bytes as the host text path (RSS_CSV_DEVICE=0)."""
    from rss_simulator_nvidia_amd import fastcsv
    text = random_file6(31, 20000, [1, 0, 2, 3])
    src = tmp_path / "in6.csv"
    src.write_bytes(text.encode())
    timings = {}
    assert fastcsv.run_csv6(example_key, str(src), 128, 24, str(tmp_path / "dev.csv"),
                            timings=timings)
    assert timings["path"] == "device6"
    monkeypatch.setenv("RSS_CSV_DEVICE", "0")
    host = {}
    assert fastcsv.run_csv6(example_key, str(src), 128, 24, str(tmp_path / "host.csv"),
                            timings=host)
    assert host["path"] == "host6"
    assert (tmp_path / "dev.csv").read_bytes() == (tmp_path / "host.csv").read_bytes()
    c_host = fastcsv.run_counts6(example_key, str(src), 128, 24)
    monkeypatch.setenv("RSS_CSV_DEVICE", "1")
    np.testing.assert_array_equal(fastcsv.run_counts6(example_key, str(src), 128, 24), c_host)
