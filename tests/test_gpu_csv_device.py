"""GPU parity of the device CSV path (``rss_csv_hash_text``): the statistics file it
formats on the device must be byte-identical to the reference's golden outputs and to
the host path (rss_csv_parse + oracle hashes + rss_csv_format, itself pinned to pandas
and the reference by tests/test_fastcsv.py); it must refuse exactly what the host
scanner refuses."""
import functools
import os
import random

import numpy as np
import pytest

from test_fastcsv import NOT_CANONICAL, HEADER, _random_canonical, parse

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


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


def device_image(native, ctx, text, key, H, Q, reta=None):
    got = ctx.csv_hash_text(native.prepare_key(key), _bytes(text), H, Q, reta=reta)
    return None if got is None else (got[0].tobytes(), got[1].copy(), got[2])


def host_image(native, oracle_lib, text, key, H, Q, reta=None):
    tuples, layout = parse(text)
    arr = np.stack([tuples["sip"], tuples["dip"], tuples["ports"]], axis=1)
    h, q, c = oracle_lib.run(key, arr, H, Q, threads=8)
    if reta is not None:
        q = np.asarray(reta, dtype=np.uint32)[h % H]
        c = np.bincount(q, minlength=Q).astype(np.uint64)
    return native.csv_format(tuples, h, q, c, layout).tobytes(), c, len(tuples)


def test_example_matches_reference_goldens(native, ctx, golden_dir, example_key):
    text = open(os.path.join(golden_dir, "example_input", "ips.csv"), "rb").read().decode("latin-1")
    checked = 0
    for name in sorted(os.listdir(os.path.join(golden_dir, "example"))):
        if not name.endswith(".csv"):
            continue
        h, q = (int(x[1:]) for x in name[4:-4].split("_"))
        image, counts, n = device_image(native, ctx, text, example_key, h, q)
        assert image == open(os.path.join(golden_dir, "example", name), "rb").read(), name
        assert n == 100 and int(counts.sum()) == 100
        checked += 1
    assert checked >= 9


@pytest.mark.parametrize("seed", range(8))
def test_random_canonical_equals_host_path(native, ctx, oracle_lib, example_key, seed):
    rng = random.Random(100 + seed)
    order = list(range(4))
    rng.shuffle(order)
    text = _random_canonical(rng, rng.choice([1, 2, 63, 64, 65, 5000, 40000]), order,
                             crlf=seed % 2 == 1, blank_lines=seed % 3 == 0,
                             trailing_nl=seed % 4 != 2)
    H, Q = rng.choice([(128, 24), (100, 7), (512, 64), (1, 1), (65536, 1000)])
    got = device_image(native, ctx, text, example_key, H, Q)
    want = host_image(native, oracle_lib, text, example_key, H, Q)
    assert got[0] == want[0]
    np.testing.assert_array_equal(got[1], want[1])
    assert got[2] == want[2]


def test_large_file_multi_tile_scans(native, ctx, oracle_lib, example_key):
    """~2.5M rows: thousands of scan tiles in both the newline and the row-length scans,
    CRLF line ends and scattered blank lines (the compaction pass)."""
    rng = random.Random(7)
    text = _random_canonical(rng, 2_500_000, [3, 1, 0, 2], crlf=True, blank_lines=True,
                             trailing_nl=False)
    got = device_image(native, ctx, text, example_key, 128, 24)
    want = host_image(native, oracle_lib, text, example_key, 128, 24)
    assert got[2] == want[2] == 2_500_000
    assert got[0] == want[0]


def test_empty_lines_and_line_end_forms(native, ctx, oracle_lib, example_key):
    rows = ["1.2.3.4,5.6.7.8,1,2", "9.9.9.9,0.0.0.0,65535,0", "255.255.255.255,1.0.0.1,80,443"]
    for text in [HEADER + "\n".join(rows),
                 HEADER + "\n\n" + "\n\n".join(rows) + "\n\n",
                 HEADER.replace("\n", "\r\n") + "\r\n".join(rows) + "\r\n\r\n",
                 HEADER + "\n".join(rows) + "\r",
                 HEADER + "\n".join(rows) + "\n\r"]:
        got = device_image(native, ctx, text, example_key, 128, 24)
        want = host_image(native, oracle_lib, text, example_key, 128, 24)
        assert got[0] == want[0], repr(text)


@pytest.mark.parametrize("text", NOT_CANONICAL)
def test_non_canonical_refused(native, ctx, example_key, text):
    raw = text.encode("utf-8").decode("latin-1")
    assert ctx.csv_hash_text(native.prepare_key(example_key), _bytes(raw), 128, 24) is None


def test_golden_edge_inputs_refused(native, ctx, golden_dir, example_key):
    for name in ["octet_overflow.csv", "whitespace.csv", "ports_wide.csv", "extra_reordered.csv",
                 "missing_col.csv", "header_only.csv", "not_csv.csv"]:
        data = np.fromfile(os.path.join(golden_dir, "edge", name), dtype=np.uint8)
        assert ctx.csv_hash_text(native.prepare_key(example_key), data, 128, 24) is None, name


def test_mutations_accepted_exactly_when_host_accepts(native, ctx, oracle_lib, example_key):
    rng = random.Random(11)
    base = _random_canonical(rng, 60, [1, 0, 3, 2], crlf=False, blank_lines=True,
                             trailing_nl=True)
    alphabet = "0123456789.,\n\r -+\"a"
    agree = accepted = 0
    for _ in range(300):
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
        host = parse(text)
        got = device_image(native, ctx, text, example_key, 128, 24)
        assert (host is None) == (got is None), repr(text)
        if got is not None:
            accepted += 1
            assert got[0] == host_image(native, oracle_lib, text, example_key, 128, 24)[0]
        agree += 1
    assert agree == 300 and accepted > 20


def test_counts_only_and_reta(native, ctx, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import reta as rt
    rng = random.Random(3)
    text = _random_canonical(rng, 30000, [0, 1, 2, 3], crlf=False, blank_lines=False,
                             trailing_nl=True)
    key = native.prepare_key(example_key)
    image, counts, n = ctx.csv_hash_text(key, _bytes(text), 512, 16, counts_only=True)
    want = host_image(native, oracle_lib, text, example_key, 512, 16)
    assert image is None and n == 30000
    np.testing.assert_array_equal(counts, want[1])
    table = rt.weights(512, [1, 3, 0, 2] * 4)
    got = device_image(native, ctx, text, example_key, 512, 16, reta=table)
    assert got[0] == host_image(native, oracle_lib, text, example_key, 512, 16, reta=table)[0]


def test_file_to_file_streams_through_staging(native, ctx, oracle_lib, example_key, tmp_path):
    """rss_csv_hash_file: > 2 pinned staging buffers (32 MiB) of input and of output; the
    file it writes equals the in-memory image and the host path."""
    rng = random.Random(21)
    text = _random_canonical(rng, 1_800_000, [0, 2, 1, 3], crlf=False, blank_lines=True,
                             trailing_nl=True)
    src, dst = tmp_path / "in.csv", tmp_path / "out.csv"
    src.write_bytes(text.encode())
    assert src.stat().st_size > 2 * (32 << 20)
    key = native.prepare_key(example_key)
    counts, n = ctx.csv_hash_file(key, str(src), str(dst), 128, 24)
    want = host_image(native, oracle_lib, text, example_key, 128, 24)
    assert dst.read_bytes() == want[0]
    assert n == want[2]
    np.testing.assert_array_equal(counts, want[1])
    c2, n2 = ctx.csv_hash_file(key, str(src), None, 128, 24)  # counts only
    np.testing.assert_array_equal(c2, want[1])
    assert n2 == n


def test_file_api_refusals_leave_no_output(native, ctx, example_key, golden_dir, tmp_path):
    key = native.prepare_key(example_key)
    dst = tmp_path / "out.csv"
    bad = tmp_path / "bad.csv"
    bad.write_bytes((HEADER + "3.3.3.300,1.1.1.1,1,1\n").encode())
    assert ctx.csv_hash_file(key, str(bad), str(dst), 128, 24) is None
    assert not dst.exists()
    assert ctx.csv_hash_file(key, str(tmp_path / "missing.csv"), str(dst), 128, 24) is None
    good = os.path.join(golden_dir, "example_input", "ips.csv")
    assert ctx.csv_hash_file(key, good, str(tmp_path / "no_dir" / "o.csv"), 128, 24) is None
    assert ctx.csv_hash_file(key, str(tmp_path), str(dst), 128, 24) is None  # a directory
    counts, n = ctx.csv_hash_file(key, good, str(dst), 128, 24)
    assert n == 100 and dst.read_bytes() == open(
        os.path.join(golden_dir, "example", "out_h128_q24.csv"), "rb").read()


@pytest.mark.parametrize("rows,crlf,trailing_nl", [(3_400_000, False, True), (2_000_000, True, False)])
def test_file_to_file_in_segments(native, ctx, oracle_lib, example_key, tmp_path, monkeypatch,
                                  rows, crlf, trailing_nl):
    """Bodies are processed in line-aligned segments below the 4 GiB of 32-bit newline
    positions (3 GiB by default); RSS_CSV_SEGMENT_BYTES at its 64 MiB + 4 KiB floor cuts
    these files into 2-3 segments, counts summed across them, rows written in order."""
    monkeypatch.setenv("RSS_CSV_SEGMENT_BYTES", str((64 << 20) + 4096))
    rng = random.Random(rows)
    text = _random_canonical(rng, rows, [3, 1, 0, 2], crlf=crlf, blank_lines=True,
                             trailing_nl=trailing_nl)
    src, dst = tmp_path / "in.csv", tmp_path / "out.csv"
    src.write_bytes(text.encode())
    assert src.stat().st_size > (64 << 20) + 4096
    key = native.prepare_key(example_key)
    counts, n = ctx.csv_hash_file(key, str(src), str(dst), 128, 24)
    want = host_image(native, oracle_lib, text, example_key, 128, 24)
    assert n == want[2]
    np.testing.assert_array_equal(counts, want[1])
    assert dst.read_bytes() == want[0]
    c2, n2 = ctx.csv_hash_file(key, str(src), None, 128, 24)  # counts only, segmented too
    np.testing.assert_array_equal(c2, want[1])
    assert n2 == n


@functools.lru_cache(maxsize=1)
def _segmented_text():
    return _random_canonical(random.Random(5), 2_400_000, [0, 1, 2, 3], crlf=False,
                             blank_lines=False, trailing_nl=True)


@pytest.mark.parametrize("where", ["first", "last"])
def test_refusal_inside_a_segmented_file_then_recovery(native, ctx, oracle_lib, example_key,
                                                       tmp_path, monkeypatch, where):
    """A non-canonical row in the first or the last of a file's segments: the call refuses
    part-way through the streaming (no output file), and the next call on the same context
    streams the good file exactly."""
    monkeypatch.setenv("RSS_CSV_SEGMENT_BYTES", str((64 << 20) + 4096))
    text = _segmented_text()
    header, body = text.split("\n", 1)
    bad_row = "3.3.3.300,1.1.1.1,1,1\n"
    bad_text = header + "\n" + (bad_row + body if where == "first" else body + bad_row)
    src, bad, dst = tmp_path / "in.csv", tmp_path / "bad.csv", tmp_path / "out.csv"
    src.write_bytes(text.encode())
    bad.write_bytes(bad_text.encode())
    assert src.stat().st_size > (64 << 20) + 4096
    key = native.prepare_key(example_key)
    assert ctx.csv_hash_file(key, str(bad), str(dst), 128, 24) is None
    assert not dst.exists()
    counts, n = ctx.csv_hash_file(key, str(src), str(dst), 128, 24)
    want = host_image(native, oracle_lib, text, example_key, 128, 24)
    assert n == want[2]
    np.testing.assert_array_equal(counts, want[1])
    assert dst.read_bytes() == want[0]


def test_default_image_is_an_owned_copy(native, ctx, example_key):
    """csv_hash_text's default image (copied out on several threads when large) equals the
    context's own image (copy=False) and outlives the next call on the context."""
    rng = random.Random(11)
    base = _random_canonical(rng, 100_000, (0, 1, 2, 3), False, False, True)
    header, body = base.split("\n", 1)
    text = header + "\n" + body * 16  # 1.6M rows, a statistics image above 64 MiB
    key = native.prepare_key(example_key)
    owned = ctx.csv_hash_text(key, _bytes(text), 128, 24)[0]
    view = ctx.csv_hash_text(key, _bytes(text), 128, 24, copy=False)[0]
    assert owned.size > (64 << 20) and owned.tobytes() == view.tobytes()
    assert owned.ctypes.data != view.ctypes.data
    before = owned.tobytes()
    ctx.csv_hash_text(key, _bytes(text[:len(text) // 3].rsplit("\n", 1)[0] + "\n"), 100, 7)
    assert owned.tobytes() == before
