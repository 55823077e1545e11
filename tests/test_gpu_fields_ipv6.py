"""GPU parity for field selection (IPv4 kernel with remapped windows) and the IPv6 kernel:
bit-exact against the literal rotating-key oracle over the selected bytes and the
Microsoft verification-suite vectors; at scale (2^20 tuples per mask) against
oracle_run_words over the selected, zero-padded bytes."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as o

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


@pytest.mark.parametrize("mask", list(range(1, 16)))
def test_ipv4_field_masks_on_gpu(native, ctx, oracle_lib, random_golden, mask):
    g = random_golden
    key = g["key_list"][1]
    h, q, c = ctx.hash(native.prepare_key(key, mask), g["tuples"], 128, 24)
    want = np.array([oracle_lib.hash_bytes(key, o.select_fields_bytes(a, b, p, mask))
                     for a, b, p in g["tuples"]], dtype=np.uint32)
    np.testing.assert_array_equal(h, want)
    qo, co = o.queue_and_counts(want, 128, 24)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)


def test_ipv6_kat_on_gpu(native, ctx, golden_dir):
    from rss_simulator_nvidia_amd.ingest import ipv6_words
    kat = json.load(open(os.path.join(golden_dir, "ms_kat_ipv6.json")))
    key = [int(x, 16) for x in kat["key"].split(":")]
    words = np.array([ipv6_words(v["src_ip"]) + ipv6_words(v["dst_ip"]) +
                      [(v["src_port"] << 16) | v["dst_port"]] for v in kat["vectors"]],
                     dtype=np.uint32)
    h, _, _ = ctx.hash6(native.prepare_key6(key), words, 1, 1)
    assert [int(x) for x in h] == [int(v["hash_hex"], 16) for v in kat["vectors"]]
    h, _, _ = ctx.hash6(native.prepare_key6(key, "sd"), words, 1, 1)
    assert [int(x) for x in h] == [int(v["hash_ip_only_hex"], 16) for v in kat["vectors"]]


@pytest.mark.parametrize("H,Q,n", [(128, 24, 100003), (100, 7, 4099), (65536, 1000, 20001),
                                   (100000, 7, 5000), (50000, 10000, 3001), (512, 64, 0),
                                   (1, 1, 3)])
def test_ipv6_kernel_vs_oracle(native, ctx, oracle_lib, H, Q, n):
    rng = np.random.default_rng(H + n)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    words = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    h, q, c = ctx.hash6(native.prepare_key6(key), words, H, Q)
    w = oracle_lib.windows_n(key, 288)
    want = o.hash_words_np(w, words)
    for i in range(0, n, max(1, n // 64)):  # literal loop on a sample
        assert oracle_lib.hash_bytes(key, o.words_to_bytes(words[i])) == want[i]
    np.testing.assert_array_equal(h, want)
    qo, co = o.queue_and_counts(want, H, Q)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)


def test_ipv6_device_api_misaligned(native, oracle_lib):
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(7)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    n = 65541
    words = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    want = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    raw = torch.from_numpy(words.view(np.int32).reshape(-1)).to(dev)
    shifted = torch.empty(9 * n + 1, dtype=torch.int32, device=dev)
    shifted[1:] = raw
    k6 = native.prepare_key6(key)
    for src in (raw, shifted[1:]):
        hashes = torch.full((n + 1,), -1, dtype=torch.int32, device=dev)
        counts = torch.empty(24, dtype=torch.int64, device=dev)
        native.hash6_device(k6, src.data_ptr(), n, 128, 24, hashes.data_ptr(), None,
                            counts.data_ptr(), 0, s)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(hashes[:n].cpu().numpy().view(np.uint32), want)
        assert int(hashes[n]) == -1
        assert int(counts.sum()) == n


@pytest.mark.parametrize("flag_name,dtype,H,Q", [("FLAG_QUEUE_U8", np.uint8, 128, 24),
                                                 ("FLAG_QUEUE_U8", np.uint8, 100, 256),
                                                 ("FLAG_QUEUE_U16", np.uint16, 65536, 1000),
                                                 (None, np.uint32, 512, 64)])
def test_ipv6_narrow_queue_outputs(native, oracle_lib, flag_name, dtype, H, Q):
    """RSS_FLAG_QUEUE_U8 / U16 on the IPv6 kernel: aligned (4 queues per store) and
    misaligned (scalar stores) queue buffers, no bytes written outside the output."""
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(H + Q)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    n = 40003
    words = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    h = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    qo = (h % H) % Q
    raw = torch.from_numpy(words.view(np.int32).reshape(-1)).to(dev)
    k6 = native.prepare_key6(key)
    item = np.dtype(dtype).itemsize
    flags = getattr(native, flag_name) if flag_name else 0
    for offset in (0, item):
        buf = torch.full((n * item + 64,), 0xAB, dtype=torch.uint8, device=dev)
        qn = min(H, Q)  # count vectors are min(H, Q) long (_native.queue_modulus)
        counts = torch.empty(qn, dtype=torch.int64, device=dev)
        native.hash6_device(k6, raw.data_ptr(), n, H, Q, None, buf.data_ptr() + offset,
                            counts.data_ptr(), flags, s)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        np.testing.assert_array_equal(got[offset:offset + n * item].view(dtype), qo.astype(dtype))
        assert (got[:offset] == 0xAB).all() and (got[offset + n * item:] == 0xAB).all()
        np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64),
                                      np.bincount(qo.astype(np.int64), minlength=qn))
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    with pytest.raises(DeviceError, match="QUEUE_U8"):
        native.hash6_device(k6, 0, 0, 1024, 257, None, None, None, native.FLAG_QUEUE_U8)


def test_cli_ipv6_and_fields(tmp_path, golden_dir, oracle_lib, capsys):
    from cli_cases import run_main
    rng = np.random.default_rng(3)
    rows = ["src_ip,dst_ip,src_port,dst_port"]
    import ipaddress
    words = []
    for _ in range(500):
        a = ipaddress.IPv6Address(int(rng.integers(0, 2**62)) << 64 | int(rng.integers(0, 2**62)))
        b = ipaddress.IPv6Address(int(rng.integers(0, 2**62)) << 40)
        sp, dp = int(rng.integers(0, 65536)), int(rng.integers(0, 65536))
        rows.append("%s,%s,%d,%d" % (a, b, sp, dp))
        words.append([int.from_bytes(a.packed[4 * k:4 * k + 4], "big") for k in range(4)] +
                     [int.from_bytes(b.packed[4 * k:4 * k + 4], "big") for k in range(4)] +
                     [sp << 16 | dp])
    src = tmp_path / "v6.csv"
    src.write_text("\n".join(rows) + "\n")
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    key = [int(x, 16) for x in open(key_file).read().split(":")]
    for fields, nbytes in (("sdfn", 36), ("sd", 32)):
        out = tmp_path / ("out_%s.csv" % fields)
        status, _, _, exc = run_main(["--key-file", key_file, "--ips-file", str(src),
                                      "--htable-size", "128", "--num-queues", "24", "--csv",
                                      str(out), "--ipv6", "--hash-fields", fields], capsys)
        assert status == 0, exc
        import pandas as pd
        lines = out.read_text().splitlines()
        table = pd.read_csv(str(out), skiprows=len(lines) - 501)
        want = [oracle_lib.hash_bytes(key, o.words_to_bytes(w)[:nbytes]) for w in words]
        assert table.hash_result.tolist() == want
        assert table.queue_number.tolist() == [h % 128 % 24 for h in want]


@pytest.mark.parametrize("fmt", ["pcap", "pcapng"])
def test_cli_pcap_gpu(tmp_path, golden_dir, oracle_lib, capsys, fmt):
    """20K-packet synthetic capture (Ethernet/VLAN, TCP/UDP/ICMP, repeats) through --pcap,
    as a classic pcap and as a pcapng image."""
    from cli_cases import run_main
    from pcap_builder import ether, ipv4, l4, pcap_file, pcapng_section
    from rss_simulator_nvidia_amd import pcap
    rng = np.random.default_rng(9)
    pk = []
    for i in range(20000):
        a, b = tuple(int(x) for x in rng.integers(0, 256, 4)), tuple(int(x) for x in rng.integers(0, 256, 4))
        proto = (6, 17, 1)[i % 3]
        body = l4(int(rng.integers(0, 65536)), int(rng.integers(0, 65536))) if proto != 1 else b"\x00" * 20
        pk.append(ether(ipv4(a, b, proto, body), vlans=[(0x8100, 5)] if i % 5 == 0 else ()))
        if i % 7 == 0:
            pk.append(pk[-1])  # repeated packet of the same flow
    path = tmp_path / ("cap." + fmt)
    path.write_bytes(pcap_file(pk) if fmt == "pcap" else pcapng_section(pk))
    out = tmp_path / "out.csv"
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    status, so, _, exc = run_main(["--key-file", key_file, "--ips-file", str(path), "--pcap",
                                   "--htable-size", "512", "--num-queues", "16", "--csv", str(out),
                                   "--pcap-l4", "udp"], capsys)
    assert status == 0, exc
    key = [int(x, 16) for x in open(key_file).read().split(":")]
    t, _, _ = pcap.read_flows(str(path), "udp")
    assert len(t) == 20000
    h, q, c = oracle_lib.run(key, np.stack([t["sip"], t["dip"], t["ports"]], axis=1), 512, 16)
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    assert [int(x.split(",")[4]) for x in body] == h.tolist()
    assert lines[1:17] == ["%d,%d" % (i, c[i]) for i in range(16) if c[i]]


def test_cli_pcap_ipv6_gpu(tmp_path, golden_dir, oracle_lib, capsys):
    """--pcap --ipv6 on the GPU: IPv6 flows (extension headers, fragments, VLAN) of a pcapng
    capture through the IPv6 kernel; hashes equal the oracle's literal 36-byte loop."""
    from cli_cases import run_main
    from pcap_builder import pcapng_section
    from test_pcap import packets6_and_expected
    pk, want, _ = packets6_and_expected()
    path = tmp_path / "c6.pcapng"
    path.write_bytes(pcapng_section(pk * 50))
    out = tmp_path / "out6.csv"
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    status, so, _, exc = run_main(["--key-file", key_file, "--ips-file", str(path), "--pcap",
                                   "--ipv6", "--htable-size", "64", "--num-queues", "6",
                                   "--csv", str(out)], capsys)
    assert status == 0, exc
    key = [int(x, 16) for x in open(key_file).read().split(":")]
    uniq = list(dict.fromkeys(r[:9] for r in want))
    want_h = [oracle_lib.hash_bytes(key, b"".join(int(w).to_bytes(4, "big") for w in r))
              for r in uniq]
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    assert [int(x.split(",")[4]) for x in body] == want_h
    assert [int(x.split(",")[5]) for x in body] == [h % 64 % 6 for h in want_h]


def test_cli_ipv6_csv_fast_path_equals_pandas_path(tmp_path, golden_dir, monkeypatch, capsys):
    """--ipv6 --csv: the native IPv6 CSV path (rss_csv_parse6 / rss_csv_format6 around the
    IPv6 kernel) writes the same file as the pandas path on the GPU, byte for byte."""
    from cli_cases import run_main
    from test_fastcsv6 import random_ipv6_text
    rng = np.random.default_rng(12)
    rows = ["%s,%d,%s,%d" % (random_ipv6_text(rng), int(rng.integers(0, 65536)),
                             random_ipv6_text(rng), int(rng.integers(0, 65536)))
            for _ in range(20000)]
    path = tmp_path / "ips6.csv"
    path.write_text("dst_ip,src_port,src_ip,dst_port\r\n" + "\r\n".join(rows) + "\r\n")
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    outs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("RSS_CSV_FASTPATH", fast)
        out = tmp_path / ("out%s.csv" % fast)
        status, so, _, exc = run_main(["--key-file", key_file, "--ips-file", str(path), "--ipv6",
                                       "--htable-size", "128", "--num-queues", "24",
                                       "--csv", str(out)], capsys)
        assert status == 0, exc
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]


def _selected_words(words, spans, mask):
    """The bytes of the selected fields (spans: (bit, first byte, length) of the big-endian
    input), concatenated and zero-padded to whole words: zero bits add nothing to a Toeplitz
    hash, so oracle_run_words over them is the literal loop over the selected bytes."""
    raw = words.astype(">u4").view(np.uint8).reshape(len(words), -1)
    cols = [raw[:, a:a + n] for bit, a, n in spans if mask & bit]
    sel = np.concatenate(cols, axis=1)
    pad = (-sel.shape[1]) % 4
    if pad:
        sel = np.concatenate([sel, np.zeros((len(sel), pad), np.uint8)], axis=1)
    return np.ascontiguousarray(sel).view(">u4").astype(np.uint32)


@pytest.mark.parametrize("mask", [1, 2, 3, 4, 5, 8, 10, 12, 14, 15])
def test_ipv4_field_masks_at_scale(native, oracle_lib, example_key, mask):
    """2^20 + 3 tuples per field mask through the device API, element by element against
    oracle_run_words over the selected bytes (tests/test_oracle.py pins it to the literal
    loop); the 15-mask row is the reference's whole-tuple hash."""
    n = (1 << 20) + 3
    host = oracle_lib.generate(90 + mask, 0, n)
    spans = [(1, 0, 4), (2, 4, 4), (4, 8, 2), (8, 10, 2)]
    ho, qo, co = oracle_lib.run_words(example_key, _selected_words(host, spans, mask), 512, 24)
    dev = torch.device("cuda:0")
    t = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    h = torch.empty(n, dtype=torch.int32, device=dev)
    q = torch.empty(n, dtype=torch.int32, device=dev)
    c = torch.empty(24, dtype=torch.int64, device=dev)
    native.hash_device(native.prepare_key(example_key, mask), t.data_ptr(), n, 512, 24,
                       h.data_ptr(), q.data_ptr(), c.data_ptr(), 0,
                       torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
    np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), qo)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)


@pytest.mark.parametrize("mask", [3, 12, 1, 15])
def test_ipv6_field_masks_at_scale(native, oracle_lib, example_key, mask):
    """The IPv6 kernel with remapped windows: 2^20 + 1 tuples per mask ("sd" = the IPv6-only
    hash) against oracle_run_words over the selected bytes."""
    n = (1 << 20) + 1
    rng = np.random.default_rng(mask)
    host = rng.integers(0, 2**32, size=(n, 9), dtype=np.uint64).astype(np.uint32)
    spans = [(1, 0, 16), (2, 16, 16), (4, 32, 2), (8, 34, 2)]
    ho, qo, co = oracle_lib.run_words(example_key, _selected_words(host, spans, mask), 128, 24)
    dev = torch.device("cuda:0")
    t = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    h = torch.empty(n, dtype=torch.int32, device=dev)
    q = torch.empty(n, dtype=torch.uint8, device=dev)
    c = torch.empty(24, dtype=torch.int64, device=dev)
    native.hash6_device(native.prepare_key6(example_key, mask), t.data_ptr(), n, 128, 24,
                        h.data_ptr(), q.data_ptr(), c.data_ptr(), native.FLAG_QUEUE_U8,
                        torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
    np.testing.assert_array_equal(q.cpu().numpy().astype(np.uint32), qo)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)
