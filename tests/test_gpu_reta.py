"""GPU parity of the indirection-table queue mode (``rss_hash_device_reta``).

The 'equal' table is the reference's ``hash % htable % queues`` mapping
(``rss_simulator/simulator.py:96-98``), so it must reproduce the reference-generated
sweep fixtures exactly; arbitrary tables are checked against numpy ``reta[hash % H]``
on oracle hashes, across the histogram modes (private / shared / global bins) and the
u8 / u16 / u32 queue outputs.
"""
import numpy as np
import pytest

from rss_simulator_nvidia_amd import reta as rt

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


def test_equal_table_reproduces_reference_sweep(native, ctx, random_golden):
    g = random_golden
    key = native.prepare_key(g["key_list"][0])
    for j, (H, Q) in enumerate(g["sweep"]):
        H, Q = int(H), int(Q)
        if H > rt.MAX_ENTRIES:
            continue
        h, q, c = ctx.hash(key, g["tuples"], H, Q, reta=rt.equal(H, Q))
        np.testing.assert_array_equal(h, g["hashes"][0])
        np.testing.assert_array_equal(q, g["sweep_queue"][j])
        assert [[int(a), int(c[a])] for a in np.flatnonzero(c)] == g["sweep_counts"]["%d,%d" % (H, Q)]


@pytest.mark.parametrize("H,Q", [(128, 24), (1024, 256), (100, 7), (512, 1000), (64, 8192),
                                 (1, 1), (1000, 3)])
def test_random_tables_vs_oracle(native, ctx, oracle_lib, example_key, H, Q):
    rng = np.random.default_rng(H * 7 + Q)
    table = rng.integers(0, Q, size=H, dtype=np.uint32)
    tup = oracle_lib.generate(H + 13 * Q, 0, 300007)
    ho, _, _ = oracle_lib.run(example_key, tup, H, Q)
    qo = table[ho % H]
    co = np.bincount(qo, minlength=Q).astype(np.uint64)
    h, q, c = ctx.hash(native.prepare_key(example_key), tup, H, Q, reta=table)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)


@pytest.mark.parametrize("flag_name,dtype", [("FLAG_QUEUE_U8", np.uint8),
                                             ("FLAG_QUEUE_U16", np.uint16), (None, np.uint32)])
def test_weighted_table_device_api(native, oracle_lib, example_key, flag_name, dtype):
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    n, H, Q = 1 << 20, 128, 16
    table = np.array(rt.weights(H, [3, 1, 0, 4] * 4), dtype=np.uint32)
    tup_host = oracle_lib.generate(5, 0, n)
    ho, _, _ = oracle_lib.run(example_key, tup_host, H, Q)
    qo = table[ho % H]
    raw = torch.from_numpy(tup_host.view(np.int32).reshape(-1)).to(dev)
    item = np.dtype(dtype).itemsize
    buf = torch.full((n * item,), 0xAB, dtype=torch.uint8, device=dev)
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    flags = getattr(native, flag_name) if flag_name else 0
    key = native.prepare_key(example_key)
    native.hash_device_reta(key, raw.data_ptr(), n, H, table, Q, None, buf.data_ptr(),
                            counts.data_ptr(), flags, s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(buf.cpu().numpy().view(dtype), qo.astype(dtype))
    got = counts.cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, np.bincount(qo, minlength=Q))
    assert got[2::4].sum() == 0  # zero-weight queues are never selected


def test_table_validation(native, example_key):
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    key = native.prepare_key(example_key)
    with pytest.raises(DeviceError, match="nqueues"):
        native.hash_device_reta(key, 0, 0, 4, [0, 1, 4, 2], 4)
    with pytest.raises(DeviceError, match="exceeds"):
        native.hash_device_reta(key, 0, 0, 2048, [0] * 2048, 1)


@pytest.mark.parametrize("H,Q,flag_name", [(128, 24, "FLAG_QUEUE_U8"), (1024, 5000, None),
                                           (100, 7, "FLAG_QUEUE_U16"), (1024, 300, None)])
def test_ipv6_tables_vs_oracle(native, ctx, oracle_lib, H, Q, flag_name):
    """IPv6 kernel with an indirection table (rss_hash6_device_reta / _host_reta): queue =
    reta[hash % H] on the 36-byte hashes, all histogram modes the bin budget reaches
    (the table takes 4 * H bytes of the IPv6 kernel's 12 KiB bin region)."""
    from oracle import oracle as o
    rng = np.random.default_rng(H * 3 + Q)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    n = 100003
    words = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    want = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    table = rng.integers(0, Q, H).astype(np.uint32)
    wq = table[want % H]
    wc = np.bincount(wq, minlength=Q).astype(np.uint64)
    k6 = native.prepare_key6(key)
    h, q, c = ctx.hash6(k6, words, H, Q, reta=table)  # host path
    np.testing.assert_array_equal(h, want)
    np.testing.assert_array_equal(q, wq)
    np.testing.assert_array_equal(c, wc)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    raw = torch.from_numpy(words.view(np.int32).reshape(-1)).to(dev)
    dtype = {"FLAG_QUEUE_U8": np.uint8, "FLAG_QUEUE_U16": np.uint16, None: np.uint32}[flag_name]
    item = np.dtype(dtype).itemsize
    buf = torch.full((n * item + 16,), 0xAB, dtype=torch.uint8, device=dev)
    counts = torch.empty(Q, dtype=torch.int64, device=dev)
    flags = getattr(native, flag_name) if flag_name else 0
    native.hash6_device_reta(k6, raw.data_ptr(), n, H, table, Q, None, buf.data_ptr(),
                             counts.data_ptr(), flags, s)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    np.testing.assert_array_equal(got[:n * item].view(dtype), wq.astype(dtype))
    assert (got[n * item:] == 0xAB).all()
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), wc)


def test_ipv6_cli_reta_weights(tmp_path, golden_dir, oracle_lib, capsys):
    """--ipv6 --reta-weights through the pandas path of Simulator on the GPU."""
    from cli_cases import run_main
    from oracle import oracle as o
    rng = np.random.default_rng(4)
    n = 300
    addrs = ["2001:db8::%x" % int(x) for x in rng.integers(1, 1 << 16, 2 * n)]
    ports = rng.integers(0, 65536, (n, 2))
    path = tmp_path / "ips6.csv"
    path.write_text("src_ip,dst_ip,src_port,dst_port\n" + "".join(
        "%s,%s,%d,%d\n" % (addrs[2 * i], addrs[2 * i + 1], ports[i, 0], ports[i, 1])
        for i in range(n)))
    out = tmp_path / "out.csv"
    key_file = str(tmp_path / "k.txt")
    key = [int(x) for x in rng.integers(0, 256, 40)]
    open(key_file, "w").write(":".join("%02x" % b for b in key))
    status, _, _, exc = run_main(["--key-file", key_file, "--ips-file", str(path), "--ipv6",
                                  "--htable-size", "16", "--num-queues", "4", "--csv", str(out),
                                  "--reta-weights", "1,0,2,1"], capsys)
    assert status == 0, exc
    import ipaddress
    words = np.array([[int.from_bytes(ipaddress.IPv6Address(addrs[2 * i]).packed[j:j + 4], "big")
                       for j in range(0, 16, 4)] +
                      [int.from_bytes(ipaddress.IPv6Address(addrs[2 * i + 1]).packed[j:j + 4], "big")
                       for j in range(0, 16, 4)] +
                      [int(ports[i, 0]) << 16 | int(ports[i, 1])] for i in range(n)], dtype=np.uint32)
    want = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    table = np.array(rt.weights(16, [1, 0, 2, 1]), dtype=np.uint32)
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    assert [int(x.split(",")[4]) for x in body] == want.tolist()
    assert [int(x.split(",")[5]) for x in body] == table[want % 16].tolist()
    assert 1 not in {int(x.split(",")[5]) for x in body}  # weight 0: never selected
