"""GPU parity for key search: every key's per-queue counts == the single-key kernel
and the oracle, across modulo / histogram modes, ragged sizes and misaligned input."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


@pytest.mark.parametrize("H,Q,n", [(128, 24, 100003), (512, 64, 65536), (100, 7, 4097),
                                   (65536, 1000, 30001), (100000, 7, 20000), (50000, 10000, 9999),
                                   (1, 1, 5), (128, 24, 0),
                                   # packed-bucket kernel: 8 keys / entry (H <= 256), 4 keys
                                   # (H <= 65536), its bin-budget edges and the fallbacks past them
                                   (256, 40, 70001), (256, 41, 7001), (16, 24, 33333), (2, 3, 999),
                                   (256, 255, 5000), (65536, 80, 40003), (1024, 81, 4001),
                                   (4096, 64, 12345), (128, 1, 777), (128, 64, 5555), (256, 80, 6000),
                                   (256, 81, 3000),
                                   # round 4 (packed kernel on 5.25 KiB of conflict-free
                                   # tables): its new budget edges -- 8 keys to Q = 154, 4 keys
                                   # to 309 -- and the pair kernel's private / shared bin edge
                                   (256, 154, 7001), (256, 155, 6003), (65536, 309, 8001),
                                   (1024, 310, 5003), (1000, 160, 4001), (1000, 161, 4001)])
def test_key_search_matches_oracle(native, oracle_lib, H, Q, n):
    from rss_simulator_nvidia_amd import keysearch
    keys = keysearch.random_keys(19, seed=H + Q) + [[int(x) for x in range(52)]]
    tuples = oracle_lib.generate(H * 7 + n, 0, n)
    counts = native.HostContext(0).key_search([native.prepare_key(k) for k in keys], tuples, H, Q)
    qn = min(H, Q)  # queues >= H never occur: rows are min(H, Q) long (_native.queue_modulus)
    assert counts.shape == (len(keys), qn)
    for k, key in enumerate(keys):
        _, _, c = oracle_lib.run(key, tuples, H, Q)
        assert not c[qn:].any()
        np.testing.assert_array_equal(counts[k], c[:qn])


def test_key_search_device_api_misaligned(native, oracle_lib):
    from rss_simulator_nvidia_amd import keysearch
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    keys = keysearch.random_keys(70, seed=1)
    n, H, Q = 123457, 128, 24
    host = oracle_lib.generate(3, 0, n)
    raw = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    shifted = torch.empty(3 * n + 1, dtype=torch.int32, device=dev)
    shifted[1:] = raw
    windows = torch.from_numpy(np.stack([np.ctypeslib.as_array(native.prepare_key(k).window)
                                         for k in keys]).astype(np.uint32).view(np.int32)).to(dev)
    for src in (raw, shifted[1:]):
        counts = torch.full((len(keys), Q), 5, dtype=torch.int64, device=dev)
        native.key_search_device(windows.data_ptr(), len(keys), src.data_ptr(), n, H, Q,
                                 counts.data_ptr(), s)
        torch.cuda.synchronize()
        got = counts.cpu().numpy().view(np.uint64)
        for k in (0, 17, 69):
            np.testing.assert_array_equal(got[k], oracle_lib.run(keys[k], host, H, Q)[2])
        assert (got.sum(axis=1) == n).all()


def test_search_end_to_end_improves_on_example_key(native, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import keysearch
    tuples = oracle_lib.generate(11, 0, 200000)
    ranked = keysearch.search(tuples, 128, 24, n_keys=256, seed=2, top=3, extra_keys=[example_key])
    base = keysearch.balance(oracle_lib.run(example_key, tuples, 128, 24)[2], 128, 24)
    assert ranked[0]["max_load"] <= base["max_load"][0]
    np.testing.assert_array_equal(ranked[0]["counts"],
                                  oracle_lib.run(ranked[0]["key"], tuples, 128, 24)[2])


@pytest.mark.parametrize("nkeys", [1, 3, 7, 9, 17])
@pytest.mark.parametrize("H,Q", [(128, 24), (512, 2000), (512, 24)])
def test_key_search_odd_key_counts_flow_input(native, oracle_lib, nkeys, H, Q):
    """Keys share 8-byte table entries (8 / 4 keys by packed buckets, else pairs); a
    partial last group repeats its last key and the copies are discarded.  Flow-like tuples (one IP pair, sequential
    source ports -- bench.py --distribution flow) exercise broadcast / strided LDS reads."""
    import bench
    from rss_simulator_nvidia_amd import keysearch
    keys = keysearch.random_keys(nkeys, seed=nkeys * 31 + Q)
    tuples = bench.flow_np(777, 50021)
    counts = native.HostContext(0).key_search([native.prepare_key(k) for k in keys], tuples, H, Q)
    qn = min(H, Q)
    assert counts.shape == (nkeys, qn)
    for k, key in enumerate(keys):
        c = oracle_lib.run(key, tuples, H, Q)[2]
        assert not c[qn:].any()
        np.testing.assert_array_equal(counts[k], c[:qn])


def test_bench_key_search_launch_matches_oracle(native, oracle_lib):
    """The bench's row_f_kernels.key_search launch exactly (bench.py extra_lines): 1024 random
    keys (keysearch.random_keys seed 0) x 2^20 device-generated tuples (seed 1), H = 128,
    Q = 24, one rss_key_search_device launch -- every key's 24 counts against the oracle."""
    from rss_simulator_nvidia_amd import keysearch
    nk, nt = 1024, 1 << 20
    keys = keysearch.random_keys(nk, seed=0)
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    win = np.stack([np.ctypeslib.as_array(native.prepare_key(k).window) for k in keys])
    windows = torch.from_numpy(win.astype(np.uint32).view(np.int32)).to(dev)
    tup = torch.empty(3 * nt, dtype=torch.int32, device=dev)
    native.generate_device(1, 0, nt, tup.data_ptr(), sp)
    kc = torch.empty((nk, 24), dtype=torch.int64, device=dev)
    native.key_search_device(windows.data_ptr(), nk, tup.data_ptr(), nt, 128, 24, kc.data_ptr(), sp)
    torch.cuda.synchronize()
    got = kc.cpu().numpy().view(np.uint64)
    host = oracle_lib.generate(1, 0, nt)
    np.testing.assert_array_equal(tup.cpu().numpy().view(np.uint32).reshape(nt, 3), host)
    for k in range(nk):
        _, _, c = oracle_lib.run(keys[k], host, 128, 24, threads=16, want_hash=False,
                                 want_queue=False)
        np.testing.assert_array_equal(got[k], c, err_msg="key %d" % k)
