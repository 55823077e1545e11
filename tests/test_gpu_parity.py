"""GPU parity: the gfx950 kernel (through the C ABI) vs the reference's goldens and the oracle.

Bar: bit-exact hash_result / queue_number / per-queue counts (integer work).
Small cases compare against fixtures produced by the reference itself; large
cases compare element-wise against the C oracle (pinned to the same fixtures by
tests/test_oracle.py) and, at the full 2**28 size, through size-independent
properties (count totals, per-queue counts, hash digests).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")  # loud: never silently skip on the box
    assert _native.device_count() >= 1, "no gfx950 device visible to librss_toeplitz.so"
    return _native


@pytest.fixture(scope="module")
def ctx(native):
    return native.HostContext(0)


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


# ----------------------------------------------------------- golden fixtures --
def test_random_golden_four_keys(native, ctx, random_golden):
    g = random_golden
    for k, key in enumerate(g["key_list"]):
        h, q, c = ctx.hash(native.prepare_key(key), g["tuples"], 128, 24)
        np.testing.assert_array_equal(h, g["hashes"][k])


def test_sweep_against_reference_simulator(native, ctx, random_golden):
    g = random_golden
    key = native.prepare_key(g["key_list"][0])
    for j, (H, Q) in enumerate(g["sweep"]):
        h, q, c = ctx.hash(key, g["tuples"], int(H), int(Q))
        np.testing.assert_array_equal(h, g["hashes"][0])
        np.testing.assert_array_equal(q, g["sweep_queue"][j])
        ref = g["sweep_counts"]["%d,%d" % (H, Q)]
        assert [[int(a), int(c[a])] for a in np.flatnonzero(c)] == ref
        assert int(c.sum()) == len(h)


def test_ms_kat_and_one_hot(native, ctx, golden_dir, example_key):
    with open(os.path.join(golden_dir, "ms_kat.json")) as f:
        kat = json.load(f)
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    ms_key = [int(x, 16) for x in kat["key"].split(":")]
    t = Toeplitz(ms_key)
    for v in kat["vectors"]:
        assert t.compute_hash(v["src_ip"], v["dst_ip"], v["src_port"], v["dst_port"]) == v["hash"]
    d = np.load(os.path.join(golden_dir, "one_hot.npz"), allow_pickle=False)
    rows = d["tuples"]
    ports = ((rows[:, 2] & 0xFFFF) << 16 | (rows[:, 3] & 0xFFFF)).astype(np.uint32)
    tup = np.stack([rows[:, 0], rows[:, 1], ports], axis=1).astype(np.uint32)
    for k, key in enumerate([example_key, ms_key]):
        h, _, _ = ctx.hash(native.prepare_key(key), tup, 1, 1)
        np.testing.assert_array_equal(h, d["hashes"][k])


def test_key_lengths_and_short_keys(native, ctx, oracle_lib):
    rng = np.random.default_rng(11)
    tup = rng.integers(0, 2**32, (3000, 3), dtype=np.uint64).astype(np.uint32)
    for length in (4, 7, 15, 16, 40, 52, 64):
        key = [int(x) for x in rng.integers(0, 256, length)]
        h, _, _ = ctx.hash(native.prepare_key(key), tup, 1, 1)
        want = [oracle_lib.hash_rotating(key, int(a), int(b), int(p) >> 16, int(p) & 0xFFFF)
                for a, b, p in tup[:300]]
        np.testing.assert_array_equal(h[:300], np.array(want, dtype=np.uint32))
        if length >= 16:
            ho, _, _ = oracle_lib.run(key, tup, 1, 1)
            np.testing.assert_array_equal(h, ho)


# ---------------------------------------------------------- kernel variants --
MODULO_CASES = [
    (128, 24), (512, 8), (512, 64), (100, 7), (1, 1), (7, 7), (8, 100), (1000, 1000),
    (65536, 1000), (65537, 1000), (100000, 7), (2**31, 3), (2**32 - 1, 65535),
    (4096, 256), (4096, 257), (50000, 8192), (50000, 8193), (2**32 - 5, 2**16 + 3),
]


@pytest.mark.parametrize("H,Q", MODULO_CASES)
def test_modulo_and_histogram_paths(native, ctx, oracle_lib, example_key, H, Q):
    # covers mask / fast16 / fast32 queue modes and private / shared / global bins
    tup = oracle_lib.generate(H * 31 + Q, 0, 200003)
    key = native.prepare_key(example_key)
    h, q, c = ctx.hash(key, tup, H, Q)
    ho, qo, co = oracle_lib.run(example_key, tup, H, Q)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    qn = min(H, Q)  # the counts vector is min(H, Q) long: queues >= H never occur
    assert len(c) == qn and not co[qn:].any()
    np.testing.assert_array_equal(c, co[:qn])


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 63, 64, 65, 1023, 4097, 4 * 1024 * 512 + 3])
def test_ragged_sizes(native, ctx, oracle_lib, example_key, n):
    tup = oracle_lib.generate(77, 5, n)
    h, q, c = ctx.hash(native.prepare_key(example_key), tup, 512, 24)
    ho, qo, co = oracle_lib.run(example_key, tup, 512, 24)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)


def test_device_api_alignment_nulls_accumulate(native, oracle_lib, example_key):
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    n = 100001
    key = native.prepare_key(example_key)
    tup_host = oracle_lib.generate(9, 0, n)
    ho, qo, co = oracle_lib.run(example_key, tup_host, 128, 24)
    raw = torch.from_numpy(tup_host.view(np.int32).reshape(-1)).to(dev)
    # misaligned input (4-byte offset) forces the scalar-load variant
    shifted = torch.empty(3 * n + 1, dtype=torch.int32, device=dev)
    shifted[1:] = raw
    for src in (raw, shifted[1:]):
        hashes = torch.full((n + 1,), -1, dtype=torch.int32, device=dev)
        queues = torch.full((n + 1,), -1, dtype=torch.int32, device=dev)
        counts = torch.full((24,), 7, dtype=torch.int64, device=dev)
        native.hash_device(key, src.data_ptr(), n, 128, 24, hashes[1:].data_ptr(),
                           queues.data_ptr(), counts.data_ptr(), 0, s)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_u32(hashes[1:]), ho)
        np.testing.assert_array_equal(_u32(queues[:n]), qo)
        assert int(queues[n]) == -1 and int(hashes[0]) == -1  # no out-of-range writes
        np.testing.assert_array_equal(_u64(counts), co)
    # NULL outputs + accumulate
    counts = torch.zeros(24, dtype=torch.int64, device=dev)
    for _ in range(3):
        native.hash_device(key, raw.data_ptr(), n, 128, 24, None, None, counts.data_ptr(),
                           native.FLAG_ACCUMULATE, s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), 3 * co)
    # n == 0 zeroes counts and launches nothing
    native.hash_device(key, raw.data_ptr(), 0, 128, 24, None, None, counts.data_ptr(), 0, s)
    torch.cuda.synchronize()
    assert int(counts.sum()) == 0


def test_invalid_arguments_fail_cleanly(native, example_key):
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    key = native.prepare_key(example_key)
    with pytest.raises(DeviceError, match="must be >= 1"):
        native.hash_device(key, 0, 10, 0, 24)
    with pytest.raises(DeviceError, match="tuples is NULL"):
        native.hash_device(key, None, 10, 128, 24)


# ----------------------------------------------------------- large sizes -----
def test_16M_bit_exact_vs_oracle(native, oracle_lib, example_key):
    """BASELINE configs[1]: 16M synthetic tuples, bit-exact hash_result / queue_number."""
    n, H, Q = 1 << 24, 128, 24
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(Q, dtype=torch.int64, device=dev)
    key = native.prepare_key(example_key)
    native.generate_device(0x5EED, 0, n, tuples.data_ptr(), s)
    native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                       counts.data_ptr(), 0, s)
    torch.cuda.synchronize()
    host = oracle_lib.generate(0x5EED, 0, n)
    np.testing.assert_array_equal(_u32(tuples).reshape(n, 3), host)
    ho, qo, co = oracle_lib.run(example_key, host, H, Q, threads=16)
    np.testing.assert_array_equal(_u32(hashes), ho)
    np.testing.assert_array_equal(_u32(queues), qo)
    np.testing.assert_array_equal(_u64(counts), co)


def test_256M_sweep_counts_and_digest(native, oracle_lib, example_key):
    """configs[2]/[4]: 2**28 tuples, queues x htable sweep -- per-queue counts must equal
    the oracle's, and hash digests (sum, xor) must match over the whole batch."""
    n = 1 << 28
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    key = native.prepare_key(example_key)
    native.generate_device(0x5EED, 0, n, tuples.data_ptr(), s)
    native.hash_device(key, tuples.data_ptr(), n, 1, 1, hashes.data_ptr(), None, None, 0, s)
    torch.cuda.synchronize()
    host = oracle_lib.generate(0x5EED, 0, n)
    ho, _, _ = oracle_lib.run(example_key, host, 1, 1, threads=16, want_queue=False)
    del host
    dh = _u32(hashes)
    np.testing.assert_array_equal(dh, ho)
    for H in (128, 512):
        for Q in (8, 16, 24, 64):
            counts = torch.empty(Q, dtype=torch.int64, device=dev)
            native.hash_device(key, tuples.data_ptr(), n, H, Q, None, None, counts.data_ptr(), 0, s)
            torch.cuda.synchronize()
            want = np.bincount(((ho % H) % Q).astype(np.int64), minlength=Q).astype(np.uint64)
            np.testing.assert_array_equal(_u64(counts), want)
            assert int(want.sum()) == n


@pytest.mark.parametrize("width,flag_name,dtype", [("u8", "FLAG_QUEUE_U8", np.uint8),
                                                   ("u16", "FLAG_QUEUE_U16", np.uint16)])
@pytest.mark.parametrize("H,Q", [(128, 24), (512, 256), (100, 7), (65536, 1000)])
def test_narrow_queue_outputs(native, oracle_lib, example_key, width, flag_name, dtype, H, Q):
    if width == "u8" and Q > 256:
        pytest.skip("u8 holds at most 256 queues")
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    n = 65537
    key = native.prepare_key(example_key)
    tup_host = oracle_lib.generate(H + Q, 0, n)
    _, qo, co = oracle_lib.run(example_key, tup_host, H, Q)
    raw = torch.from_numpy(tup_host.view(np.int32).reshape(-1)).to(dev)
    item = np.dtype(dtype).itemsize
    for offset in (0, item):  # aligned (4-tuple stores) and misaligned (scalar stores)
        buf = torch.full((n * item + 64,), 0xAB, dtype=torch.uint8, device=dev)
        counts = torch.empty(Q, dtype=torch.int64, device=dev)
        native.hash_device(key, raw.data_ptr(), n, H, Q, None, buf.data_ptr() + offset,
                           counts.data_ptr(), getattr(native, flag_name), s)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        np.testing.assert_array_equal(got[offset:offset + n * item].view(dtype), qo.astype(dtype))
        assert (got[:offset] == 0xAB).all() and (got[offset + n * item:] == 0xAB).all()
        np.testing.assert_array_equal(_u64(counts), co)


def test_narrow_queue_rejects_overflowing_queue_count(native, example_key):
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    key = native.prepare_key(example_key)
    with pytest.raises(DeviceError, match="QUEUE_U8"):
        native.hash_device(key, 0, 0, 1024, 257, None, None, None, native.FLAG_QUEUE_U8)


def test_graph_capture_and_replay(native, oracle_lib, example_key):
    """rss_hash_device is stream-ordered and capture-safe: capture zero + hash in a HIP
    graph, replay it on changing inputs, results match the oracle each time."""
    dev = torch.device("cuda:0")
    n, H, Q = 300001, 512, 24
    key = native.prepare_key(example_key)
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.empty(n, dtype=torch.uint8, device=dev)
    counts = torch.empty(Q, dtype=torch.int64, device=dev)

    def body():
        counts.zero_()
        native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                           counts.data_ptr(), native.FLAG_ACCUMULATE | native.FLAG_QUEUE_U8,
                           torch.cuda.current_stream(dev).cuda_stream)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream(dev).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for seed in (1, 2, 3):
        host = oracle_lib.generate(seed, 0, n)
        tuples.copy_(torch.from_numpy(host.view(np.int32).reshape(-1)))
        g.replay()
        torch.cuda.synchronize()
        ho, qo, co = oracle_lib.run(example_key, host, H, Q)
        np.testing.assert_array_equal(_u32(hashes), ho)
        np.testing.assert_array_equal(queues.cpu().numpy(), qo.astype(np.uint8))
        np.testing.assert_array_equal(_u64(counts), co)


def test_concurrent_streams_and_keys(native, oracle_lib, example_key):
    """Two keys on two streams at once (independent launches share nothing)."""
    dev = torch.device("cuda:0")
    n = 1 << 20
    keys = [example_key, list(range(40))]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    host = oracle_lib.generate(5, 0, n)
    tuples = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    outs = []
    for k, s in zip(keys, streams):
        h = torch.empty(n, dtype=torch.int32, device=dev)
        c = torch.empty(24, dtype=torch.int64, device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        native.hash_device(native.prepare_key(k), tuples.data_ptr(), n, 128, 24, h.data_ptr(),
                           None, c.data_ptr(), 0, s.cuda_stream)
        outs.append((h, c))
    torch.cuda.synchronize()
    for k, (h, c) in zip(keys, outs):
        ho, _, co = oracle_lib.run(k, host, 128, 24)
        np.testing.assert_array_equal(_u32(h), ho)
        np.testing.assert_array_equal(_u64(c), co)


@pytest.mark.parametrize("H,Q", [(128, 24), (512, 64), (65536, 1000)])
def test_flow_like_distribution_vs_oracle(native, oracle_lib, example_key, H, Q):
    """SURVEY.md 8(d)'s flow-like input (bench.py --distribution flow: one IP pair,
    sequential source ports), built on the device exactly as the bench builds it."""
    import bench
    n = (1 << 22) + 7
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    bench.flow_device(torch, tuples, 12345, n, dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(Q, dtype=torch.int64, device=dev)
    native.hash_device(native.prepare_key(example_key), tuples.data_ptr(), n, H, Q,
                       hashes.data_ptr(), queues.data_ptr(), counts.data_ptr(), 0, s)
    torch.cuda.synchronize()
    host = bench.flow_np(12345, n)
    np.testing.assert_array_equal(_u32(tuples).reshape(n, 3), host)
    ho, qo, co = oracle_lib.run(example_key, host, H, Q, threads=16)
    np.testing.assert_array_equal(_u32(hashes), ho)
    np.testing.assert_array_equal(_u32(queues), qo)
    np.testing.assert_array_equal(_u64(counts), co)
