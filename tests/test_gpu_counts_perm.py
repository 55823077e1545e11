"""Counts-only launches with a power-of-two H <= 256 run ``rss_counts_perm_kernel`` (byte
tables in registers, v_perm lookups) instead of the LDS-table kernel.  Bar: per-queue counts
bit-exact to the C oracle and to the LDS-table kernel (the hooks build's ``counts_perm=0``) on the same
inputs, over every H it takes, every queue mode (mask, identity Q >= H, FAST8), ragged tails
(n % 4 = 1..3), tiny n, key lengths that wrap, accumulation, and the shapes that must stay on
the LDS kernel (misaligned tuples, H > 256, Q > 256)."""
import numpy as np
import pytest

from hooks import hooks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


def _counts(native, key, tuples_ptr, n, H, Q, perm, accumulate_from=None):
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    flags = 0
    if accumulate_from is not None:
        counts.copy_(torch.from_numpy(accumulate_from.view(np.int64)))
        flags = native.FLAG_ACCUMULATE
    if perm:  # the product library
        native.hash_device(key, tuples_ptr, n, H, Q, None, None, counts.data_ptr(), flags, s)
    else:
        with hooks(counts_perm=0):
            native.hash_device(key, tuples_ptr, n, H, Q, None, None, counts.data_ptr(), flags, s)
    torch.cuda.synchronize()
    return counts.cpu().numpy().view(np.uint64)


HQ = [(1, 1), (2, 3), (4, 4), (8, 5), (16, 16), (32, 7), (64, 200), (128, 24), (128, 64),
      (128, 127), (256, 255), (256, 256), (256, 100), (512, 24), (128, 300)]


@pytest.mark.parametrize("H,Q", HQ)
def test_counts_equal_oracle_and_lut_kernel(native, oracle_lib, example_key, H, Q):
    n = (1 << 20) + 3
    host = oracle_lib.generate(11, 0, n)
    dev = torch.device("cuda:0")
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    key = native.prepare_key(example_key)
    _, _, want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
    got = _counts(native, key, tup.data_ptr(), n, H, Q, perm=True)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(_counts(native, key, tup.data_ptr(), n, H, Q, perm=False), want)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 4095, 4096, 4097, 4099, 1 << 14])
def test_ragged_and_tiny_batches(native, oracle_lib, example_key, n):
    host = oracle_lib.generate(5, 100, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(example_key)
    for H, Q in ((128, 24), (256, 256), (64, 9)):
        _, _, want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
        np.testing.assert_array_equal(_counts(native, key, tup.data_ptr(), n, H, Q, True), want)


@pytest.mark.parametrize("klen", [4, 7, 16, 40, 52])
def test_key_lengths(native, oracle_lib, klen):
    rng = np.random.default_rng(klen)
    kb = [int(x) for x in rng.integers(0, 256, klen)]
    n = 50003
    host = oracle_lib.generate(9, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(kb)
    for H, Q in ((128, 24), (32, 32), (256, 7)):
        _, _, want = oracle_lib.run(kb, host, H, Q, want_hash=False, want_queue=False)
        np.testing.assert_array_equal(_counts(native, key, tup.data_ptr(), n, H, Q, True), want)


def test_accumulate_and_misaligned(native, oracle_lib, example_key):
    n = 300001
    host = oracle_lib.generate(3, 0, n)
    flat = host.view(np.int32).reshape(-1)
    buf = torch.zeros(flat.size + 4, dtype=torch.int32, device="cuda:0")
    buf[1:1 + flat.size] = torch.from_numpy(flat).to("cuda:0")  # 4-byte offset: LDS kernel
    key = native.prepare_key(example_key)
    _, _, want = oracle_lib.run(example_key, host, 128, 24, want_hash=False, want_queue=False)
    mis = _counts(native, key, buf.data_ptr() + 4, n, 128, 24, True)
    np.testing.assert_array_equal(mis, want)
    aligned = torch.from_numpy(flat).to("cuda:0")
    start = np.arange(24, dtype=np.uint64) * np.uint64(1000)
    acc = _counts(native, key, aligned.data_ptr(), n, 128, 24, True, accumulate_from=start)
    np.testing.assert_array_equal(acc, want + start)


def test_flow_like_input(native, oracle_lib, example_key):
    """bench --distribution flow shape: constant fields broadcast in every v_perm byte"""
    import bench
    n = 1 << 18
    host = bench.flow_np(0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(example_key)
    _, _, want = oracle_lib.run(example_key, host, 128, 24, want_hash=False, want_queue=False)
    np.testing.assert_array_equal(_counts(native, key, tup.data_ptr(), n, 128, 24, True), want)


@pytest.mark.parametrize("H,Q", [(128, 24), (256, 256), (64, 200), (2, 3), (16, 16), (512, 24)])
@pytest.mark.parametrize("n", [1, 3, 4, 4097, (1 << 18) + 2])
def test_ipv6_counts_equal_lut_kernel(native, example_key, H, Q, n):
    """IPv6 counts only (rss_hash6_device): the register-table kernel (nine words, 108
    fields) equals the LDS-table IPv6 kernel, which the Microsoft IPv6 KAT and the oracle pin
    (tests/test_gpu_fields_ipv6.py); ragged n, every queue mode, and H > 256 (LDS kernel)."""
    rng = np.random.default_rng(n * 1000 + H + Q)
    words = torch.from_numpy(rng.integers(-2**31, 2**31, 9 * n, dtype=np.int64).astype(np.int32)).to("cuda:0")
    key6 = native.prepare_key6(example_key)
    s = torch.cuda.current_stream().cuda_stream
    got = {}
    for perm in (True, False):
        c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
        with hooks(counts_perm=int(perm)):
            native.hash6_device(key6, words.data_ptr(), n, H, Q, None, None, c.data_ptr(), 0, s)
            torch.cuda.synchronize()
        got[perm] = c.cpu().numpy()
    np.testing.assert_array_equal(got[True], got[False])
    assert int(got[True].sum()) == n
