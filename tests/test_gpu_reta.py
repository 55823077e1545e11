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
