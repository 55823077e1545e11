"""Single-pass counts and the balanced tail on the IPv6 kernel (``rss_hash6_device_ws``).

The IPv6 counterpart of ``tests/test_gpu_single_pass.py``: the launch writes the counts
itself from a caller-owned workspace that every launch leaves zero, and launches
of >= 16 grid rows (2^24 tuples) hand their last rows out per workgroup slot.  Results are
those of ``rss_hash6_device`` (pinned by the Microsoft IPv6 vectors and the oracle in
``tests/test_gpu_fields_ipv6.py``): hash, ``hash % H % Q`` and its ``value_counts``
(``simulator.py:94-113`` on the 36-byte input).
"""
import ctypes

import numpy as np
import pytest

from hooks import hooks
from oracle import oracle as o

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    return _native


def _workspace(native, H, Q, dev):
    return torch.zeros(native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)


@pytest.mark.parametrize("H,Q,n,width", [(128, 24, 100003, "u8"), (100, 7, 4099, "u32"),
                                         (65536, 1000, 20001, "u16"), (128, 129, 7777, "u8"),
                                         (512, 64, 0, "u32"), (1, 1, 3, "u32"),
                                         (50000, 10000, 3001, "u32")])
def test_ipv6_single_pass_vs_oracle(native, oracle_lib, H, Q, n, width):
    """Full outputs and counts of the ws launch against the oracle; stale counts are
    overwritten, the workspace is left zero, RSS_FLAG_ACCUMULATE adds (last case: more
    queues than LDS bins -- the launch histograms in ranges and ignores the workspace)."""
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(H * 7 + n)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    words = rng.integers(0, 2**32, (max(n, 1), 9), dtype=np.uint64).astype(np.uint32)[:n]
    want = o.hash_words_np(oracle_lib.windows_n(key, 288), words)
    qo, co = o.queue_and_counts(want, H, Q)
    qn = min(H, Q)
    assert not co[qn:].any()
    co = co[:qn]  # count vectors are min(H, Q) long (_native.queue_modulus)
    raw = torch.from_numpy(words.view(np.int32).reshape(-1)).to(dev) if n else \
        torch.empty(9, dtype=torch.int32, device=dev)
    k6 = native.prepare_key6(key)
    dt = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32}[width]
    flag = {"u8": native.FLAG_QUEUE_U8, "u16": native.FLAG_QUEUE_U16, "u32": 0}[width]
    item = np.dtype(dt).itemsize
    ws = _workspace(native, H, Q, dev)
    hashes = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    queues = torch.empty(max(n, 1) * item, dtype=torch.uint8, device=dev)
    counts = torch.full((qn,), 99, dtype=torch.int64, device=dev)
    for _ in range(3):  # one workspace, launch after launch
        native.hash6_device(k6, raw.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                            counts.data_ptr(), flag, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(hashes[:n].cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(queues[:n * item].cpu().numpy().view(dt), qo.astype(dt))
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), co)
    assert int(ws.abs().sum()) == 0
    native.hash6_device(k6, raw.data_ptr(), n, H, Q, None, None, counts.data_ptr(),
                        native.FLAG_ACCUMULATE, s, ws.data_ptr())  # counts only, accumulating
    torch.cuda.synchronize()
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), 2 * co)
    assert int(ws.abs().sum()) == 0


def test_ipv6_single_pass_needs_workspace(native):
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    lib = native.load()
    k6 = native.prepare_key6(list(range(40)))
    rc = lib.rss_hash6_device_ws(ctypes.byref(k6), None, 0, 128, 24, None, None, 8, 0,
                                 None, None)
    assert rc == -22 and b"workspace" in lib.rss_last_error()
    with pytest.raises(DeviceError):
        native.hash6_device(k6, 0, 0, 128, 24, None, None, 8, 0, None, 12)  # misaligned


@pytest.mark.parametrize("n", [(1 << 24) + 5, (1 << 25) + 4 * 1024 + 3])
def test_ipv6_balanced_tail_equals_static(native, oracle_lib, n):
    """Launches of >= 16 rows take the balanced tail: every output equals the static
    grid-stride launch's (the hooks build's balance=0) and the plain launch's, the counts equal, balanced
    and static launches alternate on one workspace, and sampled hashes equal the oracle."""
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    raw = torch.randint(-2**31, 2**31 - 1, (9 * n,), dtype=torch.int32, device=dev, generator=g)
    key = list(range(7, 47))
    k6 = native.prepare_key6(key)
    H, Q = 128, 24
    ws = _workspace(native, H, Q, dev)
    ref_h = torch.empty(n, dtype=torch.int32, device=dev)
    ref_q = torch.empty(n, dtype=torch.uint8, device=dev)
    ref_c = torch.empty(Q, dtype=torch.int64, device=dev)
    native.hash6_device(k6, raw.data_ptr(), n, H, Q, ref_h.data_ptr(), ref_q.data_ptr(),
                        ref_c.data_ptr(), native.FLAG_QUEUE_U8, s)  # plain, static walk
    h = torch.empty_like(ref_h)
    q = torch.empty_like(ref_q)
    c = torch.empty_like(ref_c)
    for balance in (1, 0, 1, 1, 0):
        h.zero_()
        q.fill_(0xFF)
        with hooks(balance=balance):
            native.hash6_device(k6, raw.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(),
                                c.data_ptr(), native.FLAG_QUEUE_U8, s, ws.data_ptr())
            torch.cuda.synchronize()
        assert torch.equal(h, ref_h) and torch.equal(q, ref_q) and torch.equal(c, ref_c), balance
        assert int(ws.abs().sum()) == 0
    assert int(ref_c.sum()) == n
    words = raw.cpu().numpy().view(np.uint32).reshape(n, 9)
    idx = np.concatenate([np.arange(4096), np.arange(n - 4096, n),
                          np.random.default_rng(1).integers(0, n, 8192)])
    want = o.hash_words_np(oracle_lib.windows_n(key, 288), words[idx])
    np.testing.assert_array_equal(ref_h.cpu().numpy().view(np.uint32)[idx], want)
    np.testing.assert_array_equal(ref_q.cpu().numpy()[idx], ((want % H) % Q).astype(np.uint8))
