"""Single-pass counts (``rss_hash_device_ws``): the launch writes the per-queue counts
itself from a caller-owned workspace (each queue's last arriving add writes its count), so a batch needs no zeroing launch before
it.  Bar: hash / queue / counts bit-exact to the C oracle (the ``value_counts`` of
``simulator.py:107-113``) and to ``rss_hash_device`` on the same inputs, over the kernels
that take the workspace (LDS-table kernel with private and shared bins, the register-table
counts-only kernel, 4-tuple and 1-tuple lanes) and the shapes that do not (many queues);
overwrite and RSS_FLAG_ACCUMULATE; one-workgroup grids; n = 0; the workspace left zero after
every launch and reused over many launches, HIP-graph replay and two streams at once."""
import contextlib

import numpy as np
import pytest

from hooks import hooks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

DEV = "cuda:0"


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


def _dev_tuples(host, offset_bytes=0):
    """Packed tuples on the device, starting `offset_bytes` into the allocation."""
    raw = host.view(np.uint8).reshape(-1)
    buf = torch.empty(len(raw) + 16, dtype=torch.uint8, device=DEV)
    buf[offset_bytes:offset_bytes + len(raw)].copy_(torch.from_numpy(raw))
    return buf, buf.data_ptr() + offset_bytes


def _ws(native, H, Q):
    nbytes = native.counts_workspace_bytes(H, Q)
    assert nbytes == 8 * (min(H, Q) + 2)  # spare (ticket fold), sums, balanced-tail counter
    return torch.zeros(nbytes // 8, dtype=torch.int64, device=DEV)


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


# (H, Q, outputs): private bins (Q <= 256), shared bins (Q up to 8192), the counts-only
# register-table kernel (power-of-two H <= 256, no outputs), non-power-of-two H / Q
CASES = [(128, 24, True), (128, 24, False), (512, 24, True), (256, 256, False),
         (1000, 7, True), (4096, 1000, True), (65536, 8000, True), (100000, 3, False),
         (16, 16, False), (1, 1, True)]


@pytest.mark.parametrize("H,Q,outputs", CASES)
def test_single_pass_equals_oracle(native, oracle_lib, example_key, H, Q, outputs):
    n = (1 << 20) + 5
    host = oracle_lib.generate(21, 0, n)
    want_h, want_q, want_c = oracle_lib.run(example_key, host, H, Q)
    _buf, tp = _dev_tuples(host)
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    h = torch.empty(n, dtype=torch.int32, device=DEV) if outputs else None
    q = torch.empty(n, dtype=torch.int32, device=DEV) if outputs else None
    ws = _ws(native, H, Q)
    counts = torch.full((Q,), 12345, dtype=torch.int64, device=DEV)  # overwritten
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    native.hash_device(key, tp, n, H, Q, ptr(h), ptr(q), counts.data_ptr(), 0, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), want_c)
    assert int(ws.abs().sum()) == 0
    if outputs:
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), want_h)
        np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), want_q)
    # accumulate: adds this batch's counts to what the buffer holds
    base = np.arange(Q, dtype=np.uint64) * 1000003
    counts.copy_(torch.from_numpy(base.view(np.int64)))
    native.hash_device(key, tp, n, H, Q, ptr(h), ptr(q), counts.data_ptr(),
                       native.FLAG_ACCUMULATE, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), base + want_c)
    assert int(ws.abs().sum()) == 0


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 4096, 4099, 65537])
@pytest.mark.parametrize("outputs", [True, False])
def test_small_grids(native, oracle_lib, example_key, n, outputs):
    """One to a few workgroups: the last-workgroup hand-off with gridDim 1 and ragged tails."""
    H, Q = 128, 24
    host = oracle_lib.generate(5, 7, n)
    _, _, want_c = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
    _buf, tp = _dev_tuples(host)
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    ws = _ws(native, H, Q)
    counts = torch.full((Q,), -1, dtype=torch.int64, device=DEV)
    h = torch.empty(n, dtype=torch.int32, device=DEV) if outputs else None
    native.hash_device(key, tp, n, H, Q, h.data_ptr() if outputs else None, None,
                       counts.data_ptr(), 0, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), want_c)
    assert int(ws.abs().sum()) == 0


def test_zero_tuples_overwrites_with_zeros(native, example_key):
    key = native.prepare_key(example_key)
    ws = _ws(native, 128, 24)
    counts = torch.full((24,), 77, dtype=torch.int64, device=DEV)
    native.hash_device(key, None, 0, 128, 24, None, None, counts.data_ptr(), 0,
                       torch.cuda.current_stream().cuda_stream, ws.data_ptr())
    torch.cuda.synchronize()
    assert int(counts.abs().sum()) == 0
    native.hash_device(key, None, 0, 128, 24, None, None, counts.data_ptr(),
                       native.FLAG_ACCUMULATE, torch.cuda.current_stream().cuda_stream,
                       ws.data_ptr())
    torch.cuda.synchronize()
    assert int(counts.abs().sum()) == 0


@pytest.mark.parametrize("offset,qflag", [(4, 0), (0, "u8"), (0, "u16"), (12, "u8")])
def test_unaligned_and_narrow_queues(native, oracle_lib, example_key, offset, qflag):
    """1-tuple lanes (misaligned input) and u8 / u16 queue outputs take the workspace too."""
    n, H, Q = (1 << 18) + 3, 128, 24
    host = oracle_lib.generate(9, 0, n)
    want_h, want_q, want_c = oracle_lib.run(example_key, host, H, Q)
    _keep, tp = _dev_tuples(host, offset)
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    dtype, flag = {0: (torch.int32, 0), "u8": (torch.uint8, native.FLAG_QUEUE_U8),
                   "u16": (torch.int16, native.FLAG_QUEUE_U16)}[qflag]
    h = torch.empty(n, dtype=torch.int32, device=DEV)
    q = torch.empty(n, dtype=dtype, device=DEV)
    ws = _ws(native, H, Q)
    counts = torch.full((Q,), 5, dtype=torch.int64, device=DEV)
    native.hash_device(key, tp, n, H, Q, h.data_ptr(), q.data_ptr(), counts.data_ptr(), flag, s,
                       ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), want_c)
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), want_h)
    got_q = q.cpu().numpy().astype(np.int64) & {0: 0xFFFFFFFF, "u8": 0xFF, "u16": 0xFFFF}[qflag]
    np.testing.assert_array_equal(got_q, want_q.astype(np.int64))
    assert int(ws.abs().sum()) == 0


def test_many_queues_leave_workspace_untouched(native, oracle_lib, example_key):
    """More queues than LDS bins: the range passes zero the counts as rss_hash_device does."""
    n, H, Q = 1 << 18, 1 << 20, 20000
    host = oracle_lib.generate(3, 0, n)
    _, _, want_c = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
    _buf, tp = _dev_tuples(host)
    key = native.prepare_key(example_key)
    ws = _ws(native, H, Q)
    counts = torch.full((Q,), 9, dtype=torch.int64, device=DEV)
    native.hash_device(key, tp, n, H, Q, None, None, counts.data_ptr(), 0,
                       torch.cuda.current_stream().cuda_stream, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_u64(counts), want_c)
    assert int(ws.abs().sum()) == 0


def test_workspace_reused_over_many_batches(native, oracle_lib, example_key):
    """40 launches back to back on one workspace, alternating outputs / counts only and
    overwrite / accumulate: each batch's counts exact."""
    n, H, Q = (1 << 19) + 1, 128, 24
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    batches = []
    for i in range(3):
        host = oracle_lib.generate(40 + i, 0, n)
        batches.append((_dev_tuples(host), oracle_lib.run(example_key, host, H, Q,
                                                          want_hash=False, want_queue=False)[2]))
    ws = _ws(native, H, Q)
    h = torch.empty(n, dtype=torch.int32, device=DEV)
    outs = [torch.empty(Q, dtype=torch.int64, device=DEV) for _ in range(40)]
    for i, c in enumerate(outs):
        (_, tp), _ = batches[i % 3]
        native.hash_device(key, tp, n, H, Q, h.data_ptr() if i % 2 else None, None, c.data_ptr(),
                           0, s, ws.data_ptr())
    acc = torch.zeros(Q, dtype=torch.int64, device=DEV)
    for i in range(6):
        (_, tp), _ = batches[i % 3]
        native.hash_device(key, tp, n, H, Q, None, None, acc.data_ptr(), native.FLAG_ACCUMULATE,
                           s, ws.data_ptr())
    torch.cuda.synchronize()
    for i, c in enumerate(outs):
        np.testing.assert_array_equal(_u64(c), batches[i % 3][1])
    np.testing.assert_array_equal(_u64(acc), 2 * sum(b[1] for b in batches))
    assert int(ws.abs().sum()) == 0


def test_graph_replay(native, oracle_lib, example_key):
    """A captured rss_hash_device_ws launch is one graph node; replays overwrite the counts."""
    n, H, Q = 1 << 20, 128, 24
    host = oracle_lib.generate(8, 0, n)
    _, _, want_c = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
    _keep, tp = _dev_tuples(host)
    key = native.prepare_key(example_key)
    ws = _ws(native, H, Q)
    h = torch.empty(n, dtype=torch.int32, device=DEV)
    q = torch.empty(n, dtype=torch.uint8, device=DEV)
    counts = torch.zeros(Q, dtype=torch.int64, device=DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g):
            native.hash_device(key, tp, n, H, Q, h.data_ptr(), q.data_ptr(), counts.data_ptr(),
                               native.FLAG_QUEUE_U8, torch.cuda.current_stream().cuda_stream,
                               ws.data_ptr())
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(5):
        counts.fill_(3)
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_u64(counts), want_c)
    assert int(ws.abs().sum()) == 0


def test_two_streams_two_workspaces(native, oracle_lib, example_key):
    """Concurrent launches on two streams, each with its own workspace."""
    n, H, Q = (1 << 20) + 2, 128, 24
    key = native.prepare_key(example_key)
    hosts = [oracle_lib.generate(60 + i, 0, n) for i in range(2)]
    wants = [oracle_lib.run(example_key, x, H, Q, want_hash=False, want_queue=False)[2]
             for x in hosts]
    dev_t = [_dev_tuples(x) for x in hosts]
    streams = [torch.cuda.Stream() for _ in range(2)]
    wss = [_ws(native, H, Q) for _ in range(2)]
    counts = [torch.empty(Q, dtype=torch.int64, device=DEV) for _ in range(2)]
    torch.cuda.synchronize()
    for _ in range(4):
        for i in range(2):
            native.hash_device(key, dev_t[i][1], n, H, Q, None, None, counts[i].data_ptr(), 0,
                               streams[i].cuda_stream, wss[i].data_ptr())
    torch.cuda.synchronize()
    for i in range(2):
        np.testing.assert_array_equal(_u64(counts[i]), wants[i])
        assert int(wss[i].abs().sum()) == 0


def test_workspace_required_with_counts(native, example_key):
    """rss_hash_device_ws refuses a NULL or misaligned workspace when counts are wanted,
    before any device work; without counts the workspace is not used."""
    key = native.prepare_key(example_key)
    counts = torch.zeros(24, dtype=torch.int64, device=DEV)
    ws = _ws(native, 128, 24)
    s = torch.cuda.current_stream().cuda_stream
    lib = native.load()
    import ctypes
    rc = lib.rss_hash_device_ws(ctypes.byref(key), None, 0, 128, 24, None, None,
                                counts.data_ptr(), 0, None, s)
    assert rc == -22  # RSS_EINVAL
    assert b"workspace" in lib.rss_last_error()
    with pytest.raises(native.DeviceError, match="workspace"):
        native.hash_device(key, None, 0, 128, 24, None, None, counts.data_ptr(), 0, s,
                           ws.data_ptr() + 4)
    native.hash_device(key, None, 0, 128, 24, None, None, None, 0, s, 0)


def test_stress_one_workspace_many_launches(native, oracle_lib, example_key):
    """1800 back-to-back launches on one workspace over batches of 1000, 2^20 + 3 and 2^22
    tuples (grids of one and of every CU), with and without per-tuple outputs: every launch's
    counts exact (``tools/ws_stress.py`` runs the same at 6300 launches)."""
    H, Q = 128, 24
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    batches = []
    for seed, n in ((1, 1000), (2, (1 << 20) + 3), (3, 1 << 22)):
        host = oracle_lib.generate(seed, 0, n)
        want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)[2]
        batches.append((n, torch.from_numpy(host.view(np.int32).reshape(-1)).to(DEV), want))
    ws = _ws(native, H, Q)
    h = torch.empty(1 << 22, dtype=torch.int32, device=DEV)
    outs = torch.zeros((600, Q), dtype=torch.int64, device=DEV)
    for _ in range(3):
        for i in range(600):
            n, t, _ = batches[i % 3]
            native.hash_device(key, t.data_ptr(), n, H, Q, h.data_ptr() if i % 2 else None, None,
                               outs[i].data_ptr(), 0, s, ws.data_ptr())
        got = outs.cpu().numpy().view(np.uint64)
        for i in range(600):
            np.testing.assert_array_equal(got[i], batches[i % 3][2])
        outs.zero_()
    assert int(ws.abs().sum()) == 0


@pytest.mark.parametrize("n", [1 << 24, (1 << 24) + 4099, 3 * (1 << 23) + 5, (1 << 25) + 1234567])
def test_balanced_tail_equals_oracle(native, oracle_lib, example_key, n):
    """Single-pass launches of >= 16 grid rows hand their last ~1/10 of the rows out per
    workgroup slot (the balanced tail): every tuple is hashed exactly once --
    hashes and u8 queues element-wise equal to the oracle, counts exact, launch after launch
    on one workspace (left zero, its tail counter included) -- and equal to the static
    grid-stride launch (the hooks build's balance=0) on the same buffers."""
    H, Q = 128, 24
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    host = oracle_lib.generate(41, 0, n)
    h_want, q_want, c_want = oracle_lib.run(example_key, host, H, Q, fn="oracle_run_tables")
    t = torch.from_numpy(host.view(np.int32).reshape(-1)).to(DEV)
    ws = _ws(native, H, Q)
    hashes = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    queues = torch.full((n,), 255, dtype=torch.uint8, device=DEV)
    outs = torch.zeros((12, Q), dtype=torch.int64, device=DEV)
    for i in range(12):
        # launches 6..8: static ones (hooks build) on the same workspace in between
        with hooks(balance=0) if 6 <= i < 9 else contextlib.nullcontext():
            native.hash_device(key, t.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                               outs[i].data_ptr(), native.FLAG_QUEUE_U8, s, ws.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(hashes.cpu().numpy().view(np.uint32), h_want)
    np.testing.assert_array_equal(queues.cpu().numpy(), q_want.astype(np.uint8))
    got = outs.cpu().numpy().view(np.uint64)
    for i in range(12):
        np.testing.assert_array_equal(got[i], c_want)
    assert int(ws.abs().sum()) == 0


def test_balanced_tail_stress(native, oracle_lib, example_key):
    """300 back-to-back balanced single-pass launches of 2^24 + 3 tuples (and 300 of a
    small batch in between, whose launches keep the static loop) on one workspace: every
    launch's counts exact."""
    H, Q = 128, 24
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    batches = []
    for seed, n in ((5, (1 << 24) + 3), (6, 4099)):
        host = oracle_lib.generate(seed, 0, n)
        want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False,
                              fn="oracle_run_tables")[2]
        batches.append((n, torch.from_numpy(host.view(np.int32).reshape(-1)).to(DEV), want))
    ws = _ws(native, H, Q)
    h = torch.empty((1 << 24) + 3, dtype=torch.int32, device=DEV)
    outs = torch.zeros((600, Q), dtype=torch.int64, device=DEV)
    for i in range(600):
        n, t, _ = batches[i % 2]
        native.hash_device(key, t.data_ptr(), n, H, Q, h.data_ptr() if i % 4 < 2 else None,
                           None, outs[i].data_ptr(), 0, s, ws.data_ptr())
    got = outs.cpu().numpy().view(np.uint64)
    for i in range(600):
        np.testing.assert_array_equal(got[i], batches[i % 2][2])
    assert int(ws.abs().sum()) == 0


@pytest.mark.parametrize("n", [(1 << 25) + 5, (1 << 26) + 4097])
def test_balanced_tail_counts_only(native, oracle_lib, example_key, n):
    """Counts-only single-pass launches (the register-table kernel, two workgroups per CU)
    keep the static walk (the balanced tail measured 5 % slower there): counts exact over
    40 launches on one workspace of a workspace that full-output launches also use for their
    tail counter, with static launches (the hooks build's balance=0) in between."""
    H, Q = 128, 24
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    host = oracle_lib.generate(43, 0, n)
    want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False,
                          fn="oracle_run_tables")[2]
    t = torch.from_numpy(host.view(np.int32).reshape(-1)).to(DEV)
    ws = _ws(native, H, Q)
    outs = torch.zeros((40, Q), dtype=torch.int64, device=DEV)
    for i in range(40):
        with hooks(balance=0) if 5 <= i % 10 < 8 else contextlib.nullcontext():
            native.hash_device(key, t.data_ptr(), n, H, Q, None, None, outs[i].data_ptr(), 0, s,
                               ws.data_ptr())
    got = outs.cpu().numpy().view(np.uint64)
    for i in range(40):
        np.testing.assert_array_equal(got[i], want)
    assert int(ws.abs().sum()) == 0
