"""More queues than hash-table buckets (VERDICT r02 "Fix the Q >= H path").

``queue = hash % htable % nqueues`` (``simulator.py:96-98``) is < min(htable, nqueues), so
with nqueues >= htable every queue is the bucket itself.  The library sizes bins, the
queue-width check and the counts it writes by min(H, Q) (max(reta) + 1 with a table), and
the Python layer sizes every count vector by ``_native.queue_modulus`` (= min(H, Q)).
Checked against the oracle's hashes with the reference's arithmetic (Python ``%``) on:
the device-pointer API (plain, single-pass, u8 queues), the raw C ABI with a caller-sized
Q-long count vector (the tail [H, Q) zeroed, or left alone with RSS_FLAG_ACCUMULATE), key
search with Q > H, and every CLI path.
"""
import ctypes
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

H = 128
QS = [129, 20000, 300000, 4 * 10 ** 9]


def _oracle_queues(oracle_lib, key, tuples, htable, nqueues):
    h, _, _ = oracle_lib.run(key, tuples, 1, 1, want_queue=False)
    q = (h.astype(object) % htable % nqueues).astype(np.int64)
    return h, q


@pytest.mark.parametrize("Q", QS)
@pytest.mark.parametrize("single_pass", [False, True])
def test_device_api_q_ge_h(Q, single_pass, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import _native
    n = (1 << 22) + 3
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    assert _native.queue_modulus(H, Q) == (H, H)
    host = oracle_lib.generate(23, 0, n)
    tuples = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    counts = torch.full((H,), -1, dtype=torch.int64, device=dev)
    ws = (torch.zeros(_native.counts_workspace_bytes(H, Q) // 8, dtype=torch.int64, device=dev)
          if single_pass else None)
    key = _native.prepare_key(example_key)
    for _ in range(2):  # the workspace is left zero for the next launch
        _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                            counts.data_ptr(), _native.FLAG_QUEUE_U8, s,
                            ws.data_ptr() if ws is not None else None)
    torch.cuda.synchronize()
    h, q = _oracle_queues(oracle_lib, example_key, host, H, Q)
    np.testing.assert_array_equal(hashes.cpu().numpy().view(np.uint32), h)
    np.testing.assert_array_equal(queues.cpu().numpy().astype(np.int64), q)
    np.testing.assert_array_equal(counts.cpu().numpy(), np.bincount(q, minlength=H))
    if ws is not None:
        assert int(ws.abs().sum()) == 0


@pytest.mark.parametrize("use_ws", [False, True])
def test_raw_abi_counts_tail(use_ws, oracle_lib, example_key):
    """A C caller that sizes counts by its nqueues (300000) gets counts[H:] zeroed (or
    untouched with RSS_FLAG_ACCUMULATE) and bins sized by H (private LDS bins, one pass)."""
    from rss_simulator_nvidia_amd import _native
    lib = _native.load()
    n, Q = (1 << 20) + 1, 300000
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    host = oracle_lib.generate(29, 0, n)
    tuples = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    counts = torch.full((Q,), 7, dtype=torch.int64, device=dev)
    ws = None
    if use_ws:
        nbytes = ctypes.c_size_t()
        assert lib.rss_counts_workspace_bytes(Q, ctypes.byref(nbytes)) == 0
        ws = torch.zeros(nbytes.value // 8, dtype=torch.int64, device=dev)
    key = _native.prepare_key(example_key)

    def call(flags):
        if ws is None:
            rc = lib.rss_hash_device(ctypes.byref(key), tuples.data_ptr(), n, H, Q, None, None,
                                     counts.data_ptr(), flags, s)
        else:
            rc = lib.rss_hash_device_ws(ctypes.byref(key), tuples.data_ptr(), n, H, Q, None,
                                        None, counts.data_ptr(), flags, ws.data_ptr(), s)
        assert rc == 0, lib.rss_last_error()

    _, q = _oracle_queues(oracle_lib, example_key, host, H, Q)
    want = np.bincount(q, minlength=H)
    call(0)
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    np.testing.assert_array_equal(c[:H], want)
    assert not c[H:].any()
    counts[H:] = 5  # accumulate: the tail is left as the caller had it
    call(_native.FLAG_ACCUMULATE)
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    np.testing.assert_array_equal(c[:H], 2 * want)
    assert (c[H:] == 5).all()


def test_key_search_q_ge_h(oracle_lib, example_key):
    """Key search rows keep the caller's nqueues stride; queues >= H stay zero."""
    from rss_simulator_nvidia_amd import _native, keysearch
    lib = _native.load()
    n, Q, nk = (1 << 18) + 5, 300, 5
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    host = oracle_lib.generate(31, 0, n)
    tuples = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    keys = keysearch.random_keys(nk, seed=3)
    win = np.stack([np.ctypeslib.as_array(_native.prepare_key(k).window) for k in keys])
    windows = torch.from_numpy(win.astype(np.uint32).view(np.int32)).to(dev)
    counts = torch.full((nk, Q), 9, dtype=torch.int64, device=dev)
    rc = lib.rss_key_search_device(windows.data_ptr(), nk, tuples.data_ptr(), n, H, Q,
                                   counts.data_ptr(), s)
    assert rc == 0, lib.rss_last_error()
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    for i, k in enumerate(keys):
        _, q = _oracle_queues(oracle_lib, k, host, H, Q)
        np.testing.assert_array_equal(c[i, :H], np.bincount(q, minlength=H))
        assert not c[i, H:].any()
    # the Python wrapper sizes the matrix [keys, min(H, Q)]
    out = torch.empty((nk, H), dtype=torch.int64, device=dev)
    _native.key_search_device(windows.data_ptr(), nk, tuples.data_ptr(), n, H, Q, out.data_ptr(), s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), c[:, :H])


PATHS = {"device": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "1"},
         "host": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "0"},
         "pandas": {"RSS_CSV_FASTPATH": "0", "RSS_CSV_DEVICE": "1"}}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("Q", QS)
def test_cli_q_ge_h(path, Q, golden_dir, tmp_path, monkeypatch):
    """The CLI on the reference's example input: queue = hash % 128 for every Q >= 128, the
    counts section lists the non-empty queues (value_counts), as the reference writes it."""
    from rss_simulator_nvidia_amd.main import main
    for k, v in PATHS[path].items():
        monkeypatch.setenv(k, v)
    out = tmp_path / "o.csv"
    main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
          "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", str(H), "--num-queues", str(Q), "--csv", str(out)])
    lines = out.read_text().splitlines()
    header = "src_ip,dst_ip,src_port,dst_port,hash_result,queue_number"
    start = lines.index(header)
    body = pd.read_csv(out, skiprows=start)
    ref_path = os.path.join(golden_dir, "example", "out_h128_q24.csv")
    ref = pd.read_csv(ref_path, skiprows=open(ref_path).read().splitlines().index(header))
    assert (body.hash_result == ref.hash_result).all()
    want_q = [int(h) % H % Q for h in body.hash_result]
    assert list(body.queue_number) == want_q
    vc = pd.Series(want_q).value_counts().sort_index()
    counts = pd.read_csv(out, nrows=start - 1)
    assert list(counts.queue_number) == list(vc.index) and list(counts.counts) == list(vc.values)


def test_histogram_counts_q_ge_h(golden_dir):
    """Histogram mode: the device counts are min(H, Q) long; the figure pads them to Q bins."""
    from rss_simulator_nvidia_amd import histogram
    from rss_simulator_nvidia_amd.simulator import Simulator
    with open(os.path.join(golden_dir, "example_input", "hash_key.txt")) as f:
        key = [int(x, 16) for x in f.read().split(":")]
    sim = Simulator(key, H, 20000)
    sim.load_ips_from_csv(os.path.join(golden_dir, "example_input", "ips.csv"))
    sim.calc_hash()
    sim.calc_queue_number()
    c = sim.queue_counts
    assert len(c) == H
    q = sim.data_frame["queue_number"].to_numpy()
    np.testing.assert_array_equal(c, np.bincount(q, minlength=H))
    import matplotlib
    matplotlib.use("Agg")
    fig = histogram.figure(c, "k", H, 20000)
    assert len(fig.axes[0].patches) == 20000
