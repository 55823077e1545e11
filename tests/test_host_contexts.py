"""Host-side logic of the multi-GPU option of the reference API (CPU, no device): the
IPv6 split of ``MultiHostContext.hash6`` (the contiguous ranges of ``rss_hash_host_multi``
/ ``sharding.shard_range``, each range written in place, counts summed, a worker's error
re-raised on the caller), ``host_context``'s routing and caching, and the ``devices=``
plumbing of ``Simulator`` / ``Toeplitz``.  The device results are checked against the
oracle in ``tests/test_gpu_concurrency.py``."""
import threading

import numpy as np
import pandas as pd
import pytest

from rss_simulator_nvidia_amd import _native


class _FakeCtx:
    """Stands in for a HostContext: hash = row sum of the words, queue = hash % Q."""

    def __init__(self, fail=False):
        self.calls, self.fail = [], fail
        self.threads = set()

    def hash6(self, key6, arr, htable, nqueues, want_hash=True, want_queue=True,
              want_counts=True, reta=None, out=None):
        self.threads.add(threading.get_ident())
        if self.fail:
            raise _native.DeviceError("boom")
        self.calls.append(len(arr))
        h = arr.view(np.uint32).reshape(len(arr), 9).astype(np.uint64).sum(axis=1).astype(np.uint32)
        q = h % nqueues
        counts = np.bincount(q, minlength=nqueues).astype(np.uint64) if want_counts else None
        if out is not None:  # written in place, like HostContext.hash6
            for dst, src in zip(out, (h, q)):
                if dst is not None:
                    assert dst.shape == src.shape and dst.flags.c_contiguous
                    dst[:] = src
            return out[0], out[1], counts
        return h if want_hash else None, q if want_queue else None, counts


def _multi(ctxs):
    m = object.__new__(_native.MultiHostContext)
    m.contexts = ctxs
    return m


@pytest.mark.parametrize("n,k", [(0, 2), (1, 3), (2, 2), (10, 3), (1001, 4)])
def test_hash6_split_matches_one_context(n, k):
    rng = np.random.default_rng(n + k)
    words = rng.integers(0, 2**32, size=(n, 9), dtype=np.uint64).astype(np.uint32)
    ctxs = [_FakeCtx() for _ in range(k)]
    h, q, c = _multi(ctxs).hash6(None, words, 64, 5)
    h1, q1, c1 = _FakeCtx().hash6(None, words, 64, 5)
    np.testing.assert_array_equal(h, h1)
    np.testing.assert_array_equal(q, q1)
    np.testing.assert_array_equal(c, c1)
    base, extra = divmod(n, k)
    assert [x.calls[0] for x in ctxs] == [base + (i < extra) for i in range(k)]
    me = threading.get_ident()  # context 0 on the caller, the others on worker threads
    assert ctxs[0].threads == {me} and all(me not in x.threads for x in ctxs[1:])


def test_hash6_split_output_subsets_and_errors():
    words = np.arange(90, dtype=np.uint32).reshape(10, 9)
    h, q, c = _multi([_FakeCtx(), _FakeCtx()]).hash6(None, words, 64, 5, want_hash=False,
                                                      want_queue=False)
    assert h is None and q is None and int(c.sum()) == 10
    with pytest.raises(_native.DeviceError, match="boom"):
        _multi([_FakeCtx(), _FakeCtx(fail=True)]).hash6(None, words, 64, 5)


def test_host_context_routing(monkeypatch):
    made = []

    class FakeMulti:
        def __init__(self, devices):
            made.append(devices)

    monkeypatch.setattr(_native, "MultiHostContext", FakeMulti)
    monkeypatch.setattr(_native, "_multi_ctx", {})
    sentinel = object()
    monkeypatch.setattr(_native, "default_context", lambda: sentinel)
    assert _native.host_context(None) is sentinel
    a = _native.host_context([0, 1])
    assert _native.host_context((0, 1)) is a  # cached per device tuple
    b = _native.host_context([0, 0, 0])
    assert b is not a and made == [(0, 1), (0, 0, 0)]
    with pytest.raises(ValueError):
        _native.host_context([])


def test_simulator_passes_devices_through(monkeypatch, example_key):
    """Simulator(devices=...) -> Toeplitz.compute_queues(..., devices) -> host_context."""
    from rss_simulator_nvidia_amd.simulator import Simulator
    seen = []

    class Ctx:
        def hash(self, key, tuples, H, Q, reta=None):
            n = len(tuples)
            return (np.arange(n, dtype=np.uint32), np.arange(n, dtype=np.uint32) % Q,
                    np.bincount(np.arange(n) % Q, minlength=Q).astype(np.uint64))

    monkeypatch.setattr(_native, "host_context", lambda devices=None: seen.append(devices) or Ctx())
    monkeypatch.setattr(_native, "prepare_key", lambda key, fields=15: None)
    df = pd.DataFrame({"src_ip": ["1.2.3.4"] * 3, "dst_ip": ["5.6.7.8"] * 3,
                       "src_port": [1, 2, 3], "dst_port": [4, 5, 6]})
    for devices, want in ((None, None), ([0, 0], (0, 0))):
        sim = Simulator(example_key, 128, 24, devices=devices)
        sim.load_frame(df.copy())
        sim.calc_hash()
        assert seen[-1] == want


def test_simulator_rejects_an_empty_device_list(example_key):
    from rss_simulator_nvidia_amd.simulator import Simulator
    with pytest.raises(ValueError):
        Simulator(example_key, 128, 24, devices=[])
