"""ResidentBatch argument checks (CPU: refused before any device allocation)."""
import pytest

pytest.importorskip("torch")


def test_resident_batch_refuses_bad_sizes(example_key):
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.resident import ResidentBatch, narrowest_queue_width
    key = _native.prepare_key(example_key)
    with pytest.raises(ValueError):
        ResidentBatch(0, key, 128, 24, device="cpu")
    with pytest.raises(ValueError):
        ResidentBatch(16, key, 1024, 300, device="cpu", queue_width="u8")  # 300 queues
    with pytest.raises(ValueError):
        ResidentBatch(16, key, 128, 24, device="cpu", queue_width="u64")
    with pytest.raises(ValueError):
        ResidentBatch(16, key, 128, 24, device="cpu", queue_width="u32", queue_bytes=2)
    assert [narrowest_queue_width(q) for q in (1, 256, 257, 65536, 65537)] == \
        ["u8", "u8", "u16", "u16", "u32"]


def test_placement_takes_fewer_candidates_when_memory_runs_out():
    """choose_stream_buffers on a fake device that runs out of memory after 5 allocations:
    the probe continues with the candidates that fit (2 inputs, then the outputs that fit)
    instead of failing; the first candidate of each kind must still fit."""
    import types

    import pytest

    from rss_simulator_nvidia_amd.placement import choose_stream_buffers

    class OOM(RuntimeError):
        pass

    class Buf:
        def __init__(self, n):
            self.n = n

    class Event:
        def __init__(self, enable_timing=True):
            pass

        def elapsed_time(self, other):
            return 1.0

    def make_fake(limit):
        count = {"n": 0}

        def empty(n, dtype=None, device=None):
            count["n"] += 1
            if count["n"] > limit:
                raise OOM("out of memory")
            return Buf(n)

        cuda = types.SimpleNamespace(OutOfMemoryError=OOM, synchronize=lambda dev=None: None,
                                     empty_cache=lambda: None, Event=Event)
        return types.SimpleNamespace(empty=empty, int32="i4", uint8="u1", cuda=cuda)

    probed = []
    fake = make_fake(limit=5)  # 2 inputs + 1.5 output pairs fit
    t, h, q, rep = choose_stream_buffers(fake, "dev", 10, lambda b: None,
                                         lambda *a: probed.append(a), n_inputs=2, n_outputs=8)
    assert rep["candidates"] == {"inputs": 2, "outputs": 1}
    with pytest.raises(OOM):  # not even one input fits: the caller's error, unchanged
        choose_stream_buffers(make_fake(limit=0), "dev", 10, lambda b: None, lambda *a: None)


def _timed_fake(times_of_output):
    """Fake torch whose probe launch time is times_of_output(k) for the k-th output
    hash buffer allocated (ids in allocation order)."""
    import types

    class OOM(RuntimeError):
        pass

    class Buf:
        def __init__(self, n, dtype, ident):
            self.n, self.dtype, self.ident = n, dtype, ident

    class Event:
        def __init__(self, enable_timing=True):
            self.t = 0.0

        def elapsed_time(self, other):
            return other.t - self.t

    count = {"hash": 0}

    def empty(n, dtype=None, device=None):
        ident = None
        if dtype == "i4" and n == 10:  # an output hash buffer (inputs are 3n)
            ident = count["hash"]
            count["hash"] += 1
        return Buf(n, dtype, ident)

    cuda = types.SimpleNamespace(OutOfMemoryError=OOM, synchronize=lambda dev=None: None,
                                 empty_cache=lambda: None, Event=Event)
    fake = types.SimpleNamespace(empty=empty, int32="i4", uint8="u1", cuda=cuda)

    def probe(t, h, q, ev):
        if ev is not None:
            ev[1].t = times_of_output(h.ident)
    return fake, probe


@pytest.mark.parametrize("fast_at,max_rounds,want_rounds", [
    (3, 3, 1),      # a fast-tier candidate in the first round: no more rounds
    (15, 3, 2),     # first round all slow, the second finds one
    (None, 3, 3),   # no fast tier on the box: every round probed, the best slow set kept
    (15, 1, 1),     # one round requested: no retry
    ("mid", 3, 2)])  # first round slow + middle tier (best/slowest 0.92): probe on
def test_placement_rounds_until_a_faster_tier(fast_at, max_rounds, want_rounds):
    from rss_simulator_nvidia_amd.placement import choose_stream_buffers
    if fast_at == "mid":  # outputs 0-5 slow, 6-11 middle tier, 12-23 with one fast set (17)
        fake, probe = _timed_fake(lambda k: 0.879 if k < 6 else (0.785 if k == 17 else 0.808))
        t, h, q, rep = choose_stream_buffers(fake, "dev", 10, lambda b: None, probe, n_inputs=2,
                                             n_outputs=12, max_rounds=max_rounds)
        assert rep["rounds"] == want_rounds and h.ident == 17 and rep["chosen_ms"] == 0.785
        return
    fake, probe = _timed_fake(lambda k: 0.785 if k == fast_at else 0.865 + 0.001 * (k % 3))
    t, h, q, rep = choose_stream_buffers(fake, "dev", 10, lambda b: None, probe, n_inputs=2,
                                         n_outputs=12, max_rounds=max_rounds)
    assert rep["rounds"] == want_rounds
    assert rep["candidates"] == {"inputs": 2, "outputs": 12 * want_rounds}
    if fast_at is not None and fast_at < 12 * want_rounds:
        assert h.ident == fast_at and rep["chosen_ms"] == 0.785
    else:
        assert rep["chosen_ms"] == 0.865
