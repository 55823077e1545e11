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
        ResidentBatch(16, key, 128, 300, device="cpu", queue_width="u8")
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
