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
