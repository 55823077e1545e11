"""configs[3] on one GPU: 2**30 synthetic tuples (12 GiB of tuples, so every tuple past index
357,913,941 sits beyond the 4 GiB byte offset) hashed in one launch and as the eight shards
the N=8 bench hands its ranks (``sharding.shard_range``); the shards and a whole-batch launch
run counts-only (the register-table kernel), the single full-output launch the LDS-table one.

Size-independent checks (large-N parity): the shards' per-queue counts sum to
the single launch's counts and to N; the queue column equals ``hash % H % Q``
(simulator.py:94-98) and its histogram equals the counts; windows around every shard
boundary, the 4 GiB crossing and the end of the batch are element-wise equal to the C oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 1 << 30
SEED = 0x5EED
WINDOW = 1 << 16


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    assert _native.device_count() >= 1, "no gfx950 device visible to librss_toeplitz.so"
    return _native


def test_1G_tuples_single_launch_and_eight_shards(native, oracle_lib, example_key):
    from rss_simulator_nvidia_amd.sharding import shard_range
    H, Q, world = 128, 24, 8
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    key = native.prepare_key(example_key)
    tuples = torch.empty(3 * N, dtype=torch.int32, device=dev)
    hashes = torch.empty(N, dtype=torch.int32, device=dev)
    queues = torch.empty(N, dtype=torch.uint8, device=dev)
    counts = torch.empty(Q, dtype=torch.int64, device=dev)
    native.generate_device(SEED, 0, N, tuples.data_ptr(), s)
    native.hash_device(key, tuples.data_ptr(), N, H, Q, hashes.data_ptr(), queues.data_ptr(),
                       counts.data_ptr(), native.FLAG_QUEUE_U8, s)
    shard_counts = []
    for rank in range(world):
        start, count = shard_range(N, rank, world)
        c = torch.empty(Q, dtype=torch.int64, device=dev)
        native.hash_device(key, tuples.data_ptr() + 12 * start, count, H, Q, None, None,
                           c.data_ptr(), 0, s)
        shard_counts.append(c)
    # the whole batch counts-only in one launch (rss_counts_perm_kernel, 2^30 tuples)
    whole = torch.empty(Q, dtype=torch.int64, device=dev)
    native.hash_device(key, tuples.data_ptr(), N, H, Q, None, None, whole.data_ptr(), 0, s)
    torch.cuda.synchronize()

    total = counts.cpu().numpy().view(np.uint64)
    assert int(total.sum()) == N
    summed = sum(c.cpu().numpy().view(np.uint64) for c in shard_counts)
    np.testing.assert_array_equal(summed, total)
    np.testing.assert_array_equal(whole.cpu().numpy().view(np.uint64), total)

    # element-wise against the oracle around shard boundaries, 4 GiB and the end
    starts = {0, N - WINDOW, (1 << 32) // 12 - WINDOW // 2}
    for rank in range(1, world):
        starts.add(shard_range(N, rank, world)[0] - WINDOW // 2)
    for a in sorted(starts):
        host = oracle_lib.generate(SEED, a, WINDOW)
        np.testing.assert_array_equal(
            tuples[3 * a:3 * (a + WINDOW)].cpu().numpy().view(np.uint32).reshape(WINDOW, 3), host)
        ho, qo, _ = oracle_lib.run(example_key, host, H, Q)
        np.testing.assert_array_equal(hashes[a:a + WINDOW].cpu().numpy().view(np.uint32), ho)
        np.testing.assert_array_equal(queues[a:a + WINDOW].cpu().numpy(), qo.astype(np.uint8))
    del tuples
    torch.cuda.empty_cache()

    # whole batch: queue == hash % H % Q, and the queue histogram equals the counts
    hist = np.zeros(Q, dtype=np.uint64)
    step = 1 << 27
    for a in range(0, N, step):
        h = hashes[a:a + step].cpu().numpy().view(np.uint32)
        q = queues[a:a + step].cpu().numpy()
        np.testing.assert_array_equal(q, ((h % H) % Q).astype(np.uint8))
        hist += np.bincount(q, minlength=Q).astype(np.uint64)
    np.testing.assert_array_equal(hist, total)
