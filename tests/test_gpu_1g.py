"""configs[3] on one GPU, pinned to the oracle: 2**30 synthetic tuples (12 GiB of tuples, so
every tuple past index 357,913,941 sits beyond the 4 GiB byte offset), launched exactly as
``bench.py``'s configs[3] block launches them -- ``ResidentBatch`` buffers, u8 queues,
``CountsPipeline(bucket=1, single_pass=True)`` steps (``rss_hash_device_ws``: single-pass
counts, balanced tail, the 64-bit kernel instance) -- and as the eight ``shard_range`` shards
the N=8 bench hands its ranks, each a single-pass launch of its own.

Every check is against the C oracle (``tests/golden/bench_digest.npz``, made by
``tests/golden/make_bench_digest.py`` with the literal rotating loop): all 1024 per-2^20-block
hash / queue digests of the whole batch and of every shard, the batch's counts and every
shard's counts (``golden_counts``), plus element-wise windows around each shard boundary, the
4 GiB crossing and the end against the oracle run here.  Matches ``simulator.py:94-113``.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 1 << 30
SEED, H, Q, WORLD = 0x5EED, 128, 24, 8
WINDOW = 1 << 16


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    assert _native.device_count() >= 1, "no gfx950 device visible to librss_toeplitz.so"
    return _native


def _counts(t):
    return [int(x) & ((1 << 64) - 1) for x in t.tolist()]


def test_configs3_launch_vs_oracle_digests(native, oracle_lib, example_key):
    import bench
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    from rss_simulator_nvidia_amd.sharding import CountsPipeline, shard_range
    gold = bench.load_digest()
    assert gold is not None and int(gold["total"]) >= N
    assert bench.digest_applies(gold, example_key, H, Q, "uniform")
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    key = native.prepare_key(example_key)
    batch = ResidentBatch(N, key, H, Q, device=dev, queue_width="u8", placement=(1, 2),
                          fill=lambda t: native.generate_device(SEED, 0, N, t.data_ptr(), sp),
                          stream=stream)

    # bench.py run_configs3 at world size 1: one launch per batch, one histogram per batch
    pipe = CountsPipeline(Q, dev, single_pass=True, htable=H, bucket=1)
    for _ in range(3):
        pipe.step(lambda c, workspace: batch.hash(counts=c, workspace=workspace))
    last = pipe.drain()
    torch.cuda.synchronize()
    assert int(pipe.workspace.abs().sum()) == 0  # every launch leaves the workspace zero
    v = bench.verify_outputs(torch, gold, batch.hashes, batch.queue_view(), 0, N)
    assert v["ok"] is True and v["blocks"] == 1024, v
    assert _counts(last) == bench.golden_counts(gold, 0, N)

    # element-wise against the literal loop at the shard boundaries, 4 GiB and the end
    got_h = batch.hashes
    got_q = batch.queue_view()
    starts = {0, N - WINDOW, (1 << 32) // 12 - WINDOW // 2}
    for rank in range(1, WORLD):
        starts.add(shard_range(N, rank, WORLD)[0] - WINDOW // 2)
    for a in sorted(starts):
        host = oracle_lib.generate(SEED, a, WINDOW)
        ho, qo, _ = oracle_lib.run(example_key, host, H, Q, fn="oracle_run")
        np.testing.assert_array_equal(got_h[a:a + WINDOW].cpu().numpy().view(np.uint32), ho)
        np.testing.assert_array_equal(got_q[a:a + WINDOW].cpu().numpy(), qo.astype(np.uint8))

    # the eight shards of the N=8 bench, each one single-pass launch over its range of the
    # same resident arrays (outputs cleared first, so every shard must write its own range)
    batch.hashes.zero_()
    batch.queues.fill_(0xFF)
    ws = pipe.workspace
    shard_counts = []
    for rank in range(WORLD):
        start, count = shard_range(N, rank, WORLD)
        c = torch.full((Q,), -1, dtype=torch.int64, device=dev)  # stale: overwritten
        native.hash_device(key, batch.tuples.data_ptr() + 12 * start, count, H, Q,
                           batch.hashes.data_ptr() + 4 * start, batch.queues.data_ptr() + start,
                           c.data_ptr(), native.FLAG_QUEUE_U8, sp, ws.data_ptr())
        shard_counts.append((start, count, c))
    torch.cuda.synchronize()
    assert int(ws.abs().sum()) == 0
    for start, count, c in shard_counts:
        want = bench.golden_counts(gold, start, count)
        assert want is not None and _counts(c) == want, (start, count)
        vs = bench.verify_outputs(torch, gold, batch.hashes[start:start + count],
                                  got_q[start:start + count], start, count)
        assert vs["ok"] is True and vs["blocks"] == count >> 20, (start, vs)

    # the whole batch counts-only in one launch (rss_counts_perm_kernel over 2^30 tuples)
    whole = torch.empty(Q, dtype=torch.int64, device=dev)
    native.hash_device(key, batch.tuples.data_ptr(), N, H, Q, None, None, whole.data_ptr(), 0, sp)
    torch.cuda.synchronize()
    assert _counts(whole) == bench.golden_counts(gold, 0, N)
