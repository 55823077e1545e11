"""The bench's exact timed launch at full size, element by element.

``bench.py``'s step is one ``rss_hash_device_ws`` launch (single-pass counts, u8 queue
column) over 2^28 resident tuples placed by ``ResidentBatch``, H = 128, Q = 24 (BASELINE
configs[2]).  Here the same launch -- same buffers, same flags, the workspace reused launch
after launch as the bench reuses it -- is compared with the C oracle on every one of the
2^28 tuples (hash_result, queue_number) and on the counts (``simulator.py:94-113``), and
with the committed per-block digests bench.py checks after its timed region.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SEED, N, H, Q = 0x5EED, 1 << 28, 128, 24


def test_bench_launch_2p28_elementwise(oracle_lib, example_key):
    import bench
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    key = _native.prepare_key(example_key)
    batch = ResidentBatch(N, key, H, Q, device=dev, queue_width="u8", placement=(2, 3),
                          fill=lambda t: _native.generate_device(SEED, 0, N, t.data_ptr(), sp),
                          stream=stream)
    pipe = CountsPipeline(Q, dev, single_pass=True, htable=H)

    def launch(c, workspace):  # bench.py's launch(), verbatim in effect
        _native.hash_device(key, batch.tuples.data_ptr(), N, H, Q, batch.hashes.data_ptr(),
                            batch.queues.data_ptr(), c.data_ptr(), _native.FLAG_QUEUE_U8, sp,
                            workspace.data_ptr())

    for _ in range(6):  # several launches on one workspace, alternating count buffers
        counts = pipe.step(launch)
    counts = pipe.drain()
    torch.cuda.synchronize()
    assert int(pipe.workspace.abs().sum()) == 0  # left zero for the next launch

    tup = oracle_lib.generate(SEED, 0, N)
    h, q, c = oracle_lib.run(example_key, tup, H, Q, fn="oracle_run_tables")
    del tup
    got_h = batch.hashes.cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(got_h != h)
    assert bad.size == 0, "hash mismatches at %s" % bad[:8]
    got_q = batch.queue_view().cpu().numpy()
    bad = np.flatnonzero(got_q != q.astype(np.uint8))
    assert bad.size == 0, "queue mismatches at %s" % bad[:8]
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), c)
    # the literal rotating restatement on a sample of the same launch (incl. the 4 GiB-past
    # byte offsets of the input at the end of the batch)
    for first in (0, N - (1 << 16)):
        t = oracle_lib.generate(SEED, first, 1 << 16)
        ho, qo, _ = oracle_lib.run(example_key, t, H, Q, fn="oracle_run")
        np.testing.assert_array_equal(got_h[first:first + (1 << 16)], ho)
        np.testing.assert_array_equal(got_q[first:first + (1 << 16)], qo.astype(np.uint8))
    # what bench.py checks after its timed region
    gold = bench.load_digest()
    v = bench.verify_outputs(torch, gold, batch.hashes, batch.queue_view(), 0, N)
    assert v["ok"] is True and v["blocks"] == N >> 20, v
    assert [int(x) for x in counts.tolist()] == bench.golden_counts(gold, 0, N)

    # RSS_FLAG_ADDR64 (the placement probe's and the clock settle's launches: 64-bit
    # addressing, a kernel symbol of its own) writes the same bytes, plain and single-pass
    h32, q32 = batch.hashes.clone(), batch.queues.clone()
    for ws in (None, pipe.workspace):
        batch.hashes.zero_()
        batch.queues.fill_(0xFF)
        c64 = torch.zeros(Q, dtype=torch.int64, device=dev)
        _native.hash_device(key, batch.tuples.data_ptr(), N, H, Q, batch.hashes.data_ptr(),
                            batch.queues.data_ptr(), c64.data_ptr(),
                            _native.FLAG_QUEUE_U8 | _native.FLAG_ADDR64 |
                            (_native.FLAG_ACCUMULATE if ws is None else 0), sp,
                            ws.data_ptr() if ws is not None else None)
        torch.cuda.synchronize()
        assert torch.equal(batch.hashes, h32) and torch.equal(batch.queues, q32)
        np.testing.assert_array_equal(c64.cpu().numpy().view(np.uint64), c)
    assert int(pipe.workspace.abs().sum()) == 0
