"""Placement of the resident stream buffers (``placement.choose_stream_buffers``): every
candidate combination is probed with the real kernel, the fastest is returned, the
returned input holds the generated tuples, and the kernel on the chosen buffers gives the
oracle's results."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def test_choose_stream_buffers_probes_and_keeps_the_fastest(oracle_lib, example_key):
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.placement import choose_stream_buffers
    n, H, Q = (1 << 20) + 3, 128, 24
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    key = _native.prepare_key(example_key)
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    seen = []

    def fill(t):
        _native.generate_device(0x5EED, 0, n, t.data_ptr(), stream.cuda_stream)

    def probe(t, h, q, ev):
        seen.append((t.data_ptr(), h.data_ptr(), q.data_ptr()))
        if ev is not None:
            ev[0].record(stream)
        _native.hash_device(key, t.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(),
                            counts.data_ptr(), _native.FLAG_QUEUE_U8, stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)

    tuples, hashes, queues, rep = choose_stream_buffers(torch, dev, n, fill, probe, n_inputs=2,
                                                        n_outputs=3, probe_reps=4, probe_warm=1)
    assert len(set(seen)) == 6 and len(seen) == 6 * 5
    times = rep["probe_median_ms"]
    assert set(times) == {"in%d_out%d" % (i, j) for i in range(2) for j in range(3)}
    assert round(rep["chosen_ms"], 4) == min(times.values()) == times[rep["chosen"]]
    assert tuples.numel() == 3 * n and hashes.numel() == n and queues.numel() == n
    hashes.zero_()
    _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                        counts.data_ptr(), _native.FLAG_QUEUE_U8, stream.cuda_stream)
    torch.cuda.synchronize()
    tup = tuples.cpu().numpy().view(np.uint32).reshape(n, 3)
    np.testing.assert_array_equal(tup, oracle_lib.generate(0x5EED, 0, n))
    h, q, c = oracle_lib.run(example_key, tup, H, Q)
    np.testing.assert_array_equal(hashes.cpu().numpy().view(np.uint32), h)
    np.testing.assert_array_equal(queues.cpu().numpy(), q.astype(np.uint8))
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), c)


@pytest.mark.parametrize("width,placement", [("auto", (2, 3)), ("u16", (1, 1)), ("u32", (1, 2))])
def test_resident_batch_equals_oracle(oracle_lib, example_key, width, placement):
    """ResidentBatch: placed buffers, then batch after batch on the same buffers -- every
    pass gives the oracle's hash / queue / counts, overwritten or accumulated."""
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    n, H, Q = (1 << 18) + 5, 512, 64
    dev = torch.device("cuda:0")
    key = _native.prepare_key(example_key)
    s = torch.cuda.current_stream(dev).cuda_stream
    batch = ResidentBatch(n, key, H, Q, device=dev, queue_width=width, placement=placement,
                          fill=lambda t: _native.generate_device(7, 0, n, t.data_ptr(), s))
    assert batch.report["candidates"] == {"inputs": placement[0], "outputs": placement[1]}
    counts = torch.full((Q,), 12345, dtype=torch.int64, device=dev)
    for first in (0, n):  # a second batch written by the caller into the same input
        _native.generate_device(7, first, n, batch.tuples.data_ptr(), s)
        batch.hash(counts)
        batch.hash(counts, accumulate=True)
        torch.cuda.synchronize()
        tup = oracle_lib.generate(7, first, n)
        h, q, c = oracle_lib.run(example_key, tup, H, Q)
        np.testing.assert_array_equal(batch.hashes.cpu().numpy().view(np.uint32), h)
        qv = batch.queue_view().cpu().numpy()
        qv = qv.view({1: np.uint8, 2: np.uint16, 4: np.uint32}[qv.itemsize])
        np.testing.assert_array_equal(qv.astype(np.uint32), q)
        np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), 2 * c)
    assert int(batch.workspace.abs().sum()) == 0  # single-pass workspace left zero


def test_counts_pipeline_steps_a_resident_batch(oracle_lib, example_key):
    """INTEGRATION.md's loop: ``CountsPipeline.step(batch.hash)`` -- single-pass counts on the
    pipeline's workspace, batch after batch -- gives each batch's oracle counts."""
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    n, H, Q = (1 << 18) + 3, 128, 24
    dev = torch.device("cuda:0")
    key = _native.prepare_key(example_key)
    s = torch.cuda.current_stream(dev).cuda_stream
    batch = ResidentBatch(n, key, H, Q, device=dev, placement=(1, 2))
    pipe = CountsPipeline(Q, dev, htable=H)
    assert pipe.workspace is not None
    for first in (0, n, 2 * n, 0):
        _native.generate_device(11, first, n, batch.tuples.data_ptr(), s)
        counts = pipe.step(batch.hash)
        torch.cuda.synchronize()
        want = oracle_lib.run(example_key, oracle_lib.generate(11, first, n), H, Q,
                              want_hash=False, want_queue=False)[2]
        np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), want)
    np.testing.assert_array_equal(pipe.drain().cpu().numpy().view(np.uint64), want)
    assert int(pipe.workspace.abs().sum()) == 0



def test_choose_buffer_keeps_the_fastest_candidate():
    from rss_simulator_nvidia_amd.placement import choose_buffer
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    seen = []

    def probe(buf, ev):
        seen.append(buf.data_ptr())
        if ev is not None:
            ev[0].record(s)
        buf.fill_(7)
        if ev is not None:
            ev[1].record(s)

    buf, times = choose_buffer(torch, dev, 1 << 20, probe, candidates=3, probe_reps=3,
                               probe_warm=1)
    assert len(set(seen)) == 3 and len(seen) == 12 and buf.data_ptr() in seen
    assert buf.numel() == 1 << 20 and buf.dtype == torch.uint8 and set(times) == {"buf0", "buf1", "buf2"}
