"""sharding.CountsPipeline on the GPU (no process group): the two count buffers alternate,
so every step's counts must be exactly that step's histogram -- never a leftover of the
step two earlier -- and the previous step's counts must still hold when the next step has
been issued -- with single-pass counts (rss_hash_device_ws, the default on a GPU) and with
a zeroing launch before each pass.  (A three-buffer variant that zeroed the next buffer on a side stream measured
20 us per step of cross-stream overhead against 7 us for zeroing in line; not adopted.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("single_pass", [True, False])
def test_counts_pipeline_steps_equal_oracle(oracle_lib, example_key, single_pass):
    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    n, H, Q = (1 << 20) + 1, 128, 24
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    key = _native.prepare_key(example_key)
    batches = []
    for i in range(4):  # four different batches, used round-robin
        host = oracle_lib.generate(100 + i, 0, n)
        batches.append((torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev),
                        oracle_lib.run(example_key, host, H, Q, want_hash=False,
                                       want_queue=False)[2]))
    pipe = CountsPipeline(Q, dev, single_pass=single_pass, htable=H)
    assert (pipe.workspace is not None) == single_pass
    prev = None
    for i in range(11):
        tup, want = batches[i % 4]
        if single_pass:  # rss_hash_device_ws overwrites the buffer: no zeroing launch
            launch = lambda counts, workspace, tup=tup: _native.hash_device(  # noqa: E731
                key, tup.data_ptr(), n, H, Q, None, None, counts.data_ptr(), 0, s,
                workspace.data_ptr())
        else:
            launch = lambda counts, tup=tup: _native.hash_device(  # noqa: E731
                key, tup.data_ptr(), n, H, Q, None, None, counts.data_ptr(),
                _native.FLAG_ACCUMULATE, s)
        c = pipe.step(launch)
        if prev is not None:  # step i-1's counts are still valid after step i is issued
            torch.cuda.synchronize()
            np.testing.assert_array_equal(prev[0].cpu().numpy().view(np.uint64), prev[1])
        prev = (c, want)
    last = pipe.drain()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(last.cpu().numpy().view(np.uint64), batches[10 % 4][1])
    if single_pass:  # every launch leaves the workspace zero
        assert int(pipe.workspace.abs().sum()) == 0
