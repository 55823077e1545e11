"""Sharded path with the HIP kernel: world-2 ``gloo`` group, both ranks on cuda:0 (the
box has one GPU; the driver's 8-GPU run uses RCCL).  Each rank generates its contiguous
shard on the device and runs ``sharding.hash_shard``; the concatenated hashes and the
all-reduced counts must equal the oracle on the whole stream (sharded ==
single-device, exactly)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, key, n_total, htable, nqueues, out_dir):
    import torch.distributed as dist

    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.sharding import hash_shard, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, count = shard_range(n_total, rank, world)
        dev = torch.device("cuda:0")
        tuples = torch.empty(3 * max(count, 1), dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        _native.generate_device(0x5EED, start, count, tuples.data_ptr(), s)
        hashes = torch.empty(max(count, 1), dtype=torch.int32, device=dev)
        counts = torch.empty(nqueues, dtype=torch.int64, device=dev)
        hash_shard(_native.prepare_key(key), tuples, count, htable, nqueues, hashes=hashes,
                   counts=counts)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, "h%d.npy" % rank), hashes[:count].cpu().numpy())
        np.save(os.path.join(out_dir, "c%d.npy" % rank), counts.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [1_000_003, 5])
def test_two_ranks_on_device_equal_oracle(tmp_path, oracle_lib, example_key, n_total):
    import torch.multiprocessing as mp
    world, H, Q = 2, 128, 24
    mp.start_processes(_worker, args=(world, _free_port(), example_key, n_total, H, Q,
                                      str(tmp_path)), nprocs=world, start_method="spawn")
    ho, _, co = oracle_lib.run(example_key, oracle_lib.generate(0x5EED, 0, n_total), H, Q)
    got = np.concatenate([np.load(tmp_path / ("h%d.npy" % r)).view(np.uint32)
                          for r in range(world)])
    np.testing.assert_array_equal(got, ho)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("c%d.npy" % r)).view(np.uint64), co)
