"""Multi-rank path on CPU: world_size-2 ``gloo`` process group, tuple sharding and the
count all-reduce (the per-shard compute is the oracle here; the GPU box and the
driver's 8-GPU run exercise the same code with the HIP kernel and RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rss_simulator_nvidia_amd.sharding import allreduce_counts, shard_range, world_info


@pytest.mark.parametrize("n,world", [(0, 1), (10, 3), (7, 8), (2**28 + 5, 8), (1000, 2)])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0
    for (s0, c0), (s1, _) in zip(spans, spans[1:]):
        assert s0 + c0 == s1
    assert sum(c for _, c in spans) == n
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, key, n_total, htable, nqueues, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.oracle import OracleLib
        lib = OracleLib()
        assert world_info() == (rank, world)
        start, count = shard_range(n_total, rank, world)
        tup = lib.generate(0x5EED, start, count)
        h, q, c = lib.run(key, tup, htable, nqueues, threads=1)
        counts = torch.from_numpy(c.view(np.int64).copy())
        allreduce_counts(counts)
        np.save(os.path.join(out_dir, "h%d.npy" % rank), h)
        np.save(os.path.join(out_dir, "c%d.npy" % rank), counts.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_counts_equal_single_process(world, tmp_path, oracle_lib, example_key):
    n_total, htable, nqueues = 100003, 128, 24
    mp.start_processes(_worker, args=(world, _free_port(), example_key, n_total, htable, nqueues,
                                      str(tmp_path)), nprocs=world, start_method="spawn")
    whole = oracle_lib.generate(0x5EED, 0, n_total)
    h, _, c = oracle_lib.run(example_key, whole, htable, nqueues)
    shards = np.concatenate([np.load(tmp_path / ("h%d.npy" % r)) for r in range(world)])
    np.testing.assert_array_equal(shards, h)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("c%d.npy" % r)).view(np.uint64), c)


class _GlooComm:
    """Stands in for rccl.RcclComm on CPU: the same in-place sum over the default group."""

    def __init__(self):
        self.calls = 0

    def all_reduce_counts(self, counts, stream=None):
        self.calls += 1
        dist.all_reduce(counts)
        return counts


def _pipeline_worker(rank, world, port, steps, nq, out_dir, allreduce="overlap"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rss_simulator_nvidia_amd.sharding import CountsPipeline
        comm = _GlooComm() if allreduce == "rccl" else None
        pipe = CountsPipeline(nq, "cpu", allreduce=allreduce, comm=comm)
        seen = []
        for i in range(steps):
            # step i adds (rank + 1) * (i + 1) to every queue of a freshly zeroed buffer
            c = pipe.step(lambda counts, i=i: counts.add_((rank + 1) * (i + 1)))
            seen.append(c.data_ptr())
        last = pipe.drain()
        assert len(set(seen)) == min(2, steps) and last.data_ptr() == seen[-1]
        assert comm is None or comm.calls == steps
        np.save(os.path.join(out_dir, "last%d.npy" % rank), last.numpy())
        np.save(os.path.join(out_dir, "prev%d.npy" % rank), pipe.buffers[steps & 1].numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,steps,allreduce", [(2, 5, "overlap"), (3, 4, "overlap"),
                                                   (2, 1, "overlap"), (2, 5, "stream"),
                                                   (3, 4, "rccl")])
def test_counts_pipeline_reduces_every_step(world, steps, allreduce, tmp_path):
    """CountsPipeline (the bench's step shape), with each all-reduce mode: every step's
    counts summed over ranks, the buffer reused two steps later is re-zeroed, and drain()
    returns the last step's reduced counts ("rccl" through a stand-in comm over gloo)."""
    nq = 7
    mp.start_processes(_pipeline_worker, args=(world, _free_port(), steps, nq, str(tmp_path),
                                               allreduce),
                       nprocs=world, start_method="spawn")
    ranks = sum(r + 1 for r in range(world))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("last%d.npy" % r)),
                                      np.full(nq, ranks * steps))
        if steps > 1:
            np.testing.assert_array_equal(np.load(tmp_path / ("prev%d.npy" % r)),
                                          np.full(nq, ranks * (steps - 1)))


def _bucket_worker(rank, world, port, phases, bucket, nq, out_dir, allreduce):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rss_simulator_nvidia_amd.sharding import CountsPipeline
        comm = _GlooComm() if allreduce == "rccl" else None
        pipe = CountsPipeline(nq, "cpu", allreduce=allreduce, comm=comm, bucket=bucket)
        latest, i = {}, 0
        for steps in phases:  # e.g. the bench's warmup steps, drain, timed steps, drain
            for _ in range(steps):
                c = pipe.step(lambda counts, i=i: counts.add_((rank + 1) * (i + 1)))
                latest[c.data_ptr()] = (i, c)
                i += 1
            last = pipe.drain()
            assert last.data_ptr() == c.data_ptr()
        if comm is not None:
            assert comm.calls == sum(-(-s // bucket) for s in phases)
        rows = sorted(latest.values(), key=lambda v: v[0])
        np.save(os.path.join(out_dir, "rows%d.npy" % rank), np.stack([r.numpy() for _, r in rows]))
        np.save(os.path.join(out_dir, "idx%d.npy" % rank), np.array([j for j, _ in rows]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,phases,bucket,allreduce", [
    (2, (5,), 8, "rccl"), (2, (3, 20), 8, "rccl"), (3, (7, 9), 4, "overlap"),
    (2, (2, 11), 3, "stream"), (2, (16,), 8, "overlap"), (3, (1, 1, 5), 2, "rccl")])
def test_counts_pipeline_bucketed_exchange(world, phases, bucket, allreduce, tmp_path):
    """bucket=B (the bench's N > 1 default B = 8): every step's counts are still reduced on
    their own -- each row that was written last by step i holds the sum over ranks of step
    i's counts, never a row reduced twice (a drain between phases closes a partly filled
    bucket and the next step starts the other one) -- with one collective per B steps."""
    nq = 5
    mp.start_processes(_bucket_worker, args=(world, _free_port(), phases, bucket, nq,
                                             str(tmp_path), allreduce),
                       nprocs=world, start_method="spawn")
    ranks = sum(r + 1 for r in range(world))
    for r in range(world):
        idx = np.load(tmp_path / ("idx%d.npy" % r))
        rows = np.load(tmp_path / ("rows%d.npy" % r))
        assert idx[-1] == sum(phases) - 1
        assert len(idx) == min(sum(phases), 2 * bucket)
        for j, row in zip(idx, rows):
            np.testing.assert_array_equal(row, np.full(nq, ranks * (j + 1)))


def test_counts_pipeline_rejects_bad_modes():
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    with pytest.raises(ValueError, match="overlap, stream or rccl"):
        CountsPipeline(3, "cpu", allreduce="ring")
    with pytest.raises(ValueError, match="needs comm"):
        CountsPipeline(3, "cpu", allreduce="rccl")
    with pytest.raises(ValueError, match="bucket"):
        CountsPipeline(3, "cpu", bucket=0)


def test_rccl_comm_needs_a_process_group():
    from rss_simulator_nvidia_amd.rccl import RcclComm, RcclError
    with pytest.raises(RcclError, match="process group"):
        RcclComm("cpu")


def test_counts_pipeline_without_group_keeps_local_counts():
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    pipe = CountsPipeline(3, "cpu")
    for i in range(3):
        pipe.step(lambda c, i=i: c.add_(i + 1))
    np.testing.assert_array_equal(pipe.drain().numpy(), [3, 3, 3])
    np.testing.assert_array_equal(pipe.buffers[1].numpy(), [2, 2, 2])


def _rccl_fail_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rss_simulator_nvidia_amd.rccl import RcclComm, RcclError
        try:
            RcclComm("cpu", timeout_s=30)
            outcome = "constructed"
        except RcclError as err:
            outcome = "RcclError: %s" % err
        with open(os.path.join(out_dir, "r%d.txt" % rank), "w") as f:
            f.write(outcome)
        dist.barrier()  # every rank got here: nobody is left in the bootstrap
    finally:
        dist.destroy_process_group()


def test_rccl_comm_fails_together_without_a_gpu(tmp_path):
    """Without a GPU, RcclComm must fail on every rank with RcclError -- whether rank 0's
    ncclGetUniqueId or the per-rank init fails -- and no rank may hang waiting for another."""
    world = 2
    mp.start_processes(_rccl_fail_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, start_method="spawn")
    for r in range(world):
        assert (tmp_path / ("r%d.txt" % r)).read_text().startswith("RcclError"), r


def _rccl_stuck_worker(rank, world, port, out_dir):
    """RcclComm over a fake librccl whose ncclCommInitRank blocks past the timeout."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from rss_simulator_nvidia_amd import rccl

        class FakeLib:
            def ncclGetUniqueId(self, uid):
                return 0

            def ncclCommInitRank(self, comm, world, uid, rank):
                time.sleep(6)  # a bootstrap that never completes within the timeout
                return 0

            def ncclGetErrorString(self, rc):
                return b"fake"

            def ncclCommAbort(self, comm):
                return 0

            def ncclCommDestroy(self, comm):
                return 0

        rccl._LIB = FakeLib()
        torch.cuda.set_device = lambda dev: None  # no GPU here; the fake needs none
        try:
            rccl.RcclComm("cpu", timeout_s=1.0)
            outcome = "constructed"
        except rccl.RcclError as err:
            outcome = "stuck=%s %s" % (err.stuck, err)
        with open(os.path.join(out_dir, "r%d.txt" % rank), "w") as f:
            f.write(outcome)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rccl_comm_init_timeout_is_stuck(tmp_path):
    """an init that times out leaves a thread blocked inside RCCL, so every rank
    raises RcclError(stuck=True) -- the bench exits instead of falling back in-process."""
    world = 2
    mp.start_processes(_rccl_stuck_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, start_method="spawn")
    for r in range(world):
        assert (tmp_path / ("r%d.txt" % r)).read_text().startswith("stuck=True"), r
