"""The RCCL leg executed on MI355X: a world-size-1 ``nccl`` process group
(torch's ``nccl`` backend is RCCL on ROCm) runs every collective the N-GPU bench makes --
``init_process_group("nccl", device_id=...)``, the synchronous and the async
``all_reduce`` of the ``uint64[Q]`` counts from ``rss_hash_device``, the MAX all-reduce of
the timings, ``barrier(device_ids=...)`` and ``destroy_process_group``, and the bench's
default per-step exchange, ``ncclAllReduce`` through ``rccl.RcclComm`` on the launch stream
-- and the reduced counts must equal the oracle's.  A second test runs ``bench.py`` itself under
``torch.distributed.run --nproc-per-node 1``: its line must carry the CPU baseline and the
max-over-ranks roofline, as every N > 1 line of the driver's scaling run will.

One GPU per box, and RCCL refuses two ranks on one device, so world size 1 is the most
this box can run; the world-2/3 exchange itself is covered with gloo
(tests/test_sharding.py, tests/test_gpu_sharding.py)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_worker(rank, port, key, n, htable, nqueues, out_dir):
    import torch.distributed as dist

    from rss_simulator_nvidia_amd import _native
    from rss_simulator_nvidia_amd.sharding import allreduce_counts, hash_shard, world_info
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        assert world_info() == (0, 1)
        tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        _native.generate_device(0x5EED, 0, n, tuples.data_ptr(), s)
        hashes = torch.empty(n, dtype=torch.int32, device=dev)
        counts = torch.empty(nqueues, dtype=torch.int64, device=dev)
        # synchronous all-reduce inside hash_shard (sharding.allreduce_counts)
        hash_shard(_native.prepare_key(key), tuples, n, htable, nqueues, hashes=hashes,
                   counts=counts)
        # the bench's form: async all-reduce of a second buffer, waited before reuse
        counts2 = torch.zeros(nqueues, dtype=torch.int64, device=dev)
        _native.hash_device(_native.prepare_key(key), tuples.data_ptr(), n, htable, nqueues,
                            None, None, counts2.data_ptr(), _native.FLAG_ACCUMULATE, s)
        work = allreduce_counts(counts2, async_op=True)
        assert work is not None
        work.wait()
        # the bench's default form: ncclAllReduce through rccl.RcclComm on the launch stream,
        # through CountsPipeline with single-pass counts, batch after batch
        from rss_simulator_nvidia_amd.rccl import RcclComm
        from rss_simulator_nvidia_amd.sharding import CountsPipeline
        comm = RcclComm(dev)
        assert (comm.rank, comm.world) == (0, 1)
        pipe = CountsPipeline(nqueues, dev, allreduce="rccl", comm=comm, htable=htable)
        k = _native.prepare_key(key)
        for _ in range(5):
            c3 = pipe.step(lambda c, workspace: _native.hash_device(
                k, tuples.data_ptr(), n, htable, nqueues, None, None, c.data_ptr(), 0, s,
                workspace.data_ptr()))
        c3 = pipe.drain()
        # bucketed (the bench's N > 1 default): one ncclAllReduce per [3, Q] bucket, a
        # drain between phases closes a partly filled one
        pipe_b = CountsPipeline(nqueues, dev, allreduce="rccl", comm=comm, bucket=3,
                                htable=htable)
        rows = []
        for steps in (2, 5):
            for _ in range(steps):
                rows.append(pipe_b.step(lambda c, workspace: _native.hash_device(
                    k, tuples.data_ptr(), n, htable, nqueues, None, None, c.data_ptr(), 0, s,
                    workspace.data_ptr())))
            pipe_b.drain()
        c5 = torch.stack(rows[-5:])  # the last five steps' rows: all distinct, none reused
        direct = counts2.clone()
        comm.all_reduce_counts(direct)
        torch.cuda.synchronize()
        comm.destroy()
        np.save(os.path.join(out_dir, "c3.npy"), c3.cpu().numpy())
        np.save(os.path.join(out_dir, "c4.npy"), direct.cpu().numpy())
        np.save(os.path.join(out_dir, "c5.npy"), c5.cpu().numpy())
        stats = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        dist.barrier(device_ids=[0])
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, "h.npy"), hashes.cpu().numpy())
        np.save(os.path.join(out_dir, "c.npy"), counts.cpu().numpy())
        np.save(os.path.join(out_dir, "c2.npy"), counts2.cpu().numpy())
        np.save(os.path.join(out_dir, "stats.npy"), stats.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_nccl_world1_allreduce_counts_equal_oracle(tmp_path, oracle_lib, example_key):
    import torch.multiprocessing as mp
    n, H, Q = 1_000_003, 128, 24
    mp.start_processes(_rccl_worker, args=(_free_port(), example_key, n, H, Q, str(tmp_path)),
                       nprocs=1, start_method="spawn")
    ho, _, co = oracle_lib.run(example_key, oracle_lib.generate(0x5EED, 0, n), H, Q)
    np.testing.assert_array_equal(np.load(tmp_path / "h.npy").view(np.uint32), ho)
    np.testing.assert_array_equal(np.load(tmp_path / "c.npy").view(np.uint64), co)
    np.testing.assert_array_equal(np.load(tmp_path / "c2.npy").view(np.uint64), co)
    np.testing.assert_array_equal(np.load(tmp_path / "c3.npy").view(np.uint64), co)
    np.testing.assert_array_equal(np.load(tmp_path / "c4.npy").view(np.uint64), co)
    for row in np.load(tmp_path / "c5.npy").view(np.uint64):
        np.testing.assert_array_equal(row, co)
    np.testing.assert_array_equal(np.load(tmp_path / "stats.npy"), [1.5, 2.5])


@pytest.mark.timeout(300)
def test_bench_under_torchrun_nproc1_reports_baseline_and_roofline(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--tuples-per-gpu", str(1 << 22), "--no-extras", "--cpu-sample", "400",
           "--cpu-procs", "2"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["warmup"] == 1
    assert "RCCL all-reduce" in rec["config"]["parallelism"]
    assert "rccl.RcclComm" in rec["config"]["parallelism"]  # the default per-step exchange
    # one all-reduce per batch (the default); 8 batches per collective only as `bucketed`
    assert "one collective per batch" in rec["config"]["parallelism"]
    assert rec["config"]["collectives_per_batch"] == 1.0
    assert rec["bucketed"]["steps_per_collective"] == 8 and rec["bucketed"]["value"] > 0
    base = rec["cpu_baseline"]
    assert base is not None and base["value"] > 0 and base["cores"] == 2
    assert rec["settle"]["launches"] >= 16  # clock-settle launches before the warmup
    roof = rec["roofline"]
    assert roof["kernel_ms"] == roof["kernel_ms_max_rank"]
    assert roof["kernel_ms_min_max"][0] <= roof["kernel_ms_median"] <= roof["kernel_ms_min_max"][1]
    want = (1 << 22) * roof["bytes_per_tuple"] / (roof["kernel_ms_max_rank"] / 1e3) / 1e9
    assert abs(roof["achieved"] - want) < 1e-6 * want
