"""Multi-GPU data parallelism for the hot path: one process per GPU.

Tuples are independent, so a batch is block-partitioned over ranks with no
data-path communication; every rank hashes its shard on its own GPU and keeps its
``hash_result`` / ``queue_number`` slice.  The only exchange step is the per-queue
histogram: ``uint64[nqueues]`` summed with one all-reduce (RCCL over xGMI with the
``nccl`` backend; ``gloo`` in the CPU tests).  That vector is <= 512 B at the
benchmark configs, so the collective is latency-bound, not link-bound.

The reference is single-process (``simulator.py:74-116``); this module is new.
"""
import torch
import torch.distributed as dist


def shard_range(n_total, rank, world):
    """Contiguous block partition: ``(start, count)`` of rank's shard of ``n_total``.

    The first ``n_total % world`` ranks get one extra tuple, so shards differ by at
    most one and concatenate, in rank order, to the whole batch.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %d for world %d" % (rank, world))
    base, extra = divmod(int(n_total), world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def world_info():
    """``(rank, world)`` of the default process group, ``(0, 1)`` when not distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def allreduce_counts(counts, group=None, async_op=False):
    """Sum per-queue counts over ranks in place (int64 tensor; uint64 bit pattern).

    Counts are exact integers, so the reduced histogram equals the single-device
    histogram of the whole batch bit for bit.  Whenever a process group is
    initialised the collective is issued, at world size 1 too (a no-op sum, but the
    same RCCL call the N-GPU run makes); without one the counts are returned as they
    are.  ``async_op`` returns the work handle (``None`` when nothing was issued).
    """
    if dist.is_available() and dist.is_initialized():
        work = dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return work if async_op else counts
    return None if async_op else counts


def hash_shard(key, tuples, n, htable, nqueues, hashes=None, queues=None, counts=None,
               accumulate=False, group=None):
    """Hash this rank's resident shard on the current device, then all-reduce counts.

    ``tuples`` is a device tensor of at least ``3 * n`` int32 (packed ``rss_tuple4``);
    ``hashes`` / ``queues`` (int32[n]) and ``counts`` (int64[nqueues]) may be None.
    Everything is enqueued on torch's current stream.
    """
    from rss_simulator_nvidia_amd import _native
    stream = torch.cuda.current_stream(tuples.device).cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _native.hash_device(key, tuples.data_ptr(), n, htable, nqueues, ptr(hashes), ptr(queues),
                        ptr(counts), _native.FLAG_ACCUMULATE if accumulate else 0, stream)
    if counts is not None:
        allreduce_counts(counts, group)
    return hashes, queues, counts


class CountsPipeline:
    """Per-step histograms of a rank that hashes batch after batch (a weak-scaling job, a
    service): step i produces its counts in buffer ``i % 2`` and issues the all-reduce of
    that buffer asynchronously, so it overlaps step i+1's hash, which writes the other
    buffer; a buffer's previous all-reduce is waited for before it is reused.  Without a
    process group the collective is skipped (counts are the rank's).

    Two ways to start a step's counts from zero:

    * ``single_pass=True`` (default on a GPU): ``launch(counts, workspace=ws)`` enqueues one
      ``rss_hash_device_ws`` launch that overwrites ``counts`` itself -- the kernel's last
      workgroup writes them from the zero-initialised ``workspace`` (int64 tensor of
      ``nqueues + 1``, shared by the steps: their launches run one after another on the
      caller's stream) -- so a step is one kernel launch and no zeroing launch;
    * ``single_pass=False``: the pipeline zeroes ``counts`` and ``launch(counts)``
      enqueues one pass that accumulates into them.

    ``counts`` is an int64 tensor of ``nqueues``.

    How each step's all-reduce is issued (``allreduce``):

    * ``"overlap"``: ``torch.distributed`` async collective on its own stream, waited for
      before the buffer is reused (one event record + one cross-stream wait on the launch
      stream per step);
    * ``"stream"``: ``torch.distributed`` with ``async_op=False`` -- with the ``nccl`` backend
      it runs on the caller's stream after the launch (two event records per step);
    * ``"rccl"``: ``rccl.RcclComm`` (``comm``) -- ``ncclAllReduce`` enqueued on the caller's
      stream after the launch and nothing else: no markers on the launch stream, buffer
      reuse ordered by the stream.  Per-step cost at world size 1 on MI355X: overlap 22 us,
      stream 8 us, rccl ~0 (``profiles/r02/rccl_step_overhead.log``).
    """

    def __init__(self, nqueues, device, group=None, single_pass=None, allreduce="overlap",
                 comm=None):
        if allreduce not in ("overlap", "stream", "rccl"):
            raise ValueError("allreduce must be overlap, stream or rccl")
        if allreduce == "rccl" and comm is None:
            raise ValueError("allreduce='rccl' needs comm (an rccl.RcclComm)")
        device = torch.device(device)
        self.buffers = [torch.zeros(nqueues, dtype=torch.int64, device=device) for _ in range(2)]
        if single_pass is None:
            single_pass = device.type == "cuda"
        self.workspace = (torch.zeros(nqueues + 1, dtype=torch.int64, device=device)
                          if single_pass else None)
        self.pending = [None, None]
        self.group = group
        self.allreduce = allreduce
        self.comm = comm
        self.steps = 0

    def step(self, launch):
        b = self.steps & 1
        if self.pending[b] is not None:
            self.pending[b].wait()  # buffer b's previous all-reduce must finish before reuse
            self.pending[b] = None
        counts = self.buffers[b]
        if self.workspace is not None:
            launch(counts, workspace=self.workspace)
        else:
            counts.zero_()
            launch(counts)
        if self.allreduce == "overlap":
            self.pending[b] = allreduce_counts(counts, self.group, async_op=True)
        elif self.allreduce == "stream":
            allreduce_counts(counts, self.group)
        else:
            self.comm.all_reduce_counts(counts)
        self.steps += 1
        return counts

    def drain(self):
        """Wait for every outstanding all-reduce; returns the last step's (reduced) counts."""
        for b in (0, 1):
            if self.pending[b] is not None:
                self.pending[b].wait()
                self.pending[b] = None
        return self.buffers[(self.steps - 1) & 1] if self.steps else None
