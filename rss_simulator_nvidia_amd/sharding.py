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

    * ``single_pass=True`` (default on a GPU when ``htable`` is given; without it the
      default is ``False``): ``launch(counts, workspace=ws)`` enqueues one
      ``rss_hash_device_ws`` launch that overwrites ``counts`` itself -- the kernel's last
      workgroup writes them from the zero-initialised ``workspace`` (int64 tensor of
      ``_native.counts_workspace_bytes(htable, nqueues) // 8`` -- the library's own size --
      shared by the steps: their launches run one after another on the caller's stream) --
      so a step is one kernel launch and no zeroing launch; it needs ``htable``;
    * ``single_pass=False``: the pipeline zeroes ``counts`` and ``launch(counts)``
      enqueues one pass that accumulates into them.

    ``counts`` is an int64 tensor of ``nqueues`` -- of ``_native.queue_modulus(htable,
    nqueues)[1]`` (= min(htable, nqueues): no queue >= htable exists) when ``htable`` is given.

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

    ``bucket`` = steps per all-reduce (default 1: every step's counts reduced on their own).
    With ``bucket=B > 1`` the count buffers are the rows of two ``[B, nqueues]`` buckets: step
    i writes row ``i % B`` of bucket ``(i // B) % 2`` and the bucket's ``B`` rows are summed
    over the ranks by ONE collective after its last step -- fewer, larger exchanges, as a
    gradient bucket batches its parameters.  Every step's counts are still reduced on their
    own (the rows are separate histograms, the sum is element-wise); a row holds the reduced
    counts once its bucket's collective has run: after the bucket's last step on the launch
    stream ("rccl" / "stream"), after ``drain()`` in any mode.  ``flush()`` issues the
    collective of a partly filled bucket (``drain()`` calls it).  At world size N > 1 each
    collective joins a step (a few tens of us over xGMI against a ~0.79 ms step) and makes
    every rank wait for the slowest one's launch, so B batches per collective divide both
    by B; a batch's histogram arrives at most B - 1 steps later.
    """

    def __init__(self, nqueues, device, group=None, single_pass=None, allreduce="overlap",
                 comm=None, bucket=1, htable=None):
        if allreduce not in ("overlap", "stream", "rccl"):
            raise ValueError("allreduce must be overlap, stream or rccl")
        if allreduce == "rccl" and comm is None:
            raise ValueError("allreduce='rccl' needs comm (an rccl.RcclComm)")
        bucket = int(bucket)
        if bucket < 1:
            raise ValueError("bucket must be >= 1")
        device = torch.device(device)
        if single_pass is None:  # a caller that gives no htable keeps zero + accumulate
            single_pass = device.type == "cuda" and htable is not None
        if single_pass and htable is None:
            raise ValueError("single_pass counts need htable: the workspace is sized by "
                             "_native.counts_workspace_bytes(htable, nqueues)")
        ws_len = None
        if htable is not None:
            from rss_simulator_nvidia_amd import _native
            if single_pass:
                ws_len = _native.counts_workspace_bytes(htable, nqueues) // 8
            nqueues = _native.queue_modulus(htable, nqueues)[1]
        self.nqueues = nqueues
        self.bucket = bucket
        self.buckets = [torch.zeros(bucket, nqueues, dtype=torch.int64, device=device)
                        for _ in range(2)]
        # buffers[k * bucket + r] = row r of bucket k (bucket=1: the two count buffers)
        self.buffers = [b[r] for b in self.buckets for r in range(bucket)]
        self.workspace = (torch.zeros(ws_len, dtype=torch.int64, device=device)
                          if single_pass else None)
        self.pending = [None, None]
        self._open = 0   # rows of the current bucket written and not yet exchanged
        self._slot = 0   # row slot of the next step (bucket = slot // B % 2, row = slot % B)
        self._last = None
        self.group = group
        self.allreduce = allreduce
        self.comm = comm
        self.steps = 0

    def _exchange(self, k, rows):
        """Issue the all-reduce of bucket k's first ``rows`` rows (one collective)."""
        counts = self.buckets[k][:rows]  # leading rows of a contiguous bucket: contiguous
        if self.allreduce == "overlap":
            self.pending[k] = allreduce_counts(counts, self.group, async_op=True)
        elif self.allreduce == "stream":
            allreduce_counts(counts, self.group)
        else:
            self.comm.all_reduce_counts(counts)

    def step(self, launch):
        k, r = (self._slot // self.bucket) & 1, self._slot % self.bucket
        if r == 0 and self.pending[k] is not None:
            self.pending[k].wait()  # bucket k's previous all-reduce must finish before reuse
            self.pending[k] = None
        counts = self.buckets[k][r]
        if self.workspace is not None:
            launch(counts, workspace=self.workspace)
        else:
            counts.zero_()
            launch(counts)
        self.steps += 1
        self._slot += 1
        self._last = counts
        self._open = r + 1  # rows of bucket k written and not yet exchanged
        if self._open == self.bucket:
            self._exchange(k, self._open)
            self._open = 0
        return counts

    def flush(self):
        """Issue the collective of a partly filled bucket (no wait); the next step starts
        the other bucket, so no row is ever exchanged twice."""
        if self._open:
            self._exchange(((self._slot - 1) // self.bucket) & 1, self._open)
            self._slot += self.bucket - self._open
            self._open = 0

    def drain(self):
        """Flush, then wait for every outstanding all-reduce; returns the last step's
        (reduced) counts."""
        self.flush()
        for b in (0, 1):
            if self.pending[b] is not None:
                self.pending[b].wait()
                self.pending[b] = None
        return self._last
