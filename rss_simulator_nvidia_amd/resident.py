"""Device-resident batches on one GPU: placed stream buffers + one kernel launch per batch.

A long-lived caller (a rank of the multi-GPU job, a service hashing batch after batch)
keeps its packed tuples and its ``hash_result`` / ``queue_number`` outputs resident in HBM
and reuses them for every batch.  :class:`ResidentBatch` owns those buffers: it allocates
them once, placed by timing the real kernel on a few candidate allocations
(:mod:`placement` -- the 12 R + 5 W stream's rate depends on where the allocations land in
physical HBM), and launches ``rss_hash_device`` on them.  What is computed
does not depend on the placement: results are those of ``Simulator.calc_hash`` /
``calc_queue_number`` / the ``value_counts`` of ``write_statistics``
(``simulator.py:74-113``) for the tuples in :attr:`tuples`.

The reference is single-process and host-only; this module is new.
"""
import torch

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.placement import choose_stream_buffers

QUEUE_FLAGS = {"u8": _native.FLAG_QUEUE_U8, "u16": _native.FLAG_QUEUE_U16, "u32": 0}
QUEUE_BYTES = {"u8": 1, "u16": 2, "u32": 4}


def narrowest_queue_width(nqueues):
    """The narrowest queue_number width that holds queues ``0 .. nqueues-1``."""
    return "u8" if nqueues <= 256 else ("u16" if nqueues <= 65536 else "u32")


class ResidentBatch:
    """``n`` resident packed tuples and their outputs on ``device``.

    ``fill(tuples)`` (optional) writes the first batch into the int32[3n] input tensor;
    without it the input is left for the caller to write (``batch.tuples``).  The
    candidate inputs are filled the same way before probing, so the probe times the
    kernel on real data.  ``placement=(inputs, outputs[, rounds])`` candidate allocations
    are probed (``rounds``: up to that many rounds of ``outputs`` more output candidates
    while none is clearly faster than the rest, placement.choose_stream_buffers) (``(1, 1)`` = no probe: the first allocation, as allocated); ``queue_bytes``
    sizes the queue buffer per tuple (4 holds any width).  ``report`` records the probe.
    """

    def __init__(self, n, key, htable, nqueues, device=None, fill=None, queue_width="auto",
                 placement=(2, 8), queue_bytes=None, stream=None):
        if n < 1:
            raise ValueError("ResidentBatch: n must be >= 1 (got %d)" % n)
        self.n = int(n)
        self.key = key
        self.htable, self.nqueues = int(htable), int(nqueues)
        self.counts_len = _native.queue_modulus(self.htable, self.nqueues)[1]
        self.queue_width = (narrowest_queue_width(self.counts_len) if queue_width == "auto"
                            else queue_width)
        if self.queue_width not in QUEUE_FLAGS:
            raise ValueError("queue_width must be auto, u8, u16 or u32")
        if self.counts_len > {"u8": 256, "u16": 65536, "u32": 1 << 32}[self.queue_width]:
            raise ValueError("%d queues do not fit queue_width %s" % (self.counts_len,
                                                                     self.queue_width))
        qbytes = queue_bytes or QUEUE_BYTES[self.queue_width]
        if qbytes < QUEUE_BYTES[self.queue_width]:
            raise ValueError("queue_bytes %d < %s width" % (qbytes, self.queue_width))
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.stream = stream or torch.cuda.current_stream(self.device)
        self._fill = fill or (lambda t: None)
        self._probe_counts = torch.zeros(self.counts_len, dtype=torch.int64, device=self.device)
        # single-pass counts workspace of this batch's launches (rss_hash_device_ws; they all
        # run in order on self.stream, so one suffices)
        self.workspace = torch.zeros(_native.counts_workspace_bytes(self.htable, self.nqueues) // 8,
                                     dtype=torch.int64, device=self.device)
        n_in, n_out = placement[0], placement[1]
        rounds = placement[2] if len(placement) > 2 else 1
        self.tuples, self.hashes, self.queues, self.report = choose_stream_buffers(
            torch, self.device, self.n, self._fill, self._probe, n_inputs=n_in,
            n_outputs=n_out, queue_bytes=qbytes, max_rounds=rounds)
        if n_in * n_out == 1:
            self.report["chosen"] = "first allocation"

    def _launch(self, tuples, hashes, queues, counts, flags, workspace=None):
        _native.hash_device(self.key, tuples.data_ptr(), self.n, self.htable, self.nqueues,
                            hashes.data_ptr() if hashes is not None else None,
                            queues.data_ptr() if queues is not None else None,
                            counts.data_ptr() if counts is not None else None,
                            flags, self.stream.cuda_stream,
                            workspace.data_ptr() if workspace is not None else None)

    def _probe(self, tuples, hashes, queues, events):
        if events is not None:
            events[0].record(self.stream)
        # RSS_FLAG_ADDR64: the same access shape as the batch's launches under a kernel
        # symbol of its own, so a profile's row for the step's kernel holds no probe launches
        self._launch(tuples, hashes, queues, self._probe_counts,
                     QUEUE_FLAGS[self.queue_width] | _native.FLAG_ACCUMULATE | _native.FLAG_ADDR64)
        if events is not None:
            events[1].record(self.stream)

    def hash(self, counts=None, accumulate=False, outputs=True, workspace=None):
        """Enqueue one pass over the resident batch on :attr:`stream`: ``hashes`` /
        ``queues`` (when ``outputs``) and ``counts`` (int64[counts_len]; summed into when
        ``accumulate``, else overwritten).  Counts are single-pass (``rss_hash_device_ws``:
        one launch, no zeroing launch before it) on ``workspace`` -- a zeroed int64 tensor of
        ``_native.counts_workspace_bytes(htable, nqueues) // 8`` no other launch uses at the
        same time -- or on the batch's own :attr:`workspace`.  Returns ``counts``."""
        flags = QUEUE_FLAGS[self.queue_width] | (_native.FLAG_ACCUMULATE if accumulate else 0)
        self._launch(self.tuples, self.hashes if outputs else None,
                     self.queues if outputs else None, counts, flags,
                     (workspace if workspace is not None else self.workspace)
                     if counts is not None else None)
        return counts

    def queue_view(self):
        """``queue_number`` of the resident batch as a tensor of the configured width."""
        dt = {"u8": torch.uint8, "u16": torch.int16, "u32": torch.int32}[self.queue_width]
        return self.queues[: self.n * QUEUE_BYTES[self.queue_width]].view(dt)
