"""A direct RCCL communicator for the per-step count all-reduce.

The multi-GPU path's one exchange is ``uint64[Q]`` summed over ranks once per batch.
Through ``torch.distributed`` every such collective also records two HIP events on the
launch stream (ProcessGroupNCCL's work-tracking events, with ``async_op=False``) or records
one and makes the launch stream wait on the collective's stream (``async_op=True``); each
marker costs the launch stream a few microseconds of drained queue per step -- 8 and 22 us
per 0.79 ms step at world size 1 (``profiles/r02/rccl_step_overhead.log``).  ``RcclComm``
calls RCCL itself: ``ncclAllReduce`` enqueued on the launch stream right after the hash
launch, stream-ordered, with nothing else on the stream.

The communicator spans the ranks of a ``torch.distributed`` process group (which does the
bootstrap: rank 0's ``ncclUniqueId`` is broadcast over it) and uses the same ``librccl.so``
torch loaded.  The reference is single-process; this module is new.
"""
import ctypes
import os
import threading

import torch
import torch.distributed as dist

NCCL_UINT64, NCCL_SUM = 5, 0  # rccl.h: ncclDataType_t ncclUint64, ncclRedOp_t ncclSum


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_uint8 * 128)]  # NCCL_UNIQUE_ID_BYTES (bytes, may hold NULs)


class RcclError(RuntimeError):
    """An RCCL call failed.  ``stuck`` is True when a communicator init timed out: its
    ``ncclCommInitRank`` may still be blocked on a helper thread of this process (holding
    bootstrap sockets and a half-built communicator), so falling back to another collective
    on the same ``librccl`` is not safe -- callers should end the process instead."""

    def __init__(self, msg, stuck=False):
        super().__init__(msg)
        self.stuck = stuck


_LIB = None


def _library():
    """torch's own ``librccl.so`` (one RCCL in the process), else the ROCm one."""
    global _LIB
    if _LIB is None:
        cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"),
                 "/opt/rocm/lib/librccl.so", "librccl.so"]
        err = None
        for path in cands:
            try:
                lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
                break
            except OSError as e:
                err = e
        else:
            raise RcclError("librccl.so not found: %s" % err)
        vp = ctypes.c_void_p
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
        lib.ncclCommDestroy.argtypes = [vp]
        lib.ncclCommAbort.argtypes = [vp]
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        for fn in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy",
                   "ncclCommAbort"):
            getattr(lib, fn).restype = ctypes.c_int
        _LIB = lib
    return _LIB


def _check(rc, what):
    if rc != 0:
        msg = _library().ncclGetErrorString(rc)
        raise RcclError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else "?"))


class RcclComm:
    """RCCL communicator over the ranks of ``group`` (default: the default group), one GPU
    (``device``) per rank.  Collective over the group: every rank constructs it.

    ``ncclCommInitRank`` runs on a helper thread and is given ``timeout_s``: a rank whose
    init has not finished by then (or failed) reports it, the ranks agree over the process
    group (a MAX all-reduce of [failed, timed out]), and if any rank failed every rank raises
    ``RcclError`` -- so callers fall back together instead of hanging in the bootstrap.  If
    any rank's init timed out the error is ``stuck``: the blocked init cannot be cancelled
    (nor its half-built communicator aborted while the helper thread still runs in it), so
    the process must not fall back to RCCL through ``torch.distributed`` -- it should exit.
    """

    def __init__(self, device, group=None, timeout_s=120.0):
        if not (dist.is_available() and dist.is_initialized()):
            raise RcclError("RcclComm needs an initialised torch.distributed process group")
        lib = _library()
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = _UniqueId()
        blob = [None]
        if self.rank == 0:  # a failure here still reaches the other ranks (as no id)
            rc = lib.ncclGetUniqueId(ctypes.byref(uid))
            blob = [ctypes.string_at(ctypes.addressof(uid), 128) if rc == 0 else ("rc", rc)]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(blob, src=src, group=group, device=self.device)
        if not isinstance(blob[0], bytes) or len(blob[0]) != 128:
            raise RcclError("no ncclUniqueId from rank 0 (%r)" % (blob[0],))
        uid = _UniqueId.from_buffer_copy(blob[0])
        comm = ctypes.c_void_p()
        result = {}

        def init():
            try:
                torch.cuda.set_device(self.device)  # the HIP device is per thread
                result["rc"] = lib.ncclCommInitRank(ctypes.byref(comm), self.world, uid, self.rank)
            except Exception as err:  # reported below, on the caller's thread
                result["err"] = err

        worker = threading.Thread(target=init, name="rccl-init", daemon=True)
        worker.start()
        worker.join(timeout_s)
        stuck = worker.is_alive()
        if stuck:
            why = "ncclCommInitRank did not finish in %.0f s" % timeout_s
        elif "err" in result:
            why = "ncclCommInitRank raised %r" % result["err"]
        elif result.get("rc", -1) != 0:
            msg = lib.ncclGetErrorString(result["rc"])
            why = "ncclCommInitRank failed (%d): %s" % (result["rc"], msg.decode() if msg else "?")
        else:
            why = None
        flags = torch.tensor([1 if why else 0, 1 if stuck else 0], dtype=torch.int32,
                             device=self.device)
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)  # every rank's outcome
        failed, any_stuck = (int(x) for x in flags.tolist())
        self._comm = comm if why is None else None
        if failed:
            # A communicator whose blocking init is still running on the helper thread is
            # left alone: RCCL hands out the handle before that init finishes, so aborting
            # it here would free memory the helper is still using.  The caller exits the
            # process instead (``stuck``).
            if self._comm is not None:
                self.destroy()
            raise RcclError(why or "ncclCommInitRank failed on another rank", stuck=bool(any_stuck))

    def all_reduce_counts(self, counts, stream=None):
        """Sum the int64 (uint64 bit pattern) tensor ``counts`` over the ranks in place,
        enqueued on ``stream`` (default: the current stream of the tensor's device)."""
        if self._comm is None:
            raise RcclError("communicator destroyed")
        if counts.dtype != torch.int64 or not counts.is_contiguous() or counts.device != self.device:
            raise ValueError("counts must be a contiguous int64 tensor on %s" % self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(_library().ncclAllReduce(counts.data_ptr(), counts.data_ptr(), counts.numel(),
                                        NCCL_UINT64, NCCL_SUM, self._comm, s.cuda_stream),
               "ncclAllReduce")
        return counts

    def destroy(self):
        if getattr(self, "_comm", None) is not None and self._comm.value:
            _check(_library().ncclCommDestroy(self._comm), "ncclCommDestroy")
        self._comm = None
