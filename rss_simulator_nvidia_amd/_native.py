"""ctypes binding of the C ABI in ``include/rss_toeplitz.h``.

The library (``librss_toeplitz.so``, built in-tree by ``__graft_entry__.build()`` /
``make -C rss_simulator_nvidia_amd/csrc``) is the only compute path of this
package: there is no CPU fallback.  Every entry point raises
:class:`~rss_simulator_nvidia_amd.exceptions.NativeLibraryError` when the library
is missing and :class:`~rss_simulator_nvidia_amd.exceptions.DeviceError` when the
HIP runtime reports a failure (including "no gfx950 device").
"""
import ctypes
import os
import threading

import numpy as np

from rss_simulator_nvidia_amd.exceptions import DeviceError, NativeLibraryError

LIB_NAME = "librss_toeplitz.so"
LIB_PATH = os.environ.get(
    "RSS_TOEPLITZ_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME))

ABI_VERSION = 1
FLAG_ACCUMULATE = 1
FLAG_QUEUE_U16 = 2
FLAG_QUEUE_U8 = 4
FLAG_ADDR64 = 8  # 64-bit addressing where 32-bit offsets fit: own kernel symbol in traces
FLAG_CSV_COUNTS_ONLY = 1
KEY_MIN_BYTES = 4

# Every symbol include/rss_toeplitz.h declares (tests/test_native_abi.py checks them).
EXPORTED_SYMBOLS = (
    "rss_key_prepare", "rss_hash_device", "rss_generate_tuples", "rss_ctx_create",
    "rss_ctx_destroy", "rss_hash_host", "rss_device_count", "rss_last_error",
    "rss_abi_version", "rss_csv_parse", "rss_csv_format_bound", "rss_csv_format",
    "rss_key_search_device", "rss_key_search_host", "rss_key_select_fields",
    "rss_key6_prepare", "rss_key6_select_fields", "rss_hash6_device", "rss_hash6_host",
    "rss_pcap_parse", "rss_hash_device_reta", "rss_hash_host_reta", "rss_csv_hash_text",
    "rss_csv_hash_file", "rss_host_alloc", "rss_host_free", "rss_hash_host_multi",
    "rss_pcap_parse6", "rss_hash6_device_reta", "rss_hash6_host_reta", "rss_csv_parse6",
    "rss_csv_format6_bound", "rss_csv_format6", "rss_csv6_hash_text", "rss_csv6_hash_file",
    "rss_counts_workspace_bytes", "rss_hash_device_ws", "rss_hash6_device_ws",
    "rss_parse_dotted", "rss_parse_ipv6",
)
FIELD_SRC_IP, FIELD_DST_IP, FIELD_SRC_PORT, FIELD_DST_PORT = 1, 2, 4, 8
FIELDS_IP, FIELDS_ALL = 3, 15
ENOTSUP = -95


class RssTuple4(ctypes.Structure):
    """``rss_tuple4``: packed 12-byte IPv4 4-tuple."""
    _fields_ = [("sip", ctypes.c_uint32), ("dip", ctypes.c_uint32), ("ports", ctypes.c_uint32)]


class RssKey(ctypes.Structure):
    """``rss_key``: prepared key (length, bytes, the 96 rotation windows)."""
    _fields_ = [
        ("len", ctypes.c_uint32),
        ("bytes", ctypes.c_uint8 * 52),
        ("window", ctypes.c_uint32 * 96),
    ]


class RssKey6(ctypes.Structure):
    """``rss_key6``: prepared key for the 288-bit IPv6 input."""
    _fields_ = [("len", ctypes.c_uint32), ("window", ctypes.c_uint32 * 288)]


class RssTuple6(ctypes.Structure):
    """``rss_tuple6``: IPv6 4-tuple as nine big-endian-valued words."""
    _fields_ = [("w", ctypes.c_uint32 * 9)]


class RssCsvLayout(ctypes.Structure):
    """``rss_csv_layout``: which column each CSV field holds."""
    _fields_ = [("field_column", ctypes.c_uint8 * 4)]


TUPLE_DTYPE = np.dtype([("sip", "<u4"), ("dip", "<u4"), ("ports", "<u4")])
assert TUPLE_DTYPE.itemsize == ctypes.sizeof(RssTuple4) == 12
TUPLE6_DTYPE = np.dtype([("sip", "<u4", (4,)), ("dip", "<u4", (4,)), ("ports", "<u4")])
assert TUPLE6_DTYPE.itemsize == ctypes.sizeof(RssTuple6) == 36

_lock = threading.Lock()
_lib = None


def _bind(lib):
    vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
    key_p = ctypes.POINTER(RssKey)
    sigs = {
        "rss_abi_version": ([], ctypes.c_int),
        "rss_last_error": ([], ctypes.c_char_p),
        "rss_key_prepare": ([ctypes.POINTER(ctypes.c_uint8), sz, key_p], ctypes.c_int),
        "rss_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "rss_hash_device": ([key_p, vp, sz, u32, u32, vp, vp, vp, u32, vp], ctypes.c_int),
        "rss_hash_device_ws": ([key_p, vp, sz, u32, u32, vp, vp, vp, u32, vp, vp], ctypes.c_int),
        "rss_counts_workspace_bytes": ([u32, ctypes.POINTER(sz)], ctypes.c_int),
        "rss_generate_tuples": ([u64, u64, sz, vp, vp], ctypes.c_int),
        "rss_ctx_create": ([ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "rss_ctx_destroy": ([vp], None),
        "rss_hash_host": ([vp, key_p, vp, sz, u32, u32, vp, vp, vp, u32], ctypes.c_int),
        "rss_csv_parse": ([vp, sz, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(RssCsvLayout),
                           ctypes.c_int], ctypes.c_int),
        "rss_csv_format_bound": ([sz, u32], sz),
        "rss_key_search_device": ([vp, sz, vp, sz, u32, u32, vp, vp], ctypes.c_int),
        "rss_key_select_fields": ([key_p, u32], ctypes.c_int),
        "rss_hash_device_reta": ([key_p, vp, sz, u32, vp, u32, vp, vp, vp, u32, vp], ctypes.c_int),
        "rss_hash_host_reta": ([vp, key_p, vp, sz, u32, vp, u32, vp, vp, vp, u32], ctypes.c_int),
        "rss_csv_hash_text": ([vp, key_p, vp, sz, u32, u32, vp, u32,
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                               vp, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rss_csv_hash_file": ([vp, key_p, ctypes.c_char_p, ctypes.c_char_p, u32, u32, vp, u32, vp,
                               ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rss_csv6_hash_text": ([vp, ctypes.POINTER(RssKey6), vp, sz, u32, u32, vp, u32,
                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                vp, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
        "rss_csv6_hash_file": ([vp, ctypes.POINTER(RssKey6), ctypes.c_char_p, ctypes.c_char_p,
                                u32, u32, vp, u32, vp, ctypes.POINTER(ctypes.c_size_t)],
                               ctypes.c_int),
        "rss_pcap_parse": ([vp, sz, vp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)],
                           ctypes.c_int),
        "rss_pcap_parse6": ([vp, sz, vp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)],
                            ctypes.c_int),
        "rss_key6_prepare": ([ctypes.POINTER(ctypes.c_uint8), sz, ctypes.POINTER(RssKey6)],
                             ctypes.c_int),
        "rss_key6_select_fields": ([ctypes.POINTER(RssKey6), u32], ctypes.c_int),
        "rss_hash6_device_ws": ([ctypes.POINTER(RssKey6), vp, sz, u32, u32, vp, vp, vp, u32, vp,
                                 vp], ctypes.c_int),
        "rss_hash6_device": ([ctypes.POINTER(RssKey6), vp, sz, u32, u32, vp, vp, vp, u32, vp],
                             ctypes.c_int),
        "rss_hash6_host": ([vp, ctypes.POINTER(RssKey6), vp, sz, u32, u32, vp, vp, vp, u32],
                           ctypes.c_int),
        "rss_hash6_device_reta": ([ctypes.POINTER(RssKey6), vp, sz, u32, vp, u32, vp, vp, vp, u32,
                                   vp], ctypes.c_int),
        "rss_hash6_host_reta": ([vp, ctypes.POINTER(RssKey6), vp, sz, u32, vp, u32, vp, vp, vp,
                                 u32], ctypes.c_int),
        "rss_key_search_host": ([vp, vp, sz, vp, sz, u32, u32, vp], ctypes.c_int),
        "rss_csv_format": ([vp, vp, vp, sz, vp, u32, ctypes.POINTER(RssCsvLayout), vp, sz,
                            ctypes.POINTER(sz), ctypes.c_int], ctypes.c_int),
        "rss_csv_parse6": ([vp, sz, vp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(RssCsvLayout),
                            ctypes.c_int], ctypes.c_int),
        "rss_csv_format6_bound": ([vp, sz, u32], sz),
        "rss_csv_format6": ([vp, vp, vp, vp, sz, vp, u32, ctypes.POINTER(RssCsvLayout), vp, sz,
                             ctypes.POINTER(sz), ctypes.c_int], ctypes.c_int),
        "rss_host_alloc": ([sz, ctypes.POINTER(vp)], ctypes.c_int),
        "rss_host_free": ([vp], None),
        "rss_hash_host_multi": ([ctypes.POINTER(vp), ctypes.c_int, key_p, vp, sz, u32, vp, u32,
                                 vp, vp, vp, u32], ctypes.c_int),
        "rss_parse_dotted": ([vp, sz, sz, vp, vp], ctypes.c_int),
        "rss_parse_ipv6": ([vp, sz, sz, vp, vp], ctypes.c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


def load():
    """Load (once) and return the native library; raise loudly if it is absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    "HIP extension %s not found; build it with `python -c "
                    "'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)" % LIB_PATH)
            try:
                lib = ctypes.CDLL(LIB_PATH)
            except OSError as err:
                raise NativeLibraryError("cannot load %s: %s" % (LIB_PATH, err))
            lib = _bind(lib)
            if lib.rss_abi_version() != ABI_VERSION:
                raise NativeLibraryError("ABI mismatch: library %d, binding %d"
                                         % (lib.rss_abi_version(), ABI_VERSION))
            _lib = lib
        return _lib


def _check(rc, what):
    if rc != 0:
        msg = load().rss_last_error().decode("utf-8", "replace")
        raise DeviceError("%s failed (%d): %s" % (what, rc, msg))


def device_count():
    out = ctypes.c_int(0)
    _check(load().rss_device_count(ctypes.byref(out)), "rss_device_count")
    return out.value


def parse_fields(spec):
    """ethtool-style field letters -> mask: s src ip, d dst ip, f src port, n dst port."""
    bits = {"s": FIELD_SRC_IP, "d": FIELD_DST_IP, "f": FIELD_SRC_PORT, "n": FIELD_DST_PORT}
    if not spec or any(c not in bits for c in spec) or len(set(spec)) != len(spec):
        raise ValueError("hash fields must be distinct letters of 'sdfn', got %r" % (spec,))
    mask = 0
    for c in spec:
        mask |= bits[c]
    return mask


def prepare_key(key_bytes, fields=FIELDS_ALL):
    """Build an :class:`RssKey` from raw key bytes (>= 4; the CLI admits 40 or 52).

    ``fields`` (mask or 'sdfn' letters) selects the hashed fields; the default hashes
    the whole 4-tuple as the reference does."""
    raw = bytes(bytearray(int(b) & 0xFF for b in key_bytes))
    if len(raw) < KEY_MIN_BYTES:
        raise ValueError("hash key must hold at least %d bytes, got %d" % (KEY_MIN_BYTES, len(raw)))
    key = RssKey()
    buf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    _check(load().rss_key_prepare(buf, len(raw), ctypes.byref(key)), "rss_key_prepare")
    if isinstance(fields, str):
        fields = parse_fields(fields)
    if fields != FIELDS_ALL:
        _check(load().rss_key_select_fields(ctypes.byref(key), fields), "rss_key_select_fields")
    return key


def prepare_key6(key_bytes, fields=FIELDS_ALL):
    """Build an :class:`RssKey6` (IPv6 input) from raw key bytes; optional field mask."""
    raw = bytes(bytearray(int(b) & 0xFF for b in key_bytes))
    if len(raw) < KEY_MIN_BYTES:
        raise ValueError("hash key must hold at least %d bytes, got %d" % (KEY_MIN_BYTES, len(raw)))
    key = RssKey6()
    buf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    _check(load().rss_key6_prepare(buf, len(raw), ctypes.byref(key)), "rss_key6_prepare")
    if isinstance(fields, str):
        fields = parse_fields(fields)
    if fields != FIELDS_ALL:
        _check(load().rss_key6_select_fields(ctypes.byref(key), fields), "rss_key6_select_fields")
    return key


def _csv_reta(reta, htable):
    """The CSV device path's indirection table: None, or htable uint32 queue ids."""
    if reta is None:
        return None
    table = np.ascontiguousarray(reta, dtype=np.uint32)
    if len(table) != htable:
        raise ValueError("indirection table has %d entries, htable is %d" % (len(table), htable))
    return table


class PinnedBuffer:
    """Page-locked host memory from ``rss_host_alloc``, freed when the last numpy view
    of it is gone (views keep this object alive through their ``base`` chain)."""

    def __init__(self, nbytes):
        self._lib = load()
        ptr = ctypes.c_void_p()
        _check(self._lib.rss_host_alloc(nbytes, ctypes.byref(ptr)), "rss_host_alloc")
        self.ptr, self.nbytes = ptr.value, nbytes
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                    "data": (ptr.value, False), "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.rss_host_free(self.ptr)
            self.ptr = None


def pinned_empty(shape, dtype):
    """Uninitialised numpy array in page-locked memory: ``HostContext.hash`` moves such
    arrays by DMA without a staging copy.  Pinning is expensive -- allocate once, reuse."""
    dtype = np.dtype(dtype)
    shape = (shape,) if np.isscalar(shape) else tuple(shape)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    raw = np.asarray(PinnedBuffer(max(nbytes, 1)))
    return raw[:nbytes].view(dtype).reshape(shape)


def ptr(a):
    """Data pointer of a numpy array, or None (NULL) for a disabled output."""
    return a.ctypes.data if a is not None else None


def _host_batch(tuples, nqueues, want_hash, want_queue, want_counts, out, ipv6=False):
    """Packed tuples (IPv4, or IPv6 with ``ipv6``) as a contiguous array + the (hash, queue,
    counts) outputs to fill."""
    arr = np.ascontiguousarray(tuples)
    dtype, words = (TUPLE6_DTYPE, 9) if ipv6 else (TUPLE_DTYPE, 3)
    if arr.dtype != dtype:
        arr = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1, words)
    n = len(arr)
    if out is not None:
        h, q = out
        for a in (h, q):
            if a is not None and (a.dtype != np.uint32 or a.shape != (n,)
                                  or not a.flags.c_contiguous):
                raise ValueError("out arrays must be contiguous uint32[%d]" % n)
    else:
        h = np.empty(n, dtype=np.uint32) if want_hash else None
        q = np.empty(n, dtype=np.uint32) if want_queue else None
    c = np.zeros(nqueues, dtype=np.uint64) if want_counts else None
    return arr, n, h, q, c


U32_MAX = 0xFFFFFFFF
RETA_QUEUE_MAX = 0xFFFF  # an indirection-table entry travels as u16 (rss_hash_device_reta)


def queue_modulus(htable, nqueues, reta=False):
    """``(htable, nqueues')`` as the C ABI's ``uint32_t`` arguments, for the same
    ``queue = hash % htable % nqueues`` (``simulator.py:96-98``) on every 32-bit hash,
    with ``nqueues'`` the number of queues a tuple can actually get -- the length of every
    per-queue count vector (queues past it are always empty).

    * ``nqueues >= htable``: ``bucket = hash % htable < htable <= nqueues``, so ``queue =
      bucket`` -> ``(htable, htable)``: bins, counts and the queue column's width are sized
      by ``min(htable, nqueues)``, never by ``nqueues`` (``--num-queues 4000000000`` with
      ``--htable-size 128`` needs 128 counts, not 32 GB);
    * ``htable >= 2**32``: ``hash % htable = hash`` (hash < 2**32), so ``queue = hash %
      nqueues``; any multiple of ``nqueues`` as the table size gives the same remainder ->
      ``((2**32 - 1) // nqueues * nqueues, nqueues)`` (ctypes would truncate 4294967297 to
      1 silently: values are rewritten exactly, never truncated);
    * both ``>= 2**32``: ``queue = hash``, whose histogram would need 2**32 entries --
      ``ValueError`` here (``Simulator`` counts that case's queues sparsely on the host);
    * with an indirection table (``reta``) queues are table entries < 2**16, so an
      ``nqueues >= 2**32`` only bounds them: it becomes 65536 (higher queues stay empty);
      the library sizes its bins by ``max(reta) + 1``.
    """
    H, Q = int(htable), int(nqueues)
    if H < 0 or Q < 0:  # ctypes would wrap -1 to 2**32 - 1
        raise ValueError("htable (%d) and nqueues (%d) must be >= 1" % (H, Q))
    if H == 0 or Q == 0:
        return H, Q  # the library refuses it (RSS_EINVAL, "must be >= 1")
    if reta:
        return H, (Q if Q <= U32_MAX else RETA_QUEUE_MAX + 1)
    if H <= U32_MAX:
        return H, min(H, Q)
    if Q <= U32_MAX:
        return U32_MAX // Q * Q, Q
    raise ValueError("htable %d and nqueues %d both >= 2**32: every hash would be its own queue "
                     "(a 2**32-entry histogram); not supported" % (H, Q))


def queues_are_hashes(htable, nqueues, reta=None):
    """True when ``hash % htable % nqueues == hash`` for every 32-bit hash (both >= 2**32,
    no table): the one case :func:`queue_modulus` refuses, whose queues are the hashes."""
    return reta is None and int(htable) > U32_MAX and int(nqueues) > U32_MAX


def _reta_table(reta, htable):
    table = np.ascontiguousarray(reta, dtype=np.uint32)
    if len(table) != htable:
        raise ValueError("indirection table has %d entries, htable is %d" % (len(table), htable))
    return table


def _copy_out(image, chunk=64 << 20):
    """A copy of a large context-owned image, in 64 MiB slices on up to 8 threads (numpy
    releases the GIL for the copies): a fresh destination's page faults bound a one-thread
    copy at ~14 GB/s, 0.063 s for a 16M-row statistics image on the GPU box."""
    n = image.size
    threads = min(8, len(os.sched_getaffinity(0)), -(-n // chunk))
    if threads < 2:
        return image.copy()
    dst = np.empty_like(image)
    step = -(-n // threads)

    def part(i):
        np.copyto(dst[i * step:(i + 1) * step], image[i * step:(i + 1) * step])

    workers = [threading.Thread(target=part, args=(i,)) for i in range(1, threads)]
    for w in workers:
        w.start()
    part(0)
    for w in workers:
        w.join()
    return dst


class HostContext:
    """Owns an ``rss_ctx`` (device buffers + streams) for host-memory batches.

    Thread-safe: the library serialises the calls on one context (``struct rss_ctx``'s
    lock, ``include/rss_toeplitz.h``), so the process-wide :func:`default_context` can
    serve many threads at once, as the reference's per-call ``Toeplitz.compute_hash``
    (``toeplitz.py:59``) can.  Calls on different contexts run concurrently."""

    def __init__(self, device=0):
        self._lib = load()
        self._ctx = ctypes.c_void_p()
        # held across rss_csv_hash_text and the copy of its context-owned image, which the
        # next call on the context (from any thread) may overwrite
        self._image_lock = threading.Lock()
        _check(self._lib.rss_ctx_create(device, ctypes.byref(self._ctx)), "rss_ctx_create")
        self.device = device

    def close(self):
        if self._ctx:
            self._lib.rss_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def hash(self, key, tuples, htable, nqueues, want_hash=True, want_queue=True, want_counts=True,
             reta=None, out=None):
        """Hash packed tuples (structured ``TUPLE_DTYPE`` or uint32 (n, 3)) on the GPU.

        ``reta`` (optional, ``htable`` queue ids) maps buckets to queues instead of
        ``bucket % nqueues``.  ``out`` (optional) = caller-owned ``(hash_u32[n],
        queue_u32[n])`` to fill, e.g. :func:`pinned_empty` arrays reused across batches
        (page-locked tuples and outputs skip the staging copies).  Returns
        ``(hash_u32, queue_u32, counts_u64)``; disabled outputs are None.
        """
        htable, nqueues = queue_modulus(htable, nqueues, reta is not None)
        arr, n, h, q, c = _host_batch(tuples, nqueues, want_hash, want_queue, want_counts, out)
        if reta is None:
            _check(self._lib.rss_hash_host(self._ctx, ctypes.byref(key), ptr(arr), n, htable,
                                           nqueues, ptr(h), ptr(q), ptr(c), 0), "rss_hash_host")
        else:
            table = _reta_table(reta, htable)
            _check(self._lib.rss_hash_host_reta(self._ctx, ctypes.byref(key), ptr(arr), n, htable,
                                                table.ctypes.data, nqueues, ptr(h), ptr(q), ptr(c),
                                                0), "rss_hash_host_reta")
        return h, q, c


    def hash6(self, key6, tuples6, htable, nqueues, want_hash=True, want_queue=True,
              want_counts=True, reta=None, out=None):
        """IPv6 batch (``TUPLE6_DTYPE`` or uint32 (n, 9)) -> (hash, queue, counts) through
        the same staging, small-batch path and pipeline as :meth:`hash`; ``reta`` and
        ``out`` (page-locked arrays skip the staging copies) as there."""
        htable, nqueues = queue_modulus(htable, nqueues, reta is not None)
        arr, n, h, q, c = _host_batch(tuples6, nqueues, want_hash, want_queue, want_counts, out,
                                      ipv6=True)
        if reta is None:
            _check(self._lib.rss_hash6_host(self._ctx, ctypes.byref(key6), ptr(arr), n, htable,
                                            nqueues, ptr(h), ptr(q), ptr(c), 0), "rss_hash6_host")
        else:
            table = _reta_table(reta, htable)
            _check(self._lib.rss_hash6_host_reta(self._ctx, ctypes.byref(key6), ptr(arr), n,
                                                 htable, ptr(table), nqueues, ptr(h), ptr(q),
                                                 ptr(c), 0), "rss_hash6_host_reta")
        return h, q, c

    def csv_hash_text(self, key, data, htable, nqueues, reta=None, counts_only=False,
                      copy=True):
        """The whole ``--csv`` job on the device for a canonical file image
        (``rss_csv_hash_text``; ``rss_csv6_hash_text`` when ``key`` is an :class:`RssKey6`):
        returns ``(file_image, counts, n_rows)`` -- file_image a uint8 array (None with
        ``counts_only``) -- or None when the text is not canonical.  ``copy=False`` returns
        a zero-copy view of context-owned memory instead, valid only until the next call
        on this context (which may resize or overwrite it)."""
        htable, nqueues = queue_modulus(htable, nqueues, reta is not None)
        buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        counts = np.zeros(nqueues, dtype=np.uint64)
        out, out_len, n = ctypes.c_void_p(), ctypes.c_size_t(0), ctypes.c_size_t(0)
        table = _csv_reta(reta, htable)
        name = "rss_csv6_hash_text" if isinstance(key, RssKey6) else "rss_csv_hash_text"
        with self._image_lock:
            rc = getattr(self._lib, name)(
                self._ctx, ctypes.byref(key), buf.ctypes.data, len(buf), htable, nqueues,
                table.ctypes.data if table is not None else None,
                FLAG_CSV_COUNTS_ONLY if counts_only else 0, ctypes.byref(out),
                ctypes.byref(out_len), counts.ctypes.data, ctypes.byref(n))
            if rc == ENOTSUP:
                return None
            _check(rc, name)
            image = None
            if not counts_only:
                if out_len.value:
                    image = np.ctypeslib.as_array(
                        ctypes.cast(out, ctypes.POINTER(ctypes.c_uint8)), shape=(out_len.value,))
                    if copy:
                        image = _copy_out(image)
                else:
                    image = np.empty(0, dtype=np.uint8)
        return image, counts, n.value

    def csv_hash_file(self, key, in_path, out_path, htable, nqueues, reta=None):
        """``rss_csv_hash_file`` (``rss_csv6_hash_file`` for an :class:`RssKey6`): the
        ``--csv`` job from file to file on the device (no file-sized host buffers).
        ``out_path`` None = counts only.  Returns ``(counts, n_rows)``, or None when the
        file is not canonical or a path cannot be opened (the pandas path then raises the
        reference's error)."""
        htable, nqueues = queue_modulus(htable, nqueues, reta is not None)
        counts = np.zeros(nqueues, dtype=np.uint64)
        n = ctypes.c_size_t(0)
        table = _csv_reta(reta, htable)
        enc = lambda p: os.fsencode(p) if p is not None else None  # noqa: E731
        name = "rss_csv6_hash_file" if isinstance(key, RssKey6) else "rss_csv_hash_file"
        rc = getattr(self._lib, name)(
            self._ctx, ctypes.byref(key), enc(in_path), enc(out_path), htable, nqueues,
            table.ctypes.data if table is not None else None,
            FLAG_CSV_COUNTS_ONLY if out_path is None else 0, counts.ctypes.data, ctypes.byref(n))
        if rc == ENOTSUP:
            return None
        _check(rc, name)
        return counts, n.value

    def key_search(self, keys, tuples, htable, nqueues):
        """Per-queue counts (uint64[len(keys), nqueues]) of ``tuples`` under each prepared key."""
        htable, nqueues = queue_modulus(htable, nqueues)
        arr = np.ascontiguousarray(tuples)
        if arr.dtype != TUPLE_DTYPE:
            arr = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1, 3)
        karr = (RssKey * len(keys))(*keys)
        out = np.zeros((len(keys), nqueues), dtype=np.uint64)
        _check(self._lib.rss_key_search_host(self._ctx, karr, len(keys), arr.ctypes.data, len(arr),
                                             htable, nqueues, out.ctypes.data),
               "rss_key_search_host")
        return out


_default_ctx = None
_ctx_lock = threading.Lock()


class MultiHostContext:
    """One ``rss_ctx`` per entry of ``devices`` for host batches split over several GPUs
    (``rss_hash_host_multi``: contiguous ranges, one host thread per context, counts summed
    on the host).  A device may appear more than once (several contexts on one GPU)."""

    def __init__(self, devices):
        self.contexts = [HostContext(d) for d in devices]
        if not self.contexts:
            raise ValueError("MultiHostContext needs at least one device")
        self._lib = load()

    def close(self):
        for c in self.contexts:
            c.close()

    def hash(self, key, tuples, htable, nqueues, want_hash=True, want_queue=True, want_counts=True,
             reta=None, out=None):
        """Same contract as :meth:`HostContext.hash`, over every context's device."""
        htable, nqueues = queue_modulus(htable, nqueues, reta is not None)
        arr, n, h, q, c = _host_batch(tuples, nqueues, want_hash, want_queue, want_counts, out)
        handles = (ctypes.c_void_p * len(self.contexts))(*[x._ctx.value for x in self.contexts])
        table = _reta_table(reta, htable) if reta is not None else None
        _check(self._lib.rss_hash_host_multi(handles, len(self.contexts), ctypes.byref(key),
                                             ptr(arr), n, htable, ptr(table), nqueues, ptr(h),
                                             ptr(q), ptr(c), 0), "rss_hash_host_multi")
        return h, q, c

    def hash6(self, key6, tuples6, htable, nqueues, want_hash=True, want_queue=True,
              want_counts=True, reta=None, out=None):
        """IPv6 counterpart of :meth:`hash`: the same contiguous ranges as
        ``rss_hash_host_multi`` (``sharding.shard_range``), one host thread per context
        (ctypes releases the GIL) writing its range of the outputs in place (``out`` as for
        :meth:`hash`), counts summed here."""
        qn = queue_modulus(htable, nqueues, reta is not None)[1]
        arr, n, h, q, _ = _host_batch(tuples6, qn, want_hash, want_queue, False, out, ipv6=True)
        k = len(self.contexts)
        base, extra = divmod(n, k)
        bounds = [base * i + min(i, extra) for i in range(k + 1)]
        counts = [None] * k
        errors = []

        def work(i):
            a, b = bounds[i], bounds[i + 1]
            try:
                part = (None if h is None else h[a:b], None if q is None else q[a:b])
                counts[i] = self.contexts[i].hash6(key6, arr[a:b], htable, nqueues, want_hash,
                                                   want_queue, want_counts, reta, out=part)[2]
            except Exception as err:  # re-raised on the calling thread
                errors.append(err)

        workers = [threading.Thread(target=work, args=(i,)) for i in range(1, k)]
        for w in workers:
            w.start()
        work(0)
        for w in workers:
            w.join()
        if errors:
            raise errors[0]
        c = np.sum(counts, axis=0, dtype=np.uint64) if want_counts else None
        return h, q, c


def default_context():
    """Process-wide HostContext on device ``$RSS_DEVICE`` (default 0), created on first use."""
    global _default_ctx
    with _ctx_lock:
        if _default_ctx is None:
            _default_ctx = HostContext(int(os.environ.get("RSS_DEVICE", "0")))
        return _default_ctx


_multi_ctx = {}


def host_context(devices=None):
    """The context a host batch runs on: :func:`default_context` for ``devices`` None,
    else a process-wide :class:`MultiHostContext` over ``devices`` (a sequence of device
    ids; one may repeat, for several contexts on one GPU), created on first use."""
    if devices is None:
        return default_context()
    devs = tuple(int(d) for d in devices)
    if not devs:
        raise ValueError("devices must name at least one GPU")
    with _ctx_lock:
        ctx = _multi_ctx.get(devs)
        if ctx is None:
            ctx = _multi_ctx[devs] = MultiHostContext(devs)
        return ctx


# ------------------------------------------------------- device pointers ----
def hash_device(key, tuples_ptr, n, htable, nqueues, hash_ptr=None, queue_ptr=None,
                counts_ptr=None, flags=0, stream=None, workspace_ptr=None):
    """Stream-ordered ``rss_hash_device`` on raw device pointers (ints); ``counts_ptr``
    holds ``queue_modulus(htable, nqueues)[1]`` entries.  With ``workspace_ptr`` (a zeroed
    device buffer of :func:`counts_workspace_bytes` bytes, one launch at a time) the
    launch is ``rss_hash_device_ws``: single-pass counts, no zeroing launch before it."""
    htable, nqueues = queue_modulus(htable, nqueues)
    if workspace_ptr is None:
        _check(load().rss_hash_device(ctypes.byref(key), tuples_ptr, n, htable, nqueues,
                                      hash_ptr, queue_ptr, counts_ptr, flags, stream),
               "rss_hash_device")
    else:
        _check(load().rss_hash_device_ws(ctypes.byref(key), tuples_ptr, n, htable, nqueues,
                                         hash_ptr, queue_ptr, counts_ptr, flags, workspace_ptr,
                                         stream), "rss_hash_device_ws")


def counts_workspace_bytes(htable, nqueues):
    """Bytes of the single-pass counts workspace of ``rss_hash_device_ws`` for (H, Q)."""
    nqueues = queue_modulus(htable, nqueues)[1]
    out = ctypes.c_size_t()
    _check(load().rss_counts_workspace_bytes(nqueues, ctypes.byref(out)),
           "rss_counts_workspace_bytes")
    return out.value


def hash_device_reta(key, tuples_ptr, n, htable, reta, nqueues, hash_ptr=None, queue_ptr=None,
                     counts_ptr=None, flags=0, stream=None):
    """Stream-ordered ``rss_hash_device_reta`` (``reta``: host sequence of htable queue ids)."""
    htable, nqueues = queue_modulus(htable, nqueues, True)
    table = np.ascontiguousarray(reta, dtype=np.uint32)
    if len(table) != htable:
        raise ValueError("indirection table has %d entries, htable is %d" % (len(table), htable))
    _check(load().rss_hash_device_reta(ctypes.byref(key), tuples_ptr, n, htable,
                                       table.ctypes.data, nqueues, hash_ptr, queue_ptr,
                                       counts_ptr, flags, stream), "rss_hash_device_reta")


def hash6_device(key6, tuples_ptr, n, htable, nqueues, hash_ptr=None, queue_ptr=None,
                 counts_ptr=None, flags=0, stream=None, workspace_ptr=None):
    """Stream-ordered ``rss_hash6_device`` on raw device pointers (ints); with
    ``workspace_ptr`` (as :func:`hash_device`) ``rss_hash6_device_ws``: single-pass counts."""
    htable, nqueues = queue_modulus(htable, nqueues)
    if workspace_ptr is None:
        _check(load().rss_hash6_device(ctypes.byref(key6), tuples_ptr, n, htable, nqueues,
                                       hash_ptr, queue_ptr, counts_ptr, flags, stream),
               "rss_hash6_device")
    else:
        _check(load().rss_hash6_device_ws(ctypes.byref(key6), tuples_ptr, n, htable, nqueues,
                                          hash_ptr, queue_ptr, counts_ptr, flags, workspace_ptr,
                                          stream), "rss_hash6_device_ws")


def hash6_device_reta(key6, tuples_ptr, n, htable, reta, nqueues, hash_ptr=None, queue_ptr=None,
                      counts_ptr=None, flags=0, stream=None):
    """Stream-ordered ``rss_hash6_device_reta`` (``reta``: host sequence of htable queue ids)."""
    htable, nqueues = queue_modulus(htable, nqueues, True)
    table = _reta_table(reta, htable)
    _check(load().rss_hash6_device_reta(ctypes.byref(key6), tuples_ptr, n, htable,
                                        table.ctypes.data, nqueues, hash_ptr, queue_ptr,
                                        counts_ptr, flags, stream), "rss_hash6_device_reta")


def key_search_device(windows_ptr, nkeys, tuples_ptr, n, htable, nqueues, counts_ptr,
                      stream=None):
    """Stream-ordered ``rss_key_search_device`` on raw device pointers (ints)."""
    htable, nqueues = queue_modulus(htable, nqueues)
    _check(load().rss_key_search_device(windows_ptr, nkeys, tuples_ptr, n, htable, nqueues,
                                        counts_ptr, stream), "rss_key_search_device")


def generate_device(seed, first_index, n, tuples_ptr, stream=None):
    """Stream-ordered ``rss_generate_tuples`` into a device buffer of n * 12 bytes."""
    _check(load().rss_generate_tuples(seed, first_index, n, tuples_ptr, stream),
           "rss_generate_tuples")


# ------------------------------------------------------------ CSV fast path --
def parse_dotted(cells, canonical=False):
    """``(ok, value)`` for a sequence of ``str`` cells (``rss_parse_dotted``): ``ok[i]``
    whether cell i is a plain ``d.d.d.d`` quad (1-3 digits per octet) -- with
    ``canonical``, whether it is also canonical (octets 0..255, no leading zeros) --
    ``value[i]`` its ``__ip_to_int`` value mod 2**32; None when the cells cannot be joined
    into one '\n'-separated UTF-8 text of exactly ``len(cells)`` cells (the caller then
    converts them one by one)."""
    n = len(cells)
    try:
        text = "\n".join(cells).encode("utf-8")
    except (TypeError, UnicodeEncodeError):
        return None
    out = np.empty(n, dtype=np.uint32)
    ok = np.empty(n, dtype=np.uint8)
    if load().rss_parse_dotted(text, len(text), n, out.ctypes.data, ok.ctypes.data) != 0:
        return None  # a cell holding '\n'
    return (ok == 2 if canonical else ok > 0), out


def parse_ipv6(cells):
    """``(ok, words)`` for a sequence of ``str`` IPv6 cells (``rss_parse_ipv6``): ``ok[i]``
    whether cell i is plain RFC 4291 text (no embedded IPv4 part, no zone), ``words[i]`` its
    four big-endian-valued words; None as :func:`parse_dotted`."""
    n = len(cells)
    try:
        text = "\n".join(cells).encode("utf-8")
    except (TypeError, UnicodeEncodeError):
        return None
    out = np.empty((n, 4), dtype=np.uint32)
    ok = np.empty(n, dtype=np.uint8)
    if load().rss_parse_ipv6(text, len(text), n, out.ctypes.data, ok.ctypes.data) != 0:
        return None
    return ok.astype(bool), out


def csv_parse(data, threads=0):
    """Parse a canonical 4-tuple CSV image (bytes / uint8 array).

    Returns ``(tuples, layout)`` or ``None`` when the file is not canonical
    (``RSS_ENOTSUP``): the caller then takes the pandas path.
    """
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    lib = load()
    cap = len(buf) // 19 + 1  # a canonical row takes >= 19 bytes ("0.0.0.0,0.0.0.0,0,0\n")
    tuples = np.empty(cap, dtype=TUPLE_DTYPE)
    n = ctypes.c_size_t(0)
    layout = RssCsvLayout()
    rc = lib.rss_csv_parse(buf.ctypes.data, len(buf), tuples.ctypes.data, cap, ctypes.byref(n),
                           ctypes.byref(layout), threads)
    if rc == ENOTSUP:
        return None
    _check(rc, "rss_csv_parse")
    return tuples[:n.value], layout


def csv_format(tuples, hashes, queues, counts, layout, threads=0):
    """Statistics CSV bytes (write_statistics layout) as a uint8 array."""
    lib = load()
    n, nq = len(tuples), len(counts)
    tuples = np.ascontiguousarray(tuples, dtype=TUPLE_DTYPE)
    hashes = np.ascontiguousarray(hashes, dtype=np.uint32)
    queues = np.ascontiguousarray(queues, dtype=np.uint32)
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    cap = lib.rss_csv_format_bound(n, nq)
    out = np.empty(cap, dtype=np.uint8)
    out_len = ctypes.c_size_t(0)
    _check(lib.rss_csv_format(tuples.ctypes.data, hashes.ctypes.data, queues.ctypes.data, n,
                              counts.ctypes.data, nq, ctypes.byref(layout), out.ctypes.data, cap,
                              ctypes.byref(out_len), threads), "rss_csv_format")
    return out[:out_len.value]


def csv_parse6(data, threads=0):
    """Parse a canonical IPv6 4-tuple CSV image: ``(tuples6, spans, layout)`` with
    ``spans`` uint64 (n, 2) = byte range of each row's text, or ``None`` when the file
    is not canonical (the pandas path then runs)."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    lib = load()
    cap = len(buf) // 9 + 1  # a canonical row takes >= 9 bytes ("::,::,0,0\n")
    tuples = np.empty(cap, dtype=TUPLE6_DTYPE)
    spans = np.empty((cap, 2), dtype=np.uint64)
    n = ctypes.c_size_t(0)
    layout = RssCsvLayout()
    rc = lib.rss_csv_parse6(buf.ctypes.data, len(buf), tuples.ctypes.data, spans.ctypes.data, cap,
                            ctypes.byref(n), ctypes.byref(layout), threads)
    if rc == ENOTSUP:
        return None
    _check(rc, "rss_csv_parse6")
    return tuples[:n.value], spans[:n.value], layout


def csv_format6(data, spans, hashes, queues, counts, layout, threads=0):
    """Statistics CSV bytes for IPv6 rows: each row's input text + hash + queue."""
    lib = load()
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    spans = np.ascontiguousarray(spans, dtype=np.uint64)
    n, nq = len(spans), len(counts)
    hashes = np.ascontiguousarray(hashes, dtype=np.uint32)
    queues = np.ascontiguousarray(queues, dtype=np.uint32)
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    cap = lib.rss_csv_format6_bound(spans.ctypes.data, n, nq)
    out = np.empty(cap, dtype=np.uint8)
    out_len = ctypes.c_size_t(0)
    _check(lib.rss_csv_format6(buf.ctypes.data, spans.ctypes.data, hashes.ctypes.data,
                               queues.ctypes.data, n, counts.ctypes.data, nq, ctypes.byref(layout),
                               out.ctypes.data, cap, ctypes.byref(out_len), threads),
           "rss_csv_format6")
    return out[:out_len.value]


# ------------------------------------------------------------------ pcap ----
def pcap_parse(data, ipv6=False):
    """pcap / pcapng image -> ``(tuples, protocols, skipped)`` or None if neither.
    ``ipv6``: one ``TUPLE6_DTYPE`` per IPv6 packet instead of one 4-tuple per IPv4 one."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    lib = load()
    cap = len(buf) // 36 + 1  # a packet record holds >= 16 B of header + a 20 B IP header
    tuples = np.empty(cap, dtype=TUPLE6_DTYPE if ipv6 else TUPLE_DTYPE)
    protos = np.empty(cap, dtype=np.uint8)
    n, skipped = ctypes.c_size_t(0), ctypes.c_size_t(0)
    fn, name = (lib.rss_pcap_parse6, "rss_pcap_parse6") if ipv6 else (lib.rss_pcap_parse,
                                                                       "rss_pcap_parse")
    rc = fn(buf.ctypes.data, len(buf), tuples.ctypes.data, protos.ctypes.data, cap,
            ctypes.byref(n), ctypes.byref(skipped))
    if rc == ENOTSUP:
        return None
    _check(rc, name)
    return tuples[:n.value], protos[:n.value], skipped.value
