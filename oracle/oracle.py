"""CPU oracle for the RSS Toeplitz hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker or the timed CPU baseline.  The
product package (``rss_simulator_nvidia_amd``) never imports it.

Parity pinned: ``tests/test_oracle.py`` checks every function below against the
golden fixtures produced by running the reference itself
(``tests/golden/make_golden.py``).

Contents (each restates noamsto/rss_simulator_nvidia v0.0.2):

* :func:`compute_hash_port` -- pure-Python per-tuple restatement of
  ``Toeplitz.compute_hash`` (``rss_simulator/toeplitz.py:46-69``) that keeps the
  reference's cost structure: the 96-bit input as a bit string, and a full-key
  bit-string rotation per input bit (``__shift_key``, ``toeplitz.py:83-98``).  This
  is the ``"port"`` CPU baseline bench.py times.
* :func:`ip_to_u32`, :func:`pack_ports` -- ``__ip_to_int`` (``toeplitz.py:100-111``)
  and the byte masking of ``__prepare_input_bytes`` (``toeplitz.py:127-142``).
* :func:`hash_batch_np` -- vectorised closed form (window i = key bits [i, i+32)),
  numpy, for mid-size checks.
* :class:`OracleLib` -- ctypes binding of ``oracle/liboracle.so`` (the C restatement
  with the literal rotating key, ``oracle/toeplitz_oracle.c``) for large-N checks, incl.
  ``run_words`` for tuples of any number of words (the 9-word IPv6 tuple).
* :func:`generate_np` -- the splitmix64 synthetic-tuple generator of
  ``include/rss_toeplitz.h`` (``rss_generate_tuples``).
* :func:`queue_and_counts` -- ``simulator.py:94-98`` and the ``value_counts`` of
  ``simulator.py:107-113``.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------- per tuple ----
def ip_to_u32(ip):
    """``toeplitz.py:110-111`` followed by the per-byte masks of ``:130-137``.

    The reference ORs ``int(octet) << shift`` as unbounded Python ints and then
    keeps bytes of the result, i.e. the value modulo 2**32.
    """
    parts = ip.split(".")
    n = int(parts[0]) << 24 | int(parts[1]) << 16 | int(parts[2]) << 8 | int(parts[3])
    return n & 0xFFFFFFFF


def pack_ports(src_port, dst_port):
    """``toeplitz.py:138-141``: each port contributes its low 16 bits."""
    return ((src_port & 0xFFFF) << 16) | (dst_port & 0xFFFF)


def _input_bits(sip, dip, sport, dport):
    data = [(sip >> 24) & 0xFF, (sip >> 16) & 0xFF, (sip >> 8) & 0xFF, sip & 0xFF,
            (dip >> 24) & 0xFF, (dip >> 16) & 0xFF, (dip >> 8) & 0xFF, dip & 0xFF,
            (sport & 0xFF00) >> 8, sport & 0xFF, (dport & 0xFF00) >> 8, dport & 0xFF]
    return "".join(format(b, "08b") for b in data)


def _rotate_key_left(key):
    bits = "".join(format(k, "08b") for k in key)
    bits = bits[1:] + bits[:1]
    return [int(bits[i:i + 8], 2) for i in range(0, len(bits), 8)]


def compute_hash_port(key, src_ip, dst_ip, src_port, dst_port):
    """Per-tuple Toeplitz hash with the reference's literal rotating key."""
    k = list(key)
    bits = _input_bits(ip_to_u32(src_ip), ip_to_u32(dst_ip), src_port, dst_port)
    result = 0
    for b in bits:
        if b == "1":
            result ^= k[0] << 24 | k[1] << 16 | k[2] << 8 | k[3]
        k = _rotate_key_left(k)
    return result


def compute_hash_u32(key, sip, dip, ports):
    """Same, on an already packed tuple (sip, dip, ports = sport << 16 | dport)."""
    k = list(key)
    bits = _input_bits(sip, dip, ports >> 16, ports & 0xFFFF)
    result = 0
    for b in bits:
        if b == "1":
            result ^= k[0] << 24 | k[1] << 16 | k[2] << 8 | k[3]
        k = _rotate_key_left(k)
    return result


FIELD_BYTES = ((1, 0, 4), (2, 4, 4), (4, 8, 2), (8, 10, 2))  # (mask bit, offset, size)


def select_fields_bytes(sip, dip, ports, fields):
    """The hash input for a field mask: selected fields of the 12-byte tuple, concatenated."""
    full = (int(sip).to_bytes(4, "big") + int(dip).to_bytes(4, "big") +
            int(ports).to_bytes(4, "big"))
    return b"".join(full[o:o + n] for bit, o, n in FIELD_BYTES if fields & bit)


# ---------------------------------------------------------------- batches ----
def windows(key):
    """window[i] = key bits [i, i + 32), MSB first (closed form of the rotation)."""
    k = 0
    for b in key[:16]:
        k = (k << 8) | int(b)
    return np.array([(k >> (96 - i)) & 0xFFFFFFFF for i in range(96)], dtype=np.uint32)


def hash_batch_np(key, tuples):
    """Vectorised hash of packed tuples (uint32 array of shape (n, 3))."""
    tuples = np.asarray(tuples, dtype=np.uint32).reshape(-1, 3)
    w = windows(key)
    h = np.zeros(len(tuples), dtype=np.uint32)
    for i in range(96):
        word = tuples[:, i >> 5]
        bit = (word >> np.uint32(31 - (i & 31))) & np.uint32(1)
        h ^= bit * w[i]
    return h


def hash_words_np(windows, words):
    """Closed form for any input length: XOR of windows[i] over the set input bits i of
    big-endian-valued uint32 words (shape (n, len(windows) // 32))."""
    words = np.asarray(words, dtype=np.uint32)
    h = np.zeros(len(words), dtype=np.uint32)
    for i in range(len(windows)):
        bit = (words[:, i >> 5] >> np.uint32(31 - (i & 31))) & np.uint32(1)
        h ^= bit * np.uint32(windows[i])
    return h


def words_to_bytes(row):
    return b"".join(int(w).to_bytes(4, "big") for w in row)


def queue_and_counts(hashes, htable, nqueues):
    """``simulator.py:96-98`` (``hash % htable % nqueues``) + per-queue counts."""
    q = (np.asarray(hashes, dtype=np.uint64) % np.uint64(htable)) % np.uint64(nqueues)
    counts = np.bincount(q.astype(np.int64), minlength=nqueues).astype(np.uint64)
    return q.astype(np.uint32), counts


_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def _mix64(x):
    x = x + _GAMMA
    x = (x ^ (x >> np.uint64(30))) * _M1
    x = (x ^ (x >> np.uint64(27))) * _M2
    return x ^ (x >> np.uint64(31))


def generate_np(seed, first_index, n):
    """splitmix64 synthetic tuples, shape (n, 3) uint32 (see include/rss_toeplitz.h)."""
    with np.errstate(over="ignore"):
        idx = np.arange(first_index, first_index + n, dtype=np.uint64)
        base = np.uint64(seed) + np.uint64(2) * idx
        r0 = _mix64(base)
        r1 = _mix64(base + np.uint64(1))
    out = np.empty((n, 3), dtype=np.uint32)
    out[:, 0] = (r0 >> np.uint64(32)).astype(np.uint32)
    out[:, 1] = (r0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out[:, 2] = (r1 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    return out


# ------------------------------------------------------------------ C lib ----
class OracleLib:
    """ctypes binding of oracle/liboracle.so (built by ``make -C oracle``)."""

    def __init__(self, path=None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError("%s missing: run `make -C oracle`" % path)
        lib = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        lib.oracle_windows.argtypes = [u8p, ctypes.c_size_t, u32p]
        lib.oracle_windows.restype = ctypes.c_int
        lib.oracle_hash_rotating.argtypes = [u8p, ctypes.c_size_t] + [ctypes.c_uint32] * 4
        lib.oracle_hash_rotating.restype = ctypes.c_uint32
        lib.oracle_run.argtypes = [u8p, ctypes.c_size_t, u32p, ctypes.c_size_t, ctypes.c_uint32,
                                   ctypes.c_uint32, u32p, u32p, u64p, ctypes.c_int]
        lib.oracle_run.restype = ctypes.c_int
        lib.oracle_run_tables.argtypes = lib.oracle_run.argtypes
        lib.oracle_run_tables.restype = ctypes.c_int
        lib.oracle_windows_n.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u32p]
        lib.oracle_windows_n.restype = ctypes.c_int
        lib.oracle_hash_bytes.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        lib.oracle_hash_bytes.restype = ctypes.c_uint32
        lib.oracle_run_words.argtypes = [u8p, ctypes.c_size_t, u32p, ctypes.c_int, ctypes.c_size_t,
                                         ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u64p,
                                         ctypes.c_int]
        lib.oracle_run_words.restype = ctypes.c_int
        lib.oracle_generate.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, u32p]
        lib.oracle_generate.restype = None
        self._lib = lib

    @staticmethod
    def _key(key):
        arr = (ctypes.c_uint8 * len(key))(*[int(b) for b in key])
        return arr, len(key)

    def windows(self, key):
        k, n = self._key(key)
        out = np.zeros(96, dtype=np.uint32)
        rc = self._lib.oracle_windows(k, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        if rc:
            raise ValueError("bad key length %d" % n)
        return out

    def hash_rotating(self, key, sip, dip, sport, dport):
        k, n = self._key(key)
        return self._lib.oracle_hash_rotating(k, n, sip, dip, sport, dport)

    def windows_n(self, key, nbits):
        k, n = self._key(key)
        out = np.zeros(nbits, dtype=np.uint32)
        if self._lib.oracle_windows_n(k, n, nbits, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))):
            raise ValueError("bad key length %d" % n)
        return out

    def hash_bytes(self, key, data):
        """Literal rotating-key Toeplitz over an arbitrary byte string."""
        k, n = self._key(key)
        d = (ctypes.c_uint8 * max(1, len(data)))(*bytearray(data))
        return self._lib.oracle_hash_bytes(k, n, d, len(data))

    def run(self, key, tuples, htable, nqueues, threads=None, want_hash=True, want_queue=True,
            fn="oracle_run"):
        """Returns (hash, queue, counts) for packed tuples of shape (n, 3).  ``fn`` =
        ``oracle_run_tables`` runs the byte-table form (the bench's optimised-CPU line)."""
        tuples = np.ascontiguousarray(tuples, dtype=np.uint32).reshape(-1, 3)
        n = len(tuples)
        k, klen = self._key(key)
        h = np.empty(n, dtype=np.uint32) if want_hash else None
        q = np.empty(n, dtype=np.uint32) if want_queue else None
        c = np.zeros(nqueues, dtype=np.uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        rc = getattr(self._lib, fn)(
            k, klen, tuples.ctypes.data_as(u32p), n, htable, nqueues,
            h.ctypes.data_as(u32p) if h is not None else None,
            q.ctypes.data_as(u32p) if q is not None else None,
            c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), threads or os.cpu_count() or 1)
        if rc:
            raise ValueError("%s failed (%d)" % (fn, rc))
        return h, q, c

    def run_words(self, key, words, htable, nqueues, threads=None):
        """(hash, queue, counts) for tuples of big-endian-valued uint32 words, shape (n, W):
        W = 9 is the 36-byte IPv6 tuple (``oracle_run_words``, the literal loop's windows)."""
        words = np.ascontiguousarray(words, dtype=np.uint32)
        n, nw = words.shape
        k, klen = self._key(key)
        h = np.empty(n, dtype=np.uint32)
        q = np.empty(n, dtype=np.uint32)
        c = np.zeros(nqueues, dtype=np.uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        rc = self._lib.oracle_run_words(k, klen, words.ctypes.data_as(u32p), nw, n, htable, nqueues,
                                        h.ctypes.data_as(u32p), q.ctypes.data_as(u32p),
                                        c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        threads or os.cpu_count() or 1)
        if rc:
            raise ValueError("oracle_run_words failed (%d)" % rc)
        return h, q, c

    def generate(self, seed, first_index, n):
        out = np.empty((n, 3), dtype=np.uint32)
        self._lib.oracle_generate(seed, first_index, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        return out
