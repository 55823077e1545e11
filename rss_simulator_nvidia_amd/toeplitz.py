"""Toeplitz hash -- drop-in for ``rss_simulator/toeplitz.py`` (``Toeplitz`` class).

Same constructor, ``hash_key`` property/setter, ``hash_key_str()`` and
``compute_hash(src_ip, dst_ip, src_port, dst_port) -> int`` as the reference
(``toeplitz.py:8-69``); the hash itself always runs in the gfx950 kernel behind
``include/rss_toeplitz.h`` (there is no CPU path).  ``compute_hash_batch`` adds the
batched form the kernel is built for.
"""
import numpy as np

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.hash_key import HashKey
from rss_simulator_nvidia_amd.ingest import ip_to_u32, pack_columns


class Toeplitz(object):
    """Toeplitz RSS-hash related functionality (``toeplitz.py:5``)."""

    def __init__(self, hash_key=None, fields=_native.FIELDS_ALL):
        """Initialise with a key (``List[int]``); a random 40-byte key if None/empty.

        ``fields`` (additive): field mask or ethtool letters ``'sdfn'`` selecting the
        hashed fields; the default hashes the whole 4-tuple like the reference."""
        self.__hash_key = hash_key if hash_key else HashKey.random_hash_key()
        self.__fields = fields
        self.__prepared = None
        self.__prepared6 = None

    @property
    def hash_key(self):
        """List representation of the hash key."""
        return self.__hash_key

    @hash_key.setter
    def hash_key(self, hash_key):
        self.__hash_key = hash_key
        self.__prepared = None
        self.__prepared6 = None

    def hash_key_str(self):
        """Colon-separated two-digit hex (``toeplitz.py:37-44``)."""
        return ":".join("{:02x}".format(_hex) for _hex in self.__hash_key)

    @property
    def prepared_key(self):
        """The :class:`rss_simulator_nvidia_amd._native.RssKey` for this key (cached)."""
        if self.__prepared is None:
            self.__prepared = _native.prepare_key(self.__hash_key, self.__fields)
        return self.__prepared

    @property
    def prepared_key6(self):
        """The :class:`rss_simulator_nvidia_amd._native.RssKey6` (IPv6 input) for this key."""
        if self.__prepared6 is None:
            self.__prepared6 = _native.prepare_key6(self.__hash_key, self.__fields)
        return self.__prepared6

    def compute_hash(self, src_ip, dst_ip, src_port, dst_port):
        """Hash one 4-tuple (``toeplitz.py:46-69``); IPs are dotted strings."""
        tuples = pack_columns([ip_to_u32(src_ip)], [ip_to_u32(dst_ip)],
                              [src_port & 0xFFFF], [dst_port & 0xFFFF])
        h, _, _ = _native.default_context().hash(self.prepared_key, tuples, 1, 1,
                                                  want_queue=False, want_counts=False)
        return int(h[0])

    def compute_hash_batch(self, tuples):
        """Hash packed tuples (``rss_tuple4`` structured array or uint32 (n, 3)) -> uint32[n]."""
        h, _, _ = _native.default_context().hash(self.prepared_key, tuples, 1, 1,
                                                  want_queue=False, want_counts=False)
        return h

    def compute_queues(self, tuples, hash_table_size, queue_number, reta=None, devices=None):
        """Hash + ``hash % htable % queues`` (or ``reta[hash % htable]``) + per-queue counts
        in one kernel pass.  Returns ``(hash_u32[n], queue_u32[n], counts_u64[queue_number])``.

        ``devices`` (additive): GPU ids to split the batch over (contiguous ranges, one
        context each, counts summed); None = the default context's one GPU.
        """
        return _native.host_context(devices).hash(self.prepared_key, np.asarray(tuples),
                                                  hash_table_size, queue_number, reta=reta)

    def compute_queues6(self, tuples6, hash_table_size, queue_number, reta=None, devices=None):
        """IPv6 counterpart of :meth:`compute_queues` (``rss_tuple6`` rows)."""
        return _native.host_context(devices).hash6(self.prepared_key6, np.asarray(tuples6),
                                                   hash_table_size, queue_number, reta=reta)
