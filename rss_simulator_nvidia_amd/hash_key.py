"""Hash-key text format -- mirrors ``rss_simulator/hash_key.py``.

A key file holds 40 or 52 colon-separated hex bytes (``hash_key.py:25-28``); a
single trailing newline is tolerated because ``$`` matches before it.
"""
import re
from random import sample

HASH_KEY_BYTES_LENGTH = 40

_HASH_KEY_RE = re.compile(
    r"^(?:(?:[0-9a-fA-F]{2}:){39}[0-9a-fA-F]{2})$|"
    r"^(?:(?:[0-9a-fA-F]{2}:){51}[0-9a-fA-F]{2})$"
)


class HashKey(object):
    """Hash-key helpers (static methods, as in the reference)."""

    @staticmethod
    def from_str(hash_key):
        """Convert a colon-hex key string to ``List[int]`` (``hash_key.py:12-32``).

        Raises:
            Exception: ``"Bad hash key given:\\n<key>"`` -- the reference's message.
        """
        if not _HASH_KEY_RE.match(hash_key):
            raise Exception("Bad hash key given:\n{hkey}".format(hkey=hash_key))
        return [int(hex_str, 16) for hex_str in hash_key.split(":")]

    @staticmethod
    def from_file(hash_key_file):
        """Read a key file (``hash_key.py:35-50``); same errors as :meth:`from_str`."""
        with open(hash_key_file) as _file:
            hash_key = _file.read()
        return HashKey.from_str(hash_key)

    @staticmethod
    def random_hash_key():
        """40 distinct random bytes (``hash_key.py:53-60``)."""
        return sample(range(256), HASH_KEY_BYTES_LENGTH)
