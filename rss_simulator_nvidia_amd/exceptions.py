"""Exceptions -- ``ParseException`` mirrors ``rss_simulator/exceptions.py:2-3``."""


class ParseException(Exception):
    """Raised when parsing exception occurred (bad or incomplete CSV input)."""


class NativeLibraryError(RuntimeError):
    """The HIP extension (librss_toeplitz.so) is missing or cannot be loaded."""


class DeviceError(RuntimeError):
    """The HIP runtime reported a failure (no gfx950 device, allocation, launch)."""
