"""MI355X-native RSS Toeplitz engine with the ``rss-simulator`` CLI/CSV surface.

Drop-in for noamsto/rss_simulator_nvidia's hot path: the Python
mirror of its interface (``main``, ``Simulator``, ``Toeplitz``, ``HashKey``) over a
C-ABI gfx950 HIP library (``include/rss_toeplitz.h``) loaded through ctypes.
"""
from rss_simulator_nvidia_amd.main import main

__all__ = ["main"]
__version__ = "0.1.0"
