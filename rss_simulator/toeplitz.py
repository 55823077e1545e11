"""``rss_simulator.toeplitz`` -> ``rss_simulator_nvidia_amd.toeplitz`` (import-compatible name)."""
from rss_simulator_nvidia_amd.toeplitz import *  # noqa: F401,F403
