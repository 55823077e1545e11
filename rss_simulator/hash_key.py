"""``rss_simulator.hash_key`` -> ``rss_simulator_nvidia_amd.hash_key`` (import-compatible name)."""
from rss_simulator_nvidia_amd.hash_key import *  # noqa: F401,F403
