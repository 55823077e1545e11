"""``rss_simulator.simulator`` -> ``rss_simulator_nvidia_amd.simulator`` (import-compatible name)."""
from rss_simulator_nvidia_amd.simulator import *  # noqa: F401,F403
