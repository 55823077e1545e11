"""``rss_simulator.exceptions`` -> ``rss_simulator_nvidia_amd.exceptions`` (import-compatible name)."""
from rss_simulator_nvidia_amd.exceptions import *  # noqa: F401,F403
