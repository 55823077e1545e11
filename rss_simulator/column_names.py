"""``rss_simulator.column_names`` -> ``rss_simulator_nvidia_amd.column_names`` (import-compatible name)."""
from rss_simulator_nvidia_amd.column_names import *  # noqa: F401,F403
