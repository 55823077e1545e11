"""``rss_simulator.arg_parse_types`` -> ``rss_simulator_nvidia_amd.arg_parse_types``."""
from rss_simulator_nvidia_amd.arg_parse_types import *  # noqa: F401,F403
