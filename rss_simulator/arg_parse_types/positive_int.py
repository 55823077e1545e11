"""``rss_simulator.arg_parse_types.positive_int`` (import-compatible name)."""
from rss_simulator_nvidia_amd.arg_parse_types.positive_int import *  # noqa: F401,F403
