"""``rss_simulator.main`` -> ``rss_simulator_nvidia_amd.main`` (import-compatible name)."""
from rss_simulator_nvidia_amd.main import build_parser, main, parse_args  # noqa: F401
