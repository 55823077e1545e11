"""``rss_simulator.arg_parse_types.arg_parse_type_decorator`` (import-compatible name)."""
from rss_simulator_nvidia_amd.arg_parse_types.arg_parse_type_decorator import *  # noqa: F401,F403
