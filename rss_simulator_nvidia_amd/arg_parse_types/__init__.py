"""argparse type helpers -- mirrors ``rss_simulator/arg_parse_types/__init__.py``."""
from rss_simulator_nvidia_amd.arg_parse_types.arg_parse_type_decorator import arg_parse_type_decorator
from rss_simulator_nvidia_amd.arg_parse_types.positive_int import PositiveInt

__all__ = ["arg_parse_type_decorator", "PositiveInt"]
