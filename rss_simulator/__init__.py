"""Import-compatible package name of the reference (``rss_simulator``), so its callers
run unchanged: every module re-exports the MI355X implementation in
``rss_simulator_nvidia_amd`` (no reference code here)."""
from rss_simulator_nvidia_amd.main import main

__all__ = ["main"]
