"""Entry point of ``python -m rss_simulator_nvidia_amd``: the same program as ``rss-simulator``."""
from rss_simulator_nvidia_amd.main import main as _cli

if __name__ == "__main__":
    _cli()
