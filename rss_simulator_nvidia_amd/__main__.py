"""``python -m rss_simulator_nvidia_amd`` == ``rss-simulator``."""
from rss_simulator_nvidia_amd import main

main()
