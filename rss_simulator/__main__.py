"""``python -m rss_simulator``: the ``rss-simulator`` command."""
from rss_simulator_nvidia_amd.main import main

if __name__ == "__main__":
    main()
