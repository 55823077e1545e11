"""Histogram mode vs the reference's figure (tests/golden/histogram.json): bar heights
and positions, caption, title and labels; and the CLI writes the PNG on both CSV paths
(device call replaced by the oracle, as in test_cli_host.py)."""
import json
import os

import matplotlib
import numpy as np
import pandas as pd
import pytest

from oracle import oracle as o
from rss_simulator_nvidia_amd import _native, histogram
from rss_simulator_nvidia_amd.main import main
from rss_simulator_nvidia_amd.toeplitz import Toeplitz
from test_cli_host import OracleContext

matplotlib.use("Agg")


@pytest.fixture(scope="module")
def golden(golden_dir):
    with open(os.path.join(golden_dir, "histogram.json")) as f:
        return json.load(f)


def example_counts(golden_dir, key, h, q):
    df = pd.read_csv(os.path.join(golden_dir, "example_input", "ips.csv"))
    tup = np.array([[o.ip_to_u32(s), o.ip_to_u32(d), o.pack_ports(sp, dp)]
                    for s, d, sp, dp in zip(df.src_ip, df.dst_ip, df.src_port, df.dst_port)],
                   dtype=np.uint32)
    return o.queue_and_counts(o.hash_batch_np(key, tup), h, q)[1]


def test_figure_matches_reference(golden, golden_dir, example_key):
    import matplotlib.pyplot as plt
    key_str = Toeplitz(example_key).hash_key_str()
    for cfg, ref in golden.items():
        h, q = (int(x) for x in cfg.split(","))
        fig = histogram.figure(example_counts(golden_dir, example_key, h, q), key_str, h, q)
        ax = fig.axes[0]
        assert [p.get_height() for p in ax.patches] == ref["heights"]
        np.testing.assert_allclose([p.get_x() for p in ax.patches], ref["lefts"], atol=1e-12)
        assert [t.get_text() for t in fig.texts] == ref["caption"]
        assert (ax.get_title(), ax.get_xlabel(), ax.get_ylabel()) == \
            (ref["title"], ref["xlabel"], ref["ylabel"])
        plt.close(fig)


@pytest.mark.parametrize("fast", ["1", "0"])
def test_cli_histogram_png(fast, golden_dir, tmp_path, monkeypatch, oracle_lib):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    monkeypatch.setenv("RSS_CSV_FASTPATH", fast)
    out = tmp_path / "hist.png"
    main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
          "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", "128", "--num-queues", "24", "--histogram-png", str(out)])
    assert out.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
