"""Histogram mode on MI355X (reference ``simulator.py:118-172``): every
(H, Q) configuration of ``tests/golden/histogram.json`` -- the figure the reference itself
drew for ``example_input`` -- replayed through ``main()`` without ``--csv`` on the real
device, on all three ingest paths:

* ``device``: canonical file, counts-only device CSV path (``rss_csv_hash_file`` with no
  output file, ``fastcsv.run_counts``);
* ``host``: canonical file, native host parse + the counts-only kernel (``RSS_CSV_DEVICE=0``);
* ``pandas``: the ``Simulator`` path (``RSS_CSV_FASTPATH=0``): ``pd.read_csv`` +
  ``calc_hash`` + ``show_histogram``.

``plt.show`` is replaced by a hook that keeps the figure; bar heights, bar positions, the
caption, title and axis labels must equal the reference's."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

matplotlib = pytest.importorskip("matplotlib")
matplotlib.use("Agg")


@pytest.fixture(scope="module")
def golden(golden_dir):
    with open(os.path.join(golden_dir, "histogram.json")) as f:
        return json.load(f)


PATHS = {"device": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "1"},
         "host": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "0"},
         "pandas": {"RSS_CSV_FASTPATH": "0", "RSS_CSV_DEVICE": "1"}}


@pytest.mark.parametrize("path", sorted(PATHS))
def test_histogram_mode_matches_reference_figure(path, golden, golden_dir, monkeypatch):
    import matplotlib.pyplot as plt

    from rss_simulator_nvidia_amd import _native, fastcsv
    from rss_simulator_nvidia_amd.main import main
    for k, v in PATHS[path].items():
        monkeypatch.setenv(k, v)
    shown = []
    monkeypatch.setattr(plt, "show", lambda *a, **k: shown.append(plt.gcf()))
    # count which device entry point served each run: the histogram must come from the kernel
    calls = {"file": 0, "hash": 0}
    ctx = _native.default_context()
    real_file, real_hash = ctx.csv_hash_file, ctx.hash

    def spy_file(*a, **k):
        calls["file"] += 1
        return real_file(*a, **k)

    def spy_hash(*a, **k):
        calls["hash"] += 1
        return real_hash(*a, **k)

    monkeypatch.setattr(ctx, "csv_hash_file", spy_file)
    monkeypatch.setattr(ctx, "hash", spy_hash)
    for cfg, ref in golden.items():
        h, q = (int(x) for x in cfg.split(","))
        before = dict(calls)
        main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
              "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
              "--htable-size", str(h), "--num-queues", str(q)])
        assert len(shown) == 1, cfg
        fig = shown.pop()
        ax = fig.axes[0]
        assert [p.get_height() for p in ax.patches] == ref["heights"], (path, cfg)
        np.testing.assert_allclose([p.get_x() for p in ax.patches], ref["lefts"], atol=1e-12)
        assert [t.get_text() for t in fig.texts] == ref["caption"], (path, cfg)
        assert (ax.get_title(), ax.get_xlabel(), ax.get_ylabel()) == \
            (ref["title"], ref["xlabel"], ref["ylabel"])
        plt.close(fig)
        if path == "device":
            assert calls["file"] == before["file"] + 1 and calls["hash"] == before["hash"]
        else:
            assert calls["hash"] == before["hash"] + 1
    assert fastcsv.enabled() == (path != "pandas")
