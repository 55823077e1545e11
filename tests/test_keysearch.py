"""Key search host logic on CPU (device call replaced by the oracle): candidate shape,
ideal slot shares, balance metrics, ranking and the CLI."""
import os

import numpy as np
import pytest

from rss_simulator_nvidia_amd import _native, keysearch
from test_cli_host import OracleContext


def test_random_keys_shape_and_reproducibility():
    a = keysearch.random_keys(50, seed=3)
    assert a == keysearch.random_keys(50, seed=3)
    assert a != keysearch.random_keys(50, seed=4)
    for k in a:
        assert len(k) == 40 and len(set(k)) == 40 and all(0 <= b < 256 for b in k)
    text = keysearch.key_text(a[0])
    from rss_simulator_nvidia_amd.hash_key import HashKey
    assert HashKey.from_str(text) == a[0]


@pytest.mark.parametrize("H,Q", [(128, 24), (100, 7), (8, 100), (1, 1), (512, 64)])
def test_slot_share_matches_bucket_mapping(H, Q):
    want = np.bincount(np.arange(H) % Q, minlength=Q) / H
    np.testing.assert_allclose(keysearch.slot_share(H, Q), want)


def test_balance_metrics():
    # H=128, Q=24: queues 0..7 own 6 buckets, 8..23 own 5
    ideal = np.array([6] * 8 + [5] * 16, dtype=np.float64) * 1000
    perfect = ideal.astype(np.uint64)
    skewed = perfect.copy()
    skewed[0] += 600
    skewed[23] -= 600
    m = keysearch.balance(np.stack([perfect, skewed]), 128, 24)
    np.testing.assert_allclose(m["max_load"], [1.0, 6600 / 6000])
    np.testing.assert_allclose(m["chi2"], [0.0, 600 ** 2 / 6000 + 600 ** 2 / 5000])
    assert list(m["used"]) == [24, 24]


def test_search_ranks_by_balance(monkeypatch, oracle_lib):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    tuples = oracle_lib.generate(1, 0, 5000)
    ranked = keysearch.search(tuples, 128, 24, n_keys=12, seed=7, top=12)
    loads = [r["max_load"] for r in ranked]
    assert loads == sorted(loads)
    for r in ranked:
        _, _, c = oracle_lib.run(r["key"], tuples, 128, 24)
        np.testing.assert_array_equal(r["counts"], c)


@pytest.mark.parametrize("H,Q", [(16, 24), (128, 129), (8, 4 * 10 ** 9)])
def test_search_with_more_queues_than_buckets(monkeypatch, oracle_lib, H, Q):
    """the device returns count rows min(H, Q) wide (``queue_modulus``), so
    ``balance`` must score them against the first min(H, Q) slot shares (queues >= H own
    no bucket) instead of broadcasting against all Q."""
    ctx = OracleContext(oracle_lib)
    width = _native.queue_modulus(H, Q)[1]
    assert width == min(H, Q)

    class NarrowContext:
        def key_search(self, keys, tuples, htable, nqueues):
            return np.stack([ctx.hash(k, tuples, htable, width)[2] for k in keys])

    monkeypatch.setattr(_native, "default_context", lambda: NarrowContext())
    tuples = oracle_lib.generate(1, 0, 3000)
    ranked = keysearch.search(tuples, H, Q, n_keys=6, seed=1, top=6)
    assert len(ranked) == 6
    for r in ranked:
        assert r["counts"].shape == (width,) and int(r["counts"].sum()) == 3000
        assert r["max_load"] >= 1.0 and r["used"] <= width
    m = keysearch.balance(np.full((1, width), 10, np.uint64), H, Q)
    np.testing.assert_allclose(m["max_load"], [1.0])  # every bucket its own queue, all equal
    np.testing.assert_allclose(m["chi2"], [0.0])


def test_cli_writes_best_key(monkeypatch, oracle_lib, golden_dir, tmp_path, capsys):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    out = tmp_path / "best.txt"
    ranked = keysearch.main(["--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
                             "--htable-size", "128", "--num-queues", "24", "--keys", "16",
                             "--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
                             "--out", str(out)])
    text = out.read_text()
    assert text == keysearch.key_text(ranked[0]["key"])
    assert "given key: max_load" in capsys.readouterr().out
