"""CLI / CSV host logic on CPU: the reference's recorded runs replayed through main().

The one device call (``HostContext.hash``, used by both the native CSV fast path and
the pandas path) is replaced by the oracle here so that argument parsing, key
parsing, CSV ingest, error messages and both CSV writers are checked without a GPU.
tests/test_gpu_cli.py replays the same cases with the real HIP path.
"""
import numpy as np
import pytest

from cli_cases import check_edge, check_example, edge_params, example_params
from oracle import oracle as o
from rss_simulator_nvidia_amd import _native


class OracleContext:
    """Stands in for _native.HostContext in CPU-only tests (test infrastructure)."""

    def __init__(self, oracle_lib):
        self.oracle_lib = oracle_lib
        self.calls = 0

    def csv_hash_text(self, *args, **kwargs):
        return None  # no device text path on CPU: the host parse/format path runs

    def csv_hash_file(self, *args, **kwargs):
        return None

    def hash(self, key, tuples, htable, nqueues, want_hash=True, want_queue=True,
             want_counts=True, reta=None):
        self.calls += 1
        if tuples.dtype.names:
            arr = np.stack([tuples["sip"], tuples["dip"], tuples["ports"]], axis=1)
        else:
            arr = np.asarray(tuples, dtype=np.uint32).reshape(-1, 3)
        # the prepared key's own windows (field selection remaps them), closed form
        h = o.hash_words_np(np.ctypeslib.as_array(key.window), arr)
        if reta is None:
            q, c = o.queue_and_counts(h, htable, nqueues)
        else:
            q = np.asarray(reta, dtype=np.uint32)[h % htable]
            c = np.bincount(q, minlength=nqueues).astype(np.uint64)
        return h, q, c

    def key_search(self, keys, tuples, htable, nqueues):
        return np.stack([self.hash(k, tuples, htable, nqueues)[2] for k in keys])

    def hash6(self, key6, tuples6, htable, nqueues, want_hash=True, want_queue=True,
              want_counts=True, reta=None):
        self.calls += 1
        words = np.ascontiguousarray(tuples6).view(np.uint32).reshape(-1, 9)
        h = o.hash_words_np(np.ctypeslib.as_array(key6.window), words)
        if reta is None:
            q, c = o.queue_and_counts(h, htable, nqueues)
        else:
            q = np.asarray(reta, dtype=np.uint32)[h % htable]
            c = np.bincount(q, minlength=nqueues).astype(np.uint64)
        return h, q, c


@pytest.fixture(params=["fast", "pandas"])
def oracle_device(request, monkeypatch, oracle_lib):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    monkeypatch.setenv("RSS_CSV_FASTPATH", "1" if request.param == "fast" else "0")


@example_params
def test_example_csv_bytes(oracle_device, name, want_stdout, tmp_path, capsys):
    check_example(name, want_stdout, tmp_path, capsys)


@edge_params
def test_edge_cases(oracle_device, name, case, tmp_path, capsys, monkeypatch):
    check_edge(name, case, tmp_path, capsys, monkeypatch)
