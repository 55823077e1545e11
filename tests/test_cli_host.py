"""CLI / CSV host logic on CPU: the reference's recorded runs replayed through main().

The one device call (``Toeplitz.compute_queues``) is replaced by the oracle here so
that argument parsing, key parsing, CSV ingest, error messages and the CSV writer
are checked without a GPU.  tests/test_gpu_cli.py replays the same cases with the
real HIP path.
"""
import numpy as np
import pytest

from cli_cases import check_edge, check_example, edge_params, example_params
from rss_simulator_nvidia_amd.toeplitz import Toeplitz


@pytest.fixture
def oracle_device(monkeypatch, oracle_lib):
    def compute_queues(self, tuples, htable, nqueues):
        arr = np.stack([tuples["sip"], tuples["dip"], tuples["ports"]], axis=1)
        return oracle_lib.run(self.hash_key, arr, htable, nqueues, threads=2)
    monkeypatch.setattr(Toeplitz, "compute_queues", compute_queues)


@example_params
def test_example_csv_bytes(oracle_device, name, want_stdout, tmp_path, capsys):
    check_example(name, want_stdout, tmp_path, capsys)


@edge_params
def test_edge_cases(oracle_device, name, case, tmp_path, capsys, monkeypatch):
    check_edge(name, case, tmp_path, capsys, monkeypatch)
