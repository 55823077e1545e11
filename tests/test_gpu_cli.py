"""CLI end to end on the GPU: the reference's recorded runs replayed through main()
with the real gfx950 path (byte-identical CSVs, same stdout / errors / exit codes)."""
import pytest

from cli_cases import check_edge, check_example, edge_params, example_params

pytestmark = pytest.mark.gpu


@example_params
def test_example_csv_bytes_gpu(name, want_stdout, tmp_path, capsys):
    check_example(name, want_stdout, tmp_path, capsys)


@edge_params
def test_edge_cases_gpu(name, case, tmp_path, capsys, monkeypatch):
    check_edge(name, case, tmp_path, capsys, monkeypatch)
