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


def test_fast_path_equals_pandas_path_large(tmp_path, monkeypatch, capsys):
    """300K generated canonical rows: native CSV path == pandas path, byte for byte."""
    import os
    import subprocess

    from cli_cases import GOLDEN, run_main
    root = os.path.dirname(GOLDEN.rstrip("/").rsplit("/", 1)[0])
    gen = str(tmp_path / "gen_csv")
    subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(root, "tools", "gen_csv.c")], check=True)
    src = str(tmp_path / "in.csv")
    subprocess.run([gen, "300000", "4242", src], check=True)
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("RSS_CSV_FASTPATH", mode)
        out = str(tmp_path / ("out%s.csv" % mode))
        status, so, _, exc = run_main(
            ["--key-file", os.path.join(GOLDEN, "example_input", "hash_key.txt"),
             "--ips-file", src, "--htable-size", "512", "--num-queues", "24", "--csv", out], capsys)
        assert status == 0, exc
        assert so == "Wrote statistics to %s.\n" % out
        outs[mode] = open(out, "rb").read()
    assert outs["1"] == outs["0"]
    assert outs["1"].count(b"\n") == 300000 + 1 + 24 + 1
