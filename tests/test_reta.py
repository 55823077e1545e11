"""Indirection tables (RETA) host side: ethtool's equal/weight fills, validation, and the
CLI (device call replaced by the oracle).  The reference's mapping is the 'equal' table,
so the golden example outputs must be reproduced through the table path too."""
import os

import numpy as np
import pytest

from cli_cases import check_example, example_cases
from rss_simulator_nvidia_amd import _native, reta
from rss_simulator_nvidia_amd.main import main
from test_cli_host import OracleContext


@pytest.mark.parametrize("H,Q", [(128, 24), (100, 7), (8, 100), (512, 64), (1, 1)])
def test_equal_is_the_reference_mapping(H, Q):
    assert reta.equal(H, Q) == [b % Q for b in range(H)]


def test_weights_like_ethtool():
    assert reta.weights(8, [1, 1]) == [0, 0, 0, 0, 1, 1, 1, 1]
    assert reta.weights(8, [1, 2, 1]) == [0, 0, 1, 1, 1, 1, 2, 2]
    assert reta.weights(6, [0, 1, 0, 1]) == [1, 1, 1, 3, 3, 3]
    t = reta.weights(128, [3, 1, 0, 4])
    assert np.bincount(t, minlength=4).tolist() == [48, 16, 0, 64]
    for bad in ([], [0, 0], [1, -1]):
        with pytest.raises(ValueError):
            reta.weights(8, bad)


def test_validate():
    assert reta.validate([0, 1, 2], 3, 3).tolist() == [0, 1, 2]
    for table, h, q in (([0, 1], 3, 3), ([0, 3, 1], 3, 3), ([-1, 0, 0], 3, 3)):
        with pytest.raises(ValueError):
            reta.validate(table, h, q)
    with pytest.raises(ValueError):
        reta.validate([0] * 1025, 1025, 1)


@pytest.fixture
def oracle_ctx(monkeypatch, oracle_lib):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))


@pytest.mark.parametrize("name,want_stdout", example_cases())
def test_equal_table_file_reproduces_golden(name, want_stdout, oracle_ctx, tmp_path, capsys,
                                            monkeypatch, golden_dir):
    h, q = (int(x[1:]) for x in name[4:-4].split("_"))
    table = tmp_path / "reta.txt"
    table.write_text(" ".join(map(str, reta.equal(h, q))))
    import cli_cases
    orig = cli_cases.main
    monkeypatch.setattr(cli_cases, "main", lambda argv: orig(argv + ["--reta-file", str(table)]))
    check_example(name, want_stdout, tmp_path, capsys)


def test_weights_cli(oracle_ctx, oracle_lib, golden_dir, tmp_path, capsys):
    out = tmp_path / "o.csv"
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    main(["--key-file", key_file, "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", "16", "--num-queues", "4", "--csv", str(out),
          "--reta-weights", "1,0,2,1"])
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    table = reta.weights(16, [1, 0, 2, 1])
    for row in body:
        f = row.split(",")
        assert int(f[5]) == table[int(f[4]) % 16]
    assert not any(r.startswith("1,") for r in lines[1:4])  # weight-0 queue gets nothing
    with pytest.raises(SystemExit):
        main(["--key-file", key_file, "--ips-file", "x", "--htable-size", "16",
              "--num-queues", "4", "--reta-weights", "a,b"])
    capsys.readouterr()
    with pytest.raises(SystemExit) as exc:  # table problems are usage errors (exit 2)
        main(["--key-file", key_file, "--ips-file", os.path.join(golden_dir, "example_input",
              "ips.csv"), "--htable-size", "16", "--num-queues", "4", "--reta-weights", "1,2"])
    assert exc.value.code == 2
    assert "--reta-weights needs one weight per queue (4)" in capsys.readouterr().err
    # the table size is checked before a table of --htable-size entries is built
    with pytest.raises(SystemExit) as exc:
        main(["--key-file", key_file, "--ips-file", "x", "--htable-size", str(10 ** 12),
              "--num-queues", "4", "--reta-weights", "1,1,1,1"])
    assert exc.value.code == 2
    assert "at most 1024 entries" in capsys.readouterr().err
