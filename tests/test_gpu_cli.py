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


def _assert_written_table_is_oracles(out_bytes, src, H, Q, oracle_lib, key):
    """The written statistics file against the C oracle, not against another product path:
    the input rows packed by the oracle's own ``ip_to_u32`` / ``pack_ports`` (``toeplitz.py:
    100-142``), hashed by ``oracle_run``; the table's ``hash_result`` / ``queue_number`` and
    the counts section (``value_counts().sort_index()``, ``simulator.py:107-113``) must be its
    results, and the table's 4-tuple columns the input's."""
    import io

    import numpy as np
    import pandas as pd

    from oracle import oracle as o
    src_df = pd.read_csv(src)
    tup = np.array([[o.ip_to_u32(a), o.ip_to_u32(b), o.pack_ports(int(c), int(d))]
                    for a, b, c, d in zip(src_df["src_ip"], src_df["dst_ip"], src_df["src_port"],
                                          src_df["dst_port"])], dtype=np.uint32).reshape(-1, 3)
    ho, qo, co = oracle_lib.run(key, tup, H, Q)
    head, rows = out_bytes.decode().split("src_ip,", 1)
    table = pd.read_csv(io.StringIO("src_ip," + rows))
    assert list(table.columns[:4]) == list(src_df.columns[:4])
    for col in src_df.columns[:4]:
        assert table[col].astype(str).tolist() == src_df[col].astype(str).tolist(), col
    np.testing.assert_array_equal(table["hash_result"].to_numpy().astype(np.uint64), ho)
    np.testing.assert_array_equal(table["queue_number"].to_numpy().astype(np.uint64), qo)
    counts = pd.read_csv(io.StringIO(head))
    nz = np.flatnonzero(co)
    np.testing.assert_array_equal(counts["queue_number"].to_numpy(), nz)
    np.testing.assert_array_equal(counts["counts"].to_numpy().astype(np.uint64), co[nz])


def test_fast_path_equals_pandas_path_large(tmp_path, monkeypatch, capsys, oracle_lib,
                                            example_key):
    """300K generated canonical rows: native CSV path == pandas path, byte for byte, and
    the table and counts are the oracle's."""
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
    _assert_written_table_is_oracles(outs["1"], src, 512, 24, oracle_lib, example_key)


@pytest.mark.parametrize("device_csv", ["1", "0"])
def test_many_queues_csv_paths_equal_pandas(tmp_path, monkeypatch, capsys, device_csv, oracle_lib,
                                            example_key):
    """--num-queues 20000 (the many-queues ranges on the device CSV path and on the host text
    path) writes the same bytes as the pandas path, and they are the oracle's table."""
    import os
    import subprocess

    from cli_cases import GOLDEN, run_main
    root = os.path.dirname(GOLDEN.rstrip("/").rsplit("/", 1)[0])
    gen = str(tmp_path / "gen_csv")
    subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(root, "tools", "gen_csv.c")], check=True)
    src = str(tmp_path / "in.csv")
    subprocess.run([gen, "50000", "77", src], check=True)
    monkeypatch.setenv("RSS_CSV_DEVICE", device_csv)
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("RSS_CSV_FASTPATH", mode)
        out = str(tmp_path / ("out%s.csv" % mode))
        status, _, _, exc = run_main(
            ["--key-file", os.path.join(GOLDEN, "example_input", "hash_key.txt"),
             "--ips-file", src, "--htable-size", "1048576", "--num-queues", "20000", "--csv", out],
            capsys)
        assert status == 0, exc
        outs[mode] = open(out, "rb").read()
    assert outs["1"] == outs["0"]
    # the counts section is the bincount of the queue column, which is hash % H % Q
    import io

    import numpy as np
    import pandas as pd
    text = outs["1"].decode()
    head, rows = text.split("src_ip,", 1)
    table = pd.read_csv(io.StringIO("src_ip," + rows))
    h = table["hash_result"].to_numpy().astype(np.uint64)
    q = table["queue_number"].to_numpy()
    np.testing.assert_array_equal(q, ((h % np.uint64(1048576)) % np.uint64(20000)).astype(q.dtype))
    counts = pd.read_csv(io.StringIO(head))
    bc = np.bincount(q, minlength=20000)
    np.testing.assert_array_equal(counts["counts"].to_numpy(), bc[counts["queue_number"].to_numpy()])
    assert int(counts["counts"].sum()) == len(q) == 50000
    _assert_written_table_is_oracles(outs["1"], src, 1048576, 20000, oracle_lib, example_key)


@pytest.mark.parametrize("H,Q", [(128, 24), (1 << 20, 20000)])
def test_csv_device_path_4m_rows_vs_oracle(tmp_path, capsys, oracle_lib, example_key, H, Q):
    """4M canonical rows (tools/gen_csv.c: row i is the splitmix64 tuple i of the seed, i.e.
    exactly oracle_generate's) through the CLI's default device CSV path; the written table's
    hash_result / queue_number columns and the counts section against oracle_run on the same
    tuples, the 4-tuple text of the first and last rows against the input."""
    import os
    import subprocess

    import numpy as np
    import pandas as pd

    from cli_cases import GOLDEN, run_main
    root = os.path.dirname(GOLDEN.rstrip("/").rsplit("/", 1)[0])
    gen = str(tmp_path / "gen_csv")
    subprocess.run(["gcc", "-O2", "-o", gen, os.path.join(root, "tools", "gen_csv.c")], check=True)
    n, seed = 4_000_000, 4711
    src, out = str(tmp_path / "in.csv"), str(tmp_path / "out.csv")
    subprocess.run([gen, str(n), str(seed), src], check=True)
    status, so, _, exc = run_main(
        ["--key-file", os.path.join(GOLDEN, "example_input", "hash_key.txt"), "--ips-file", src,
         "--htable-size", str(H), "--num-queues", str(Q), "--csv", out], capsys)
    assert status == 0, exc
    ho, qo, co = oracle_lib.run(example_key, oracle_lib.generate(seed, 0, n), H, Q, threads=16)
    with open(out, "rb") as f:
        data = f.read()
    head, rows = data.split(b"src_ip,dst_ip,src_port,dst_port,hash_result,queue_number\n", 1)
    counts = np.loadtxt(head.decode().splitlines()[1:], delimiter=",", dtype=np.uint64, ndmin=2)
    nz = np.flatnonzero(co)
    np.testing.assert_array_equal(counts[:, 0], nz)
    np.testing.assert_array_equal(counts[:, 1], co[nz])
    table = pd.read_csv(out, skiprows=len(head.decode().splitlines()) + 1, header=None,
                        usecols=[4, 5], names=["h", "q"], dtype=np.uint64)
    np.testing.assert_array_equal(table["h"].to_numpy(), ho.astype(np.uint64))
    np.testing.assert_array_equal(table["q"].to_numpy(), qo.astype(np.uint64))
    lines = rows.split(b"\n")
    with open(src, "rb") as f:
        src_lines = f.read().split(b"\n")
    for i in (0, 1, n // 2, n - 1):
        assert lines[i].rsplit(b",", 2)[0] == src_lines[i + 1]
