"""Replay the reference CLI runs recorded in tests/golden (F1 example + F4 edge cases)
through this package's ``main()`` and compare stdout / stderr / exit status / CSV bytes."""
import json
import os
import shutil

import pytest

from rss_simulator_nvidia_amd.main import main

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def example_cases():
    with open(os.path.join(GOLDEN, "example", "stdout.json")) as f:
        stdout = json.load(f)
    return sorted(stdout.items())


def edge_cases():
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        return sorted(json.load(f).items())


def run_main(argv, capsys):
    """Run the CLI in-process; return (exit status, stdout, stderr, exception or None)."""
    status, exc = 0, None
    try:
        main(argv)
    except SystemExit as e:  # argparse errors
        status = e.code
    except Exception as e:  # noqa: BLE001 -- an uncaught exception is exit status 1
        status, exc = 1, e
    out, err = capsys.readouterr()
    return status, out, err, exc


def check_example(name, want_stdout, tmp_path, capsys):
    h, q = (int(x[1:]) for x in name[len("out_"):-len(".csv")].split("_"))
    out = str(tmp_path / name)
    status, so, _, exc = run_main(
        ["--key-file", os.path.join(GOLDEN, "example_input", "hash_key.txt"),
         "--ips-file", os.path.join(GOLDEN, "example_input", "ips.csv"),
         "--htable-size", str(h), "--num-queues", str(q), "--csv", out], capsys)
    assert status == 0, exc
    assert so == want_stdout.replace("{csv}", out)
    with open(out, "rb") as f, open(os.path.join(GOLDEN, "example", name), "rb") as g:
        assert f.read() == g.read()


def check_edge(name, case, tmp_path, capsys, monkeypatch):
    work = tmp_path / "edge"
    shutil.copytree(os.path.join(GOLDEN, "edge"), work)
    for f in os.listdir(work):
        if f.startswith("out_"):
            os.remove(work / f)
    monkeypatch.chdir(work)
    status, so, err, exc = run_main(case["args"], capsys)
    assert status == case["returncode"], (status, exc, err)
    assert so == case["stdout"]
    want_err = case["stderr"]
    if status == 2:  # argparse usage error: whole stderr must match
        assert err == want_err
    elif status == 1:  # uncaught exception: last traceback line
        assert exc is not None
        got = "%s: %s" % (type(exc).__name__, exc)
        ref_type, ref_msg = want_err.split(": ", 1)
        assert type(exc).__name__ == ref_type.rsplit(".", 1)[-1], got
        assert str(exc) == ref_msg, got
    if case["output"]:
        with open(work / case["output"], "rb") as f, \
                open(os.path.join(GOLDEN, "edge", case["output"]), "rb") as g:
            assert f.read() == g.read()
    else:
        assert not os.path.exists(work / ("out_%s.csv" % name))


example_params = pytest.mark.parametrize("name,want_stdout", example_cases())
edge_params = pytest.mark.parametrize("name,case", edge_cases())
