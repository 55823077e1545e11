"""The installed ``rss-simulator`` command on MI355X: a wheel of this repo installed into a
scratch directory runs the reference's F1 example (``example_input``, H=128, Q=24) on the
device from the library the wheel carries, and writes the reference's bytes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.mark.timeout(240)
@pytest.mark.parametrize("fast", ["1", "0"])
def test_installed_command_reproduces_example(tmp_path, fast):
    from test_packaging import source_tree
    wheels, site, src = tmp_path / "whl", tmp_path / "site", tmp_path / "src"
    src.mkdir()
    source_tree(str(src))
    subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation",
                    "--no-index", "-q", "-w", str(wheels), str(src)], check=True,
                   cwd=str(tmp_path))
    (whl,) = list(wheels.glob("*.whl"))
    subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-index", "-q",
                    "--target", str(site), str(whl)], check=True)
    out_csv = tmp_path / "out.csv"
    env = dict(os.environ, PYTHONPATH=str(site), RSS_CSV_FASTPATH=fast)
    env.pop("RSS_TOEPLITZ_LIB", None)
    probe = ("import rss_simulator_nvidia_amd._native as n, sys; n.load(); "
             "sys.stdout.write(n.LIB_PATH)")
    lib = subprocess.run([sys.executable, "-c", probe], cwd="/", env=env, capture_output=True,
                         text=True, timeout=120)
    assert lib.returncode == 0, lib.stderr
    assert lib.stdout.startswith(str(site)), lib.stdout
    run = subprocess.run([sys.executable, str(site / "bin" / "rss-simulator"),
                          "--key-file", os.path.join(GOLDEN, "example_input", "hash_key.txt"),
                          "--ips-file", os.path.join(GOLDEN, "example_input", "ips.csv"),
                          "--htable-size", "128", "--num-queues", "24", "--csv", str(out_csv)],
                         cwd="/", env=env, capture_output=True, text=True, timeout=180)
    assert run.returncode == 0, run.stderr
    with open(os.path.join(GOLDEN, "example", "stdout.json")) as f:
        want = json.load(f)["out_h128_q24.csv"]
    assert run.stdout == want.replace("{csv}", str(out_csv))
    with open(os.path.join(GOLDEN, "example", "out_h128_q24.csv"), "rb") as g:
        assert out_csv.read_bytes() == g.read()
