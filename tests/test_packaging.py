"""The installable drop-in (reference ``setup.py:15-17``, ``rss_simulator/__init__.py:2``,
``__main__.py:2-4``): a wheel built offline from this repo carries the ``rss-simulator``
console script and the gfx950 library, the installed script reproduces the reference's
recorded argparse failures byte for byte, and the import-compatible ``rss_simulator``
package runs the reference's recorded F1 / F4 cases through the entry point (device call
replaced by the oracle, as in test_cli_host.py)."""
import configparser
import glob
import importlib
import json
import os
import subprocess
import sys
import zipfile

import pytest

from cli_cases import GOLDEN, check_edge, check_example, edge_cases, example_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_tree(dest):
    """The files a source distribution would hold, copied out of the checkout: pip builds
    in the source directory, and concurrent test workers must not share one."""
    import shutil
    skip = shutil.ignore_patterns("__pycache__", "*.pyc", "*.o")
    for name in ("setup.py", "pyproject.toml", "README.md"):
        shutil.copy(os.path.join(ROOT, name), os.path.join(dest, name))
    for pkg in ("rss_simulator_nvidia_amd", "rss_simulator"):
        shutil.copytree(os.path.join(ROOT, pkg), os.path.join(dest, pkg), ignore=skip)
    return dest


@pytest.fixture(scope="module")
def wheel(tmp_path_factory):
    src = source_tree(str(tmp_path_factory.mktemp("src")))
    out = tmp_path_factory.mktemp("wheel")
    subprocess.run([sys.executable, "-m", "pip", "wheel", "--no-deps", "--no-build-isolation",
                    "--no-index", "-q", "-w", str(out), src], check=True, cwd=str(out))
    (whl,) = glob.glob(str(out / "*.whl"))
    return whl


@pytest.fixture(scope="module")
def installed(wheel, tmp_path_factory):
    site = tmp_path_factory.mktemp("site")
    subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-index", "-q",
                    "--target", str(site), wheel], check=True)
    return site


def test_wheel_carries_console_script_and_library(wheel):
    with zipfile.ZipFile(wheel) as z:
        names = z.namelist()
        (ep,) = [n for n in names if n.endswith("entry_points.txt")]
        cfg = configparser.ConfigParser()
        cfg.read_string(z.read(ep).decode())
    assert cfg["console_scripts"]["rss-simulator"] == "rss_simulator_nvidia_amd.main:main"
    assert "rss_simulator_nvidia_amd/librss_toeplitz.so" in names
    for mod in ("__init__", "__main__", "main", "toeplitz", "simulator", "hash_key",
                "column_names", "exceptions"):
        assert "rss_simulator/%s.py" % mod in names


def _run_script(installed, args, cwd):
    env = dict(os.environ, PYTHONPATH=str(installed))
    script = os.path.join(str(installed), "bin", "rss-simulator")
    return subprocess.run([sys.executable, script] + args, cwd=cwd, env=env, capture_output=True,
                          text=True, timeout=120)


@pytest.mark.parametrize("name", ["htable_zero", "htable_text", "queues_neg", "key_bad",
                                  "key_41"])
def test_installed_script_argparse_errors_match_reference(installed, name, tmp_path):
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        case = json.load(f)[name]
    assert case["returncode"] == 2
    out = _run_script(installed, case["args"], os.path.join(GOLDEN, "edge"))
    assert (out.returncode, out.stdout, out.stderr) == (2, case["stdout"], case["stderr"])


def test_installed_script_help_names_the_reference_program(installed):
    out = _run_script(installed, ["--help"], ROOT)
    assert out.returncode == 0
    assert out.stdout.startswith("usage: rss-simulator [-h] --key-file PATH --ips-file PATH")
    # the script imports the installed copy, not this checkout
    env = dict(os.environ, PYTHONPATH=str(installed))
    where = subprocess.run([sys.executable, "-c", "import rss_simulator_nvidia_amd as m; "
                            "print(m.__file__)"], cwd="/", env=env, capture_output=True, text=True)
    assert where.stdout.strip().startswith(str(installed))


def _entry_point():
    with open(os.path.join(ROOT, "setup.py")) as f:
        text = f.read()
    spec = text.split('"rss-simulator=', 1)[1].split('"', 1)[0]
    mod, func = spec.split(":")
    return getattr(importlib.import_module(mod), func)


def test_shim_package_reexports_the_implementation():
    import rss_simulator
    from rss_simulator.arg_parse_types import PositiveInt
    from rss_simulator.column_names import ColumnNames
    from rss_simulator.exceptions import ParseException
    from rss_simulator.hash_key import HashKey
    from rss_simulator.simulator import Simulator
    from rss_simulator.toeplitz import Toeplitz
    import rss_simulator_nvidia_amd as impl
    assert rss_simulator.main is impl.main is _entry_point()
    # as in the reference, the package attribute `main` is the function; the module is
    # importable by name
    assert importlib.import_module("rss_simulator.main").main is impl.main
    assert Toeplitz.__module__ == "rss_simulator_nvidia_amd.toeplitz"
    assert Simulator.__module__ == "rss_simulator_nvidia_amd.simulator"
    assert ColumnNames.HASH_RESULT.value == "hash_result"
    assert PositiveInt.parse("7") == 7
    assert HashKey.from_str(":".join(["00"] * 40)) == [0] * 40
    assert issubclass(ParseException, Exception)


@pytest.fixture
def oracle_device(monkeypatch, oracle_lib):
    from test_cli_host import OracleContext

    from rss_simulator_nvidia_amd import _native
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))


@pytest.mark.parametrize("name,want_stdout", example_cases()[:3])
def test_entry_point_replays_example(oracle_device, name, want_stdout, tmp_path, capsys):
    assert _entry_point().__module__ == "rss_simulator_nvidia_amd.main"
    check_example(name, want_stdout, tmp_path, capsys)


@pytest.mark.parametrize("name,case", [c for c in edge_cases()
                                       if c[0] in ("octet_overflow", "ports_wide", "key52",
                                                   "missing_col")])
def test_entry_point_replays_edge_cases(oracle_device, name, case, tmp_path, capsys,
                                        monkeypatch):
    check_edge(name, case, tmp_path, capsys, monkeypatch)
