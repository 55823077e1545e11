"""The golden generator refuses to run against anything but the reference tree.

``tests/golden/make_golden.py`` produces every reference fixture by importing
``rss_simulator`` from ``/root/reference``.  This repository also ships an
``rss_simulator`` package (the import-compat shim over the MI355X build), so a path
mishap could otherwise generate the goldens with the build itself -- parity by
self-comparison.  These checks import the script's guards without running it (nothing
here reads /root/reference).
"""
import importlib.util
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tests", "golden", "make_golden.py")


@pytest.fixture(scope="module")
def make_golden():
    spec = importlib.util.spec_from_file_location("make_golden_under_test", SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # module level only: constants and functions
    return mod


def test_guard_refuses_the_build_shim(make_golden):
    shim = types.ModuleType("rss_simulator")
    shim.__file__ = os.path.join(ROOT, "rss_simulator", "__init__.py")
    with pytest.raises(RuntimeError, match="refusing to generate"):
        make_golden.assert_reference_module(shim)


def test_guard_refuses_lookalike_prefix(make_golden, tmp_path):
    # "/root/reference2/..." must not pass as "/root/reference/..."
    ref = tmp_path / "reference"
    ref.mkdir()
    other = tmp_path / "reference2" / "rss_simulator"
    other.mkdir(parents=True)
    mod = types.ModuleType("rss_simulator")
    mod.__file__ = str(other / "__init__.py")
    with pytest.raises(RuntimeError):
        make_golden.assert_reference_module(mod, ref=str(ref))
    inside = ref / "rss_simulator"
    inside.mkdir()
    mod.__file__ = str(inside / "__init__.py")
    assert make_golden.assert_reference_module(mod, ref=str(ref)).startswith(str(ref))


def test_guard_refuses_module_without_file(make_golden):
    with pytest.raises(RuntimeError):
        make_golden.assert_reference_module(types.ModuleType("rss_simulator"))


def test_cli_guard_exits_on_the_build_shim(make_golden):
    """The subprocess guard (run_cli) stops a CLI run that would import this repo's
    ``rss_simulator`` before any of its code runs."""
    code = ("import sys\nsys.path.insert(0, %r)\n" % ROOT) + make_golden.CLI_GUARD + \
        "print('reached main')\n"
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    assert p.returncode == make_golden.GUARD_EXIT, p.stderr
    assert "golden generator guard" in p.stderr
    assert "reached main" not in p.stdout
