"""Load the reference-side ctypes stub exactly as INTEGRATION.md prints it (test helper).

The first ```python block of INTEGRATION.md is the module a reference maintainer would add
(``rss_simulator/gpu_backend.py``); it is executed here with ``LIB`` pointed at this
tree's ``librss_toeplitz.so``, so the tests check the documented binding, not a copy.
"""
import os
import re
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "rss_simulator_nvidia_amd", "librss_toeplitz.so")


def load_stub():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        text = f.read()
    code = re.search(r"```python\n(.*?)```", text, re.S).group(1)
    placeholder = '"/path/to/rss_simulator_nvidia_amd/librss_toeplitz.so"'
    assert placeholder in code
    mod = types.ModuleType("gpu_backend")
    exec(compile(code.replace(placeholder, repr(LIB_PATH)), "INTEGRATION.md", "exec"),
         mod.__dict__)
    return mod
