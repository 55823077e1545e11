"""Test-only access to the TEST-HOOKS build of the engine (``librss_toeplitz_hooks.so``:
``csrc/rss_toeplitz.hip`` compiled with ``-DRSS_TEST_HOOKS``, declared in
``csrc/rss_test_hooks.h``).  The product library's hashing path reads no environment, and
the library exports no switches; these tests force the paths a launch takes when scratch memory runs short (u16
bins instead of u8, the 12-bit tables, the scratch column instead of residual lists, the
narrow passes, the static walk, a refused scratch block: alloc_fail), the recount of a
guarded pass and a launch that fails part-way through a host call (fail_launch) through this
build, and read the guarded bins' in-flight margin from it.

``with hooks(recount=1): ...`` points ``_native``'s library handle at the hooks build for the
duration (every ``_native`` entry point then calls it), sets the options and resets them on
exit."""
import contextlib
import ctypes
import os

from rss_simulator_nvidia_amd import _native

HOOKS_PATH = os.path.join(os.path.dirname(os.path.abspath(_native.LIB_PATH)),
                          "librss_toeplitz_hooks.so")
OPTIONS = ("recount", "range8", "small_lut", "prefetch", "balance", "counts_perm", "resid", "wide",
           "guard_sleep", "alloc_fail", "fail_launch")
MARGINS = ("hash16", "wide16", "hash8", "wide8")
_hooks = None


def load_hooks():
    """The hooks build, bound like the product library (loaded once)."""
    global _hooks
    if _hooks is None:
        if not os.path.exists(HOOKS_PATH):
            raise _native.NativeLibraryError(
                "test-hooks build %s not found; build it with `make -C "
                "rss_simulator_nvidia_amd/csrc`" % HOOKS_PATH)
        lib = _native._bind(ctypes.CDLL(HOOKS_PATH))
        lib.rss_test_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.rss_test_set_option.restype = ctypes.c_int
        lib.rss_test_reset_options.argtypes = []
        lib.rss_test_reset_options.restype = None
        lib.rss_test_guard_margin.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        lib.rss_test_guard_margin.restype = ctypes.c_int
        _hooks = lib
    return _hooks


@contextlib.contextmanager
def hooks(**options):
    """Run the body on the hooks build with ``options`` (names: OPTIONS) set."""
    lib = load_hooks()
    with _native._lock:
        saved = _native._lib
        _native._lib = lib
    try:
        lib.rss_test_reset_options()
        for name, value in options.items():
            if lib.rss_test_set_option(name.encode(), int(value)) != 0:
                raise ValueError(lib.rss_last_error().decode())
        yield lib
    finally:
        lib.rss_test_reset_options()
        with _native._lock:
            _native._lib = saved


def guard_margin(reset=True):
    """{kind: the most adds that landed on a guarded bin between the add that took it to half
    range and the guard's subtract} since the last reset (u8 kinds modulo 256)."""
    out = (ctypes.c_uint32 * 4)()
    rc = load_hooks().rss_test_guard_margin(out, 1 if reset else 0)
    if rc != 0:
        raise _native.DeviceError(load_hooks().rss_last_error().decode())
    return dict(zip(MARGINS, list(out)))
