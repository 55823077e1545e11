"""The small-batch host path (``rss_hash_host`` with n <= 16384: the kernel reads and
writes the context's mapped pinned staging in place, one stream, one sync) -- what a
reference-style caller hits when it hashes one row per ``Toeplitz.compute_hash`` call
(``simulator.py:80-92``).  Bit-exact to the oracle on every size around the switch-over
to the pipelined path, every output subset, RETA mapping, accumulation, alternating
small / large calls on one context (the staging is re-allocated under the aliases), and
one-tuple calls against the reference's README vectors."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SMALL = 1 << 14


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    return _native


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 64, 1023, 4097, SMALL - 1, SMALL, SMALL + 1,
                               SMALL + 5, 3 * SMALL])
def test_sizes_around_the_switch(native, oracle_lib, example_key, n):
    ctx = native.HostContext(0)
    tup = oracle_lib.generate(77, n, n)
    for H, Q in ((128, 24), (100, 7), (1 << 20, 1000)):
        h, q, c = ctx.hash(native.prepare_key(example_key), tup, H, Q)
        ho, qo, co = oracle_lib.run(example_key, tup, H, Q)
        np.testing.assert_array_equal(h, ho)
        np.testing.assert_array_equal(q, qo)
        np.testing.assert_array_equal(c, co)
    ctx.close()


@pytest.mark.parametrize("want", [(True, False, False), (False, True, False), (False, False, True),
                                  (True, True, False), (False, True, True)])
def test_output_subsets(native, oracle_lib, example_key, want):
    ctx = native.default_context()
    tup = oracle_lib.generate(5, 0, 999)
    h, q, c = ctx.hash(native.prepare_key(example_key), tup, 512, 24, want_hash=want[0],
                       want_queue=want[1], want_counts=want[2])
    ho, qo, co = oracle_lib.run(example_key, tup, 512, 24)
    for got, ref, w in ((h, ho, want[0]), (q, qo, want[1]), (c, co, want[2])):
        if w:
            np.testing.assert_array_equal(got, ref)
        else:
            assert got is None


def test_reta_and_alternating_sizes_on_one_context(native, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import reta
    ctx = native.HostContext(0)
    key = native.prepare_key(example_key)
    table = reta.weights(128, [3, 1, 0, 2])
    for i, n in enumerate([7, 5 << 20, 11, SMALL, 2 * SMALL + 1, 1]):
        tup = oracle_lib.generate(9, i << 24, n)
        ho = oracle_lib.run(example_key, tup, 128, 4)[0]
        h, q, c = ctx.hash(key, tup, 128, 4, reta=table)
        np.testing.assert_array_equal(h, ho)
        want_q = np.asarray(table, dtype=np.uint32)[ho % 128]
        np.testing.assert_array_equal(q, want_q)
        np.testing.assert_array_equal(c, np.bincount(want_q, minlength=4).astype(np.uint64))
    ctx.close()


def test_accumulate_flag_on_the_small_path(native, oracle_lib, example_key):
    import ctypes
    ctx = native.HostContext(0)
    key = native.prepare_key(example_key)
    tup = np.ascontiguousarray(oracle_lib.generate(3, 0, 1000))
    counts = np.full(24, 5, dtype=np.uint64)
    lib = native.load()
    rc = lib.rss_hash_host(ctx._ctx, ctypes.byref(key), tup.ctypes.data, 1000, 128, 24, None,
                           None, counts.ctypes.data, native.FLAG_ACCUMULATE)
    assert rc == 0
    np.testing.assert_array_equal(counts, oracle_lib.run(example_key, tup, 128, 24)[2] + 5)
    ctx.close()


def test_compute_hash_one_row_per_call(native, golden_dir):
    """README.md:111 vector and the MS KAT through the per-call API, many calls in a row."""
    import json
    import os

    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    with open(os.path.join(golden_dir, "ms_kat.json")) as f:
        kat = json.load(f)
    key = [int(x, 16) for x in open(os.path.join(golden_dir, "example_input",
                                                 "hash_key.txt")).read().split(":")]
    tz = Toeplitz(key)
    for _ in range(50):
        assert tz.compute_hash("3.3.3.1", "3.3.3.2", 5201, 5001) == 3151101778
    tz_ms = Toeplitz([int(x, 16) for x in kat["key"].split(":")])
    for v in kat["vectors"]:
        assert tz_ms.compute_hash(v["src_ip"], v["dst_ip"], v["src_port"], v["dst_port"]) == \
            v["hash"]
