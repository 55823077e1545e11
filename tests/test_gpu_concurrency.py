"""Reentrancy of the reference-compatible per-call API, and the multi-GPU option of it.

The reference's ``Toeplitz.compute_hash`` copies its key on every call
(``rss_simulator/toeplitz.py:59``), so a caller may run it from many threads (a
ThreadPoolExecutor over rows, to escape its per-tuple cost).  Here every ``Toeplitz`` /
``Simulator`` shares one process-wide ``rss_ctx`` whose pinned staging, streams and
scratch are re-used and re-allocated (``ctx_reserve``) from call to call; the library
serialises calls on one context (``struct rss_ctx``'s lock).  These tests drive that
context from 8 threads at once -- single tuples (the mapped small-batch path), 1K, 64K
and 5M tuples (past ``kSmallBatch``: the pipelined path, and staging growth while other
threads wait), queue counts that grow the counts buffers, ``Simulator.calc_hash`` and the
CSV image path -- and check every result against the C oracle.

``devices=`` (``Simulator`` / ``Toeplitz.compute_queues``) splits one batch over several
contexts (``rss_hash_host_multi``); on the one-GPU box the contexts share ``cuda:0``.
Replaces ``rss_simulator/simulator.py:74-98`` at several GPUs' PCIe links.
"""
import concurrent.futures as cf

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

THREADS = 8


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    return _native


def _dotted(u):
    u = np.asarray(u, dtype=np.uint64)
    return [("%d.%d.%d.%d" % (x >> 24, (x >> 16) & 255, (x >> 8) & 255, x & 255))
            for x in u.tolist()]


def _frame(tup):
    return pd.DataFrame({"src_ip": _dotted(tup[:, 0]), "dst_ip": _dotted(tup[:, 1]),
                         "src_port": (tup[:, 2] >> 16).astype(np.int64),
                         "dst_port": (tup[:, 2] & 0xFFFF).astype(np.int64)})


def _assert_counts(c, want):
    """Counts are min(H, Q) long (queue_modulus): the oracle's Q-long vector is zero past it."""
    np.testing.assert_array_equal(c, want[:len(c)])
    assert not want[len(c):].any()


def _jobs(oracle_lib, key):
    """(kind, args, expected) work items, expected results computed up front (serially)."""
    jobs = []
    rng = np.random.default_rng(6)
    for i in range(64):  # single tuples: Toeplitz.compute_hash
        t = oracle_lib.generate(100 + i, 0, 1)
        jobs.append(("one", t, int(oracle_lib.run(key, t, 1, 1)[0][0])))
    for i, (n, H, Q) in enumerate([(1000, 128, 24), (1 << 16, 512, 1000), (5 << 20, 128, 24),
                                   (1000, 1 << 20, 70000), (1 << 16, 100, 7), (3000, 64, 64),
                                   (5 << 20, 4096, 9000), (17, 128, 24)] * 2):
        t = oracle_lib.generate(200 + i, i << 24, n)
        jobs.append(("queues", (t, H, Q), oracle_lib.run(key, t, H, Q)))
    for i in range(6):  # Simulator.calc_hash on a DataFrame
        n = int(rng.integers(1, 20000))
        t = oracle_lib.generate(300 + i, 0, n).view(np.uint32).reshape(-1, 3)
        jobs.append(("sim", t, oracle_lib.run(key, t, 128, 24)))
    order = rng.permutation(len(jobs))
    return [jobs[i] for i in order]


def _run_job(job, key, tz):
    from rss_simulator_nvidia_amd.simulator import Simulator
    kind, args, want = job
    if kind == "one":
        t = np.asarray(args).view(np.uint32).reshape(-1)
        sip, dip, ports = int(t[0]), int(t[1]), int(t[2])
        got = tz.compute_hash(_dotted([sip])[0], _dotted([dip])[0], ports >> 16, ports & 0xFFFF)
        assert got == want
    elif kind == "queues":
        t, H, Q = args
        h, q, c = tz.compute_queues(t, H, Q)
        np.testing.assert_array_equal(h, want[0])
        np.testing.assert_array_equal(q, want[1])
        _assert_counts(c, want[2])
    else:
        sim = Simulator(key, 128, 24)
        sim.load_frame(_frame(args))
        sim.calc_hash()
        sim.calc_queue_number()
        df = sim.data_frame
        np.testing.assert_array_equal(df["hash_result"].to_numpy(), want[0].astype(np.int64))
        np.testing.assert_array_equal(df["queue_number"].to_numpy(), want[1].astype(np.int64))
        np.testing.assert_array_equal(sim.queue_counts, want[2])
    return kind


def test_eight_threads_on_the_default_context(native, oracle_lib, example_key):
    """The reference API (one shared default context) from 8 threads, vs the oracle."""
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    jobs = _jobs(oracle_lib, example_key)
    tz = Toeplitz(example_key)
    with cf.ThreadPoolExecutor(THREADS) as pool:
        done = list(pool.map(lambda j: _run_job(j, example_key, tz), jobs))
    assert sorted(set(done)) == ["one", "queues", "sim"]


def test_eight_threads_grow_a_fresh_context(native, oracle_lib, example_key):
    """A fresh context, so the staging and counts buffers are allocated and grown
    (ctx_reserve frees and re-allocates them) while the other threads' calls queue."""
    ctx = native.HostContext(0)
    key = native.prepare_key(example_key)
    sizes = [(1, 128, 24), (1 << 14, 128, 24), ((1 << 14) + 1, 512, 1000), (1 << 16, 4096, 9000),
             (5 << 20, 128, 24), (1000, 1 << 20, 70000), (3 << 20, 100, 7), (7, 64, 64)]
    work = []
    for i, (n, H, Q) in enumerate(sizes * 3):
        t = oracle_lib.generate(400 + i, 0, n)
        work.append((t, H, Q, oracle_lib.run(example_key, t, H, Q)))

    def one(item):
        t, H, Q, want = item
        h, q, c = ctx.hash(key, t, H, Q)
        np.testing.assert_array_equal(h, want[0])
        np.testing.assert_array_equal(q, want[1])
        _assert_counts(c, want[2])
        return len(t)

    with cf.ThreadPoolExecutor(THREADS) as pool:
        assert sum(pool.map(one, work)) == sum(len(w[0]) for w in work)
    ctx.close()


def test_per_call_time_unchanged_by_the_lock(native, example_key):
    """One-tuple calls stay in the tens of microseconds with the context's lock taken."""
    import time

    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    tz = Toeplitz(example_key)
    for _ in range(50):
        tz.compute_hash("3.3.3.1", "3.3.3.2", 5201, 5001)
    reps = 2000
    t0 = time.perf_counter()
    for _ in range(reps):
        assert tz.compute_hash("3.3.3.1", "3.3.3.2", 5201, 5001) == 3151101778
    per_call_us = (time.perf_counter() - t0) / reps * 1e6
    print("per-call compute_hash: %.1f us" % per_call_us)
    assert per_call_us < 200


def test_csv_text_images_from_many_threads(native, oracle_lib, example_key):
    """rss_csv_hash_text leaves its file image in context-owned memory: concurrent callers
    of one context each get their own image (HostContext holds the context across the call
    and the copy)."""
    ctx = native.HostContext(0)
    key = native.prepare_key(example_key)
    texts = []
    for i, n in enumerate([10, 3000, 50000, 1, 777, 20000]):
        t = oracle_lib.generate(500 + i, 0, n).view(np.uint32).reshape(-1, 3)
        df = _frame(t)
        texts.append(df.to_csv(index=False).encode())
    want = [ctx.csv_hash_text(key, x, 128, 24) for x in texts]  # serial
    for img, counts, n in want:  # and the serial images are the oracle's tables
        assert img is not None and n > 0
    first = want[1][0].tobytes().decode().splitlines()
    start = first.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number")
    t = oracle_lib.generate(501, 0, 3000)
    assert [int(r.split(",")[4]) for r in first[start + 1:]] == \
        oracle_lib.run(example_key, t, 128, 24)[0].tolist()

    def one(i):
        img, counts, n = ctx.csv_hash_text(key, texts[i % len(texts)], 128, 24)
        w = want[i % len(texts)]
        assert n == w[2]
        np.testing.assert_array_equal(counts, w[1])
        assert img.tobytes() == w[0].tobytes()
        return n

    with cf.ThreadPoolExecutor(THREADS) as pool:
        list(pool.map(one, range(48)))
    ctx.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_simulator_devices_option(native, oracle_lib, example_key, devices):
    """Simulator(devices=...) splits calc_hash over one context per entry: same table and
    counts as the oracle (and so as the one-GPU default)."""
    from rss_simulator_nvidia_amd.simulator import Simulator
    t = oracle_lib.generate(600, 0, 30001).view(np.uint32).reshape(-1, 3)
    sim = Simulator(example_key, 128, 24, devices=devices)
    sim.load_frame(_frame(t))
    sim.calc_hash()
    sim.calc_queue_number()
    h, q, c = oracle_lib.run(example_key, t, 128, 24)
    np.testing.assert_array_equal(sim.data_frame["hash_result"].to_numpy(), h.astype(np.int64))
    np.testing.assert_array_equal(sim.data_frame["queue_number"].to_numpy(), q.astype(np.int64))
    np.testing.assert_array_equal(sim.queue_counts, c)
    assert sim.queue_count_rows() == [(int(i), int(c[i])) for i in np.flatnonzero(c)]


@pytest.mark.parametrize("n", [0, 1, 2, 5 << 20])
def test_compute_queues_devices_option(native, oracle_lib, example_key, n):
    """Toeplitz.compute_queues(devices=[0, 0]) on sizes around the split, with a RETA too."""
    from rss_simulator_nvidia_amd import reta
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    tz = Toeplitz(example_key)
    t = oracle_lib.generate(700, 0, n) if n else np.zeros((0, 3), dtype=np.uint32)
    h, q, c = tz.compute_queues(t, 128, 24, devices=[0, 0])
    ho, qo, co = oracle_lib.run(example_key, t, 128, 24)
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(c, co)
    table = reta.weights(128, [3, 1, 0, 2])
    h, q, c = tz.compute_queues(t, 128, 4, reta=table, devices=[0, 0, 0])
    want_q = np.asarray(table, dtype=np.uint32)[ho % 128]
    np.testing.assert_array_equal(h, ho)
    np.testing.assert_array_equal(q, want_q)
    np.testing.assert_array_equal(c, np.bincount(want_q, minlength=4).astype(np.uint64))


def test_compute_queues6_devices_option(native, oracle_lib, example_key):
    """IPv6 batches split over [0, 0]: equal to one context, which the oracle pins on a
    sample (the full batch is checked against the one-context result)."""
    from oracle import oracle as o
    from rss_simulator_nvidia_amd.toeplitz import Toeplitz
    tz = Toeplitz(example_key)
    rng = np.random.default_rng(8)
    words = rng.integers(0, 2**32, size=(100003, 9), dtype=np.uint64).astype(np.uint32)
    h1, q1, c1 = tz.compute_queues6(words, 512, 100)
    h2, q2, c2 = tz.compute_queues6(words, 512, 100, devices=[0, 0])
    np.testing.assert_array_equal(h2, h1)
    np.testing.assert_array_equal(q2, q1)
    np.testing.assert_array_equal(c2, c1)
    for i in rng.integers(0, len(words), size=64):
        assert int(h2[i]) == oracle_lib.hash_bytes(example_key, o.words_to_bytes(words[i]))
    np.testing.assert_array_equal(q2, h2 % 512 % 100)
    np.testing.assert_array_equal(c2, np.bincount(q2, minlength=100).astype(np.uint64))


def test_every_context_entry_point_from_threads(native, oracle_lib, example_key, tmp_path):
    """Every entry point that takes a context, interleaved from 8 threads on ONE context:
    rss_hash_host, rss_hash6_host, rss_key_search_host, rss_csv_hash_text and
    rss_csv_hash_file.  Each result equals the same call made alone (and the IPv4 / key-search
    ones the oracle; the IPv6 ones the oracle on a sample)."""
    from oracle import oracle as o
    ctx = native.HostContext(0)
    key = native.prepare_key(example_key)
    key6 = native.prepare_key6(example_key)
    rng = np.random.default_rng(61)
    t4 = oracle_lib.generate(800, 0, 300000)
    w6 = rng.integers(0, 2**32, size=(70001, 9), dtype=np.uint64).astype(np.uint32)
    keys = [[int(b) for b in rng.permutation(256)[:40]] for _ in range(5)]
    ks_tuples = oracle_lib.generate(801, 0, 50000)
    text = _frame(oracle_lib.generate(802, 0, 20000)).to_csv(index=False).encode()
    src = tmp_path / "in.csv"
    src.write_bytes(text)

    want4 = oracle_lib.run(example_key, t4, 512, 24)
    want6 = ctx.hash6(key6, w6, 128, 24)
    for i in rng.integers(0, len(w6), size=32):
        assert int(want6[0][i]) == oracle_lib.hash_bytes(example_key, o.words_to_bytes(w6[i]))
    want_ks = np.stack([oracle_lib.run(k, ks_tuples, 128, 24, want_hash=False,
                                       want_queue=False)[2] for k in keys])
    img, want_txt_counts, _ = ctx.csv_hash_text(key, text, 128, 24)
    want_txt = img.tobytes()

    def one(i):
        kind = i % 5
        if kind == 0:
            h, q, c = ctx.hash(key, t4, 512, 24)
            np.testing.assert_array_equal(h, want4[0])
            np.testing.assert_array_equal(q, want4[1])
            np.testing.assert_array_equal(c, want4[2])
        elif kind == 1:
            h, q, c = ctx.hash6(key6, w6, 128, 24)
            for got, ref in zip((h, q, c), want6):
                np.testing.assert_array_equal(got, ref)
        elif kind == 2:
            got = ctx.key_search([native.prepare_key(k) for k in keys], ks_tuples, 128, 24)
            np.testing.assert_array_equal(got, want_ks)
        elif kind == 3:
            img, c, _ = ctx.csv_hash_text(key, text, 128, 24)
            assert img.tobytes() == want_txt
            np.testing.assert_array_equal(c, want_txt_counts)
        else:
            out = tmp_path / ("out%d.csv" % i)
            c, n = ctx.csv_hash_file(key, str(src), str(out), 128, 24)
            assert n == 20000 and out.read_bytes() == want_txt
            np.testing.assert_array_equal(c, want_txt_counts)
        return kind

    with cf.ThreadPoolExecutor(THREADS) as pool:
        assert sorted(set(pool.map(one, range(40)))) == [0, 1, 2, 3, 4]
    ctx.close()


def test_multi_context_batches_sharing_contexts_from_threads(native, oracle_lib, example_key):
    """rss_hash_host_multi from 8 threads over two context lists that share their contexts
    in opposite orders ([a, b] and [b, a]): each worker holds one context's lock at a time,
    so the calls interleave without deadlock and every batch equals the oracle."""
    a, b = native.HostContext(0), native.HostContext(0)

    def multi(ctxs):
        m = object.__new__(native.MultiHostContext)
        m.contexts, m._lib = ctxs, native.load()
        return m

    ab, ba = multi([a, b]), multi([b, a])
    key = native.prepare_key(example_key)
    batches = [oracle_lib.generate(900 + i, 0, n) for i, n in enumerate([3, 40000, 1 << 20, 77777])]
    want = [oracle_lib.run(example_key, t, 128, 24) for t in batches]

    def one(i):
        m = ab if i % 2 else ba
        h, q, c = m.hash(key, batches[i % 4], 128, 24)
        for got, ref in zip((h, q, c), want[i % 4]):
            np.testing.assert_array_equal(got, ref)
        return i

    with cf.ThreadPoolExecutor(THREADS) as pool:
        assert sorted(pool.map(one, range(32))) == list(range(32))
    a.close()
    b.close()
