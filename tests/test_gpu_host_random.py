"""Randomised sweep of the host-memory entry points (``rss_hash_host`` / ``rss_hash6_host``
and their ``_reta`` forms) against the C oracle: per seed a batch size anywhere from 0 to 6M
tuples (so every path -- empty, the small-batch path, one chunk, two to many pipeline chunks
with a ragged tail -- and the chunk rule's edges come up), IPv4 or IPv6, a random (H, Q) or an
indirection table, page-locked or pageable tuples and outputs, any subset of the outputs, one
context reused across the seeds (its staging grows and is reused in every order) or two /
three contexts splitting the batch (``MultiHostContext``).  ``RSS_HOST_SWEEP_CASES`` / ``RSS_HOST_SWEEP_SEED0`` widen it."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CASES = int(os.environ.get("RSS_HOST_SWEEP_CASES", "24"))
SEED0 = int(os.environ.get("RSS_HOST_SWEEP_SEED0", "0"))


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


@pytest.fixture(scope="module")
def ctx(native):
    c = native.HostContext(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def multi(native):
    """Several contexts on cuda:0 (rss_hash_host_multi / MultiHostContext.hash6 ranges)."""
    m = {k: native.MultiHostContext([0] * k) for k in (2, 3)}
    yield m
    for c in m.values():
        c.close()


def _size(rng):
    kind = rng.integers(0, 6)
    if kind == 0:
        return int(rng.integers(0, 4))
    if kind == 1:  # around the small-batch switch
        return int(16384 + rng.integers(-3, 4))
    if kind == 2:  # around the first multi-chunk sizes (256K .. 1M + a bit)
        return int(rng.integers(1 << 18, (1 << 20) + 70000))
    if kind == 3:  # around a quarter step of 64K
        return int(4 * 65536 * rng.integers(4, 24) + rng.integers(-5, 6))
    return int(rng.integers(0, 6 << 20))


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + CASES))
def test_random_host_batch_matches_oracle(native, ctx, multi, oracle_lib, example_key, seed):
    rng = np.random.default_rng(0x4057 + seed)
    n = _size(rng)
    ipv6 = bool(rng.integers(0, 2))
    H = int(rng.choice([1, 7, 64, 128, 512, 1 << 16, 1 << 30]))
    Q = int(rng.choice([1, 2, 5, 24, 64, 300, 70000]))
    use_reta = H <= 1024 and rng.integers(0, 3) == 0  # (reta.MAX_ENTRIES)
    if ipv6:
        tup = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
        ho, qo, co = oracle_lib.run_words(example_key, tup, H, Q, threads=16)
    else:
        tup = oracle_lib.generate(seed, 0, n)
        ho, qo, co = oracle_lib.run(example_key, tup, H, Q, threads=16)
    table = None
    if use_reta:
        table = rng.integers(0, Q, H).astype(np.uint32) % min(Q, 65536)
        qo = table[ho % H]
        co = np.bincount(qo, minlength=Q).astype(np.uint64)
    qn = native.queue_modulus(H, Q, use_reta)[1]
    co = co[:qn]
    want_hash, want_queue, want_counts = (bool(b) for b in rng.integers(0, 2, 3))
    pin_in, pin_out = (bool(b) for b in rng.integers(0, 2, 2))
    src = tup
    if pin_in and n:
        src = native.pinned_empty(tup.shape, np.uint32)
        src[:] = tup
    out = None
    if pin_out:
        out = (native.pinned_empty(n, np.uint32) if want_hash else None,
               native.pinned_empty(n, np.uint32) if want_queue else None)
    key = native.prepare_key6(example_key) if ipv6 else native.prepare_key(example_key)
    nctx = int(rng.choice([1, 1, 2, 3]))
    target = ctx if nctx == 1 else multi[nctx]
    call = target.hash6 if ipv6 else target.hash
    h, q, c = call(key, src, H, Q, want_hash=want_hash, want_queue=want_queue,
                   want_counts=want_counts, reta=table, out=out)
    if want_hash:
        np.testing.assert_array_equal(h, ho)
    else:
        assert h is None
    if want_queue:
        np.testing.assert_array_equal(q, qo)
    else:
        assert q is None
    if want_counts:
        np.testing.assert_array_equal(c, co)
        assert int(c.sum()) == n
    else:
        assert c is None
