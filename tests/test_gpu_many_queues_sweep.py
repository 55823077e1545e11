"""Seeded randomised sweep of the many-queues paths (more than 8192 queues) on the product
library AND on the tests' hooks build with random path options: u8 bins off (range8=0), the
12-bit tables (small_lut=0), the scratch column instead of residual lists (resid=0), narrow
instead of wide passes (wide=0), the load prefetch forced on / off, the static walk
(balance=0), refused scratch allocations (alloc_fail), every guarded pass recounted (recount=1) or read from its bins and moves alone
(recount=2) -- the alternative paths a launch takes when it gets no scratch memory, and the
two halves of a guarded pass.  Random H (power of two or not, >= Q or not), Q from 8193 to
~1.2M, n up to 2^20 + ragged tails, outputs or counts only, u16 / u32 queues, accumulation,
misaligned tuples.  Bar: bit-exact against the C oracle on every path."""
import os

import numpy as np
import pytest

from hooks import hooks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

OPTS = ("range8", "small_lut", "resid", "wide", "balance")
# RSS_MQ_SWEEP_CASES / RSS_MQ_SWEEP_SEED0 widen the sweep for a one-off deep run
CASES = int(os.environ.get("RSS_MQ_SWEEP_CASES", "64"))
SEED0 = int(os.environ.get("RSS_MQ_SWEEP_SEED0", "0"))


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


def _config(seed):
    rng = np.random.default_rng(7000 + seed)
    Q = int(rng.choice([8193, 16385, 65536, 80572, 80573, 161144, 161145, 226680,
                        int(rng.integers(8193, 1_200_000))]))
    if rng.random() < 0.3:
        H = Q if rng.random() < 0.5 else int(rng.integers(Q // 2 + 1, Q + 1))  # Q >= H
    elif rng.random() < 0.5:
        H = 1 << int(rng.integers(18, 31))
    else:
        H = int(rng.integers(Q + 1, 1 << 31))
    n = int(rng.choice([4099, (1 << 20) + int(rng.integers(0, 4)), int(rng.integers(1, 1 << 20))]))
    opts = {k: 0 for k in OPTS if rng.random() < 0.3}
    r = rng.random()
    if r < 0.2:
        opts["recount"] = 1
    elif r < 0.35:
        opts["recount"] = 2  # uniform input: no bin wraps, so the bins and moves alone are exact
    if rng.random() < 0.3:
        opts["prefetch"] = int(rng.integers(0, 2))
    if rng.random() < 0.2:  # refused scratch blocks (AllocKind bits): the fallbacks down to atomics
        opts["alloc_fail"] = int(rng.integers(1, 16))
    return dict(rng=rng, n=n, H=H, Q=Q, opts=opts, hooks=bool(opts) or rng.random() < 0.5,
                outputs=bool(rng.random() < 0.5), accumulate=bool(rng.random() < 0.3),
                misaligned=bool(rng.random() < 0.2), u16=bool(rng.random() < 0.5))


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + CASES))
def test_many_queues_paths_match_oracle(native, oracle_lib, example_key, seed):
    c = _config(seed)
    rng, n, H, Q = c["rng"], c["n"], c["H"], c["Q"]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    host = oracle_lib.generate(seed * 104729 + 3, seed, n)
    off = 1 if c["misaligned"] else 0
    raw = torch.zeros(3 * n + off, dtype=torch.int32, device=dev)
    raw[off:] = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    qn = native.queue_modulus(H, Q)[1]
    u16 = c["u16"] and qn <= 65536
    h = torch.empty(n, dtype=torch.int32, device=dev) if c["outputs"] else None
    q = (torch.empty(n, dtype=torch.int16 if u16 else torch.int32, device=dev)
         if c["outputs"] else None)
    base = rng.integers(0, 1000, qn).astype(np.int64)
    counts = torch.from_numpy(base if c["accumulate"] else np.full(qn, 5, np.int64)).to(dev)
    flags = ((native.FLAG_QUEUE_U16 if u16 else 0) if c["outputs"] else 0) | \
        (native.FLAG_ACCUMULATE if c["accumulate"] else 0)
    key = native.prepare_key(example_key)

    def launch():
        native.hash_device(key, raw.data_ptr() + 4 * off, n, H, Q,
                           h.data_ptr() if h is not None else None,
                           q.data_ptr() if q is not None else None, counts.data_ptr(), flags, s)
        torch.cuda.synchronize()

    if c["hooks"]:
        with hooks(**c["opts"]):
            launch()
    else:
        launch()
    eh, eq, ec = oracle_lib.run(example_key, host, H, Q, threads=8)
    want = ec[:qn].astype(np.uint64) + (base.astype(np.uint64) if c["accumulate"] else 0)
    msg = "H=%d Q=%d n=%d opts=%s" % (H, Q, n, c["opts"])
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), want, err_msg=msg)
    if c["outputs"]:
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), eh, err_msg=msg)
        got_q = q.cpu().numpy().view(np.uint16 if u16 else np.uint32).astype(np.uint32)
        np.testing.assert_array_equal(got_q, eq, err_msg=msg)
