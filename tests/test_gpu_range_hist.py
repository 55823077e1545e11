"""Large queue counts (more than the u32 LDS bins beside the tables hold, DESIGN.md §3 "Many
queues"): the hash pass counts the first range of queues in guarded u16 / u8 LDS bins (a bin
that wraps poisons the pass and a recount replaces it) and writes the queue column (the
caller's, a stream-ordered scratch column, or -- counts only past 161144 queues -- per-wave
residual lists); every further range is histogrammed from that column by guarded wide passes
(or, without scratch memory for them, u32 narrow passes).  Bar: hash / queue / counts
bit-exact to the C oracle on every path -- the product launch and, through the tests'
hooks build (tests/hooks.py), the paths a launch takes without scratch memory, a guarded
pass's bins alone and its recount alone, and real u16 wraps forced by delaying the guard --
across Q up to 10^6, u16 / u32 columns, caller-owned and scratch, RETA tables (whose LDS copy
shrinks the range), misaligned input and unaligned columns, heavy hitters, Zipf traffic,
ragged n and accumulation."""
import numpy as np
import pytest

from hooks import hooks

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# queues counted in the hash pass beside the 2688-byte small tables: u16 bins / u8 bins; u8
# bins per wide pass over the queue column
SPAN16, SPAN8, WIDE8 = 80572, 161144, 163840


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


@pytest.mark.parametrize("H,Q", [(1 << 20, 8193), (1 << 20, 20000), (0xFFFFFFFF, 65536),
                                 (1 << 30, 131072), (1 << 30, 131073), (99991, 50000),
                                 (1 << 30, 8192 * 33)])
@pytest.mark.parametrize("outputs", [True, False])
def test_large_q_equals_oracle(native, oracle_lib, example_key, H, Q, outputs):
    n = (1 << 20) + 7
    host = oracle_lib.generate(21, 0, n)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    h = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
    q = torch.empty(n, dtype=torch.int16 if Q <= 65536 else torch.int32, device=dev) if outputs else None
    c = torch.full((Q,), 5, dtype=torch.int64, device=dev)
    flags = (native.FLAG_QUEUE_U16 if Q <= 65536 else 0) if outputs else 0
    native.hash_device(native.prepare_key(example_key), tup.data_ptr(), n, H, Q,
                       h.data_ptr() if outputs else None, q.data_ptr() if outputs else None,
                       c.data_ptr(), flags, s)
    torch.cuda.synchronize()
    ho, qo, co = oracle_lib.run(example_key, host, H, Q)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)
    if outputs:
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
        qv = q.cpu().numpy()
        qv = qv.view(np.uint16) if qv.dtype == np.int16 else qv.view(np.uint32)
        np.testing.assert_array_equal(qv.astype(np.uint32), qo)


def test_large_q_misaligned_ragged_accumulate(native, oracle_lib, example_key):
    n, H, Q = 300007, 1 << 24, 30000
    host = oracle_lib.generate(22, 0, n)
    flat = host.view(np.int32).reshape(-1)
    buf = torch.zeros(flat.size + 1, dtype=torch.int32, device="cuda:0")
    buf[1:] = torch.from_numpy(flat).to("cuda:0")  # 4-B offset: one tuple per lane
    s = torch.cuda.current_stream().cuda_stream
    c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
    key = native.prepare_key(example_key)
    for _ in range(2):
        native.hash_device(key, buf.data_ptr() + 4, n, H, Q, None, None, c.data_ptr(),
                           native.FLAG_ACCUMULATE, s)
    torch.cuda.synchronize()
    _, _, co = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), 2 * co)


def test_large_q_with_reta(native, oracle_lib, example_key):
    """RETA entries up to 20000 over 1024 buckets: bins share the LDS with the table"""
    n, H, Q = 1 << 19, 1024, 20000
    rng = np.random.default_rng(3)
    reta = rng.integers(0, Q, H).astype(np.uint32)
    host = oracle_lib.generate(23, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    q = torch.empty(n, dtype=torch.int32, device="cuda:0")
    c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
    native.hash_device_reta(native.prepare_key(example_key), tup.data_ptr(), n, H, reta, Q, None,
                            q.data_ptr(), c.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ho, _, _ = oracle_lib.run(example_key, host, 1, 1, want_queue=False)
    want_q = reta[ho % H]
    np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), want_q)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64),
                                  np.bincount(want_q, minlength=Q).astype(np.uint64))


def test_large_q_unaligned_queue_column(native, oracle_lib, example_key):
    """a caller queue column at a 2-byte offset: the range passes read it element-wise"""
    n, H, Q = 200003, 1 << 20, 20000
    host = oracle_lib.generate(24, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    qbuf = torch.zeros(n + 8, dtype=torch.int16, device="cuda:0")
    c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
    native.hash_device(native.prepare_key(example_key), tup.data_ptr(), n, H, Q, None,
                       qbuf.data_ptr() + 2, c.data_ptr(), native.FLAG_QUEUE_U16,
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _, qo, co = oracle_lib.run(example_key, host, H, Q)
    np.testing.assert_array_equal(qbuf[1:n + 1].cpu().numpy().view(np.uint16).astype(np.uint32), qo)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)


@pytest.mark.parametrize("H,Q,outputs", [(1 << 20, 3073, True), (1 << 20, 20000, False),
                                         (0xFFFFFFFF, 65536, True), (1 << 30, 100000, False)])
def test_ipv6_large_q(native, example_key, H, Q, outputs):
    """IPv6 (12 KiB of bins beside its tables, so ranges start at 3073 queues): queue and
    counts equal hash % H % Q of the kernel's own hashes (pinned by the IPv6 KAT tests)"""
    n = (1 << 18) + 3
    rng = np.random.default_rng(Q)
    words = torch.from_numpy(rng.integers(-2**31, 2**31, 9 * n, dtype=np.int64).astype(np.int32)).to("cuda:0")
    key6 = native.prepare_key6(example_key)
    s = torch.cuda.current_stream().cuda_stream
    h = torch.empty(n, dtype=torch.int32, device="cuda:0")
    native.hash6_device(key6, words.data_ptr(), n, 1, 1, h.data_ptr(), None, None, 0, s)
    q = torch.empty(n, dtype=torch.int32, device="cuda:0") if outputs else None
    c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
    native.hash6_device(key6, words.data_ptr(), n, H, Q, None, q.data_ptr() if outputs else None,
                        c.data_ptr(), 0, s)
    torch.cuda.synchronize()
    hv = h.cpu().numpy().view(np.uint32).astype(np.uint64)
    want_q = (hv % np.uint64(H)) % np.uint64(Q)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64),
                                  np.bincount(want_q.astype(np.int64), minlength=Q).astype(np.uint64))
    if outputs:
        np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32).astype(np.uint64), want_q)


@pytest.mark.parametrize("H,Q", [(1 << 20, 20000), (1 << 30, 65536), (1 << 30, 131072),
                                 (1 << 30, 65536 * 3 + 17)])
def test_wide_equals_narrow_passes(native, oracle_lib, example_key, H, Q):
    """The wide passes (guarded u8 / u16 LDS bins + partial-matrix reduce) and the narrow
    passes a launch takes when it gets no memory for their scratch (u32 bins, one pass per
    16384 queues; forced with the hooks build's wide=0) give the oracle's counts on the same
    launch, with and without per-tuple outputs."""
    n = (1 << 22) + 3
    host = oracle_lib.generate(27, 0, n)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    want = oracle_lib.run(example_key, host, H, Q, want_hash=False, want_queue=False)[2]
    key = native.prepare_key(example_key)
    for wide in (1, 0):
        with hooks(wide=wide):
            for outputs in (True, False):
                q = (torch.empty(n, dtype=torch.int16 if Q <= 65536 else torch.int32, device=dev)
                     if outputs else None)
                c = torch.full((Q,), 3, dtype=torch.int64, device=dev)
                native.hash_device(key, tup.data_ptr(), n, H, Q, None,
                                   q.data_ptr() if outputs else None, c.data_ptr(),
                                   (native.FLAG_QUEUE_U16 if Q <= 65536 else 0) if outputs else 0, s)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want,
                                              err_msg="wide=%d outputs=%s" % (wide, outputs))


@pytest.mark.parametrize("Q,lo,hi", [(170000, SPAN8, 170000), (60000, 16384, 60000),
                                     (40000, 0, 16384), (12000, 8192, 12000)])
def test_wide_guard_bit_on_one_hot_queue(native, oracle_lib, example_key, Q, lo, hi):
    """2^25 identical tuples plus 4099 random ones, the identical tuples' queue in [lo, hi):
    every workgroup counts ~2^17 adds into one u16 bin -- of the u16 wide pass after the u8
    hash pass (q >= 161144) or of the hash pass's own u16 range (HIST_RANGE16 on the small
    tables, Q <= 80572; Q = 12000 is a single pass on the 12-bit tables) -- so the guard moves
    2^15 out of it again and again; the counts stay exact, on the product library and on the
    hooks build, which also records the guard's in-flight margin (the most adds that landed
    on the bin between its 0x7FFF add and the guard's subtract; a margin of 2^15 or more is a
    wrap, which poisons the pass and is recounted).  With RSS_MARGIN_LOG set the margins are
    appended there as JSON lines."""
    import json
    import os
    import hooks as hk
    n_same, n_rand = 1 << 25, 4099
    H = 1 << 30
    rnd = oracle_lib.generate(28, 0, n_rand)
    _, q_rnd, _ = oracle_lib.run(example_key, rnd, H, Q)
    pick = int(np.flatnonzero((q_rnd >= lo) & (q_rnd < hi))[0])
    one = rnd[pick:pick + 1]
    host = np.concatenate([np.repeat(one, n_same, axis=0), rnd])
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    _, q1, _ = oracle_lib.run(example_key, one, H, Q)
    want = oracle_lib.run(example_key, rnd, H, Q, want_hash=False, want_queue=False)[2]
    want[int(q1[0])] += n_same
    key = native.prepare_key(example_key)
    for lib in ("product", "hooks"):
        c = torch.zeros(Q, dtype=torch.int64, device=dev)
        with hooks() if lib == "hooks" else _nullcontext():
            if lib == "hooks":
                hk.guard_margin(reset=True)
            native.hash_device(key, tup.data_ptr(), len(host), H, Q, None, None, c.data_ptr(), 0, s)
            torch.cuda.synchronize()
            margin = hk.guard_margin(reset=True) if lib == "hooks" else None
        got = c.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(got, want, err_msg=lib)
        if margin is not None:
            kind = "wide16" if lo >= SPAN8 else "hash16"
            assert margin[kind] > 0, margin  # the guard fired
            log = os.environ.get("RSS_MARGIN_LOG")
            if log:
                with open(log, "a") as f:
                    f.write(json.dumps({"Q": Q, "queue": int(q1[0]), "n_same": n_same,
                                        "guard": kind, "margin": margin}) + "\n")


def _nullcontext():
    import contextlib
    return contextlib.nullcontext()


@pytest.mark.parametrize("H,Q", [(1 << 20, 16385), (0xFFFFFFFF, 65536), (1 << 30, SPAN16),
                                 (1 << 30, SPAN16 + 1), (1 << 30, 131072), (1 << 30, SPAN8 + 65535),
                                 (1 << 30, SPAN8 + 65536), (99991, 50000), (65536, 20000),
                                 (60001, 30011)])
def test_byte_tables_equal_12bit_tables(native, oracle_lib, example_key, H, Q):
    """Many-queues launches hash on the 21 conflict-free 5-bit small tables (kSmallLut: up to
    80572 queues in the hash pass's u16 bins, 161144 in u8 bins); the hooks build's small_lut=0
    keeps the 12-bit tables (16384 queues, then the queue column).  Counts only past 161144 queues: the
    scratch column holds q - 161144 as u16 up to Q = 226679 (QW_U16R), the queues themselves
    (u32) from 226680 on.  Both give the oracle's hashes, queues and counts on uniform and flow-like
    input (one address pair, sequential ports), with outputs and counts only."""
    n = (1 << 21) + 5
    uni = oracle_lib.generate(29, 0, n)
    flow = uni.copy()
    flow[:, 0], flow[:, 1] = uni[0, 0], uni[0, 1]
    flow[:, 2] = (np.arange(n, dtype=np.uint64) % (1 << 32)).astype(np.uint32)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    key = native.prepare_key(example_key)
    u16 = Q <= 65536
    for host in (uni, flow):
        tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
        ho, qo, co = oracle_lib.run(example_key, host, H, Q)
        for lut in (1, 0):
            with hooks(small_lut=lut):
                h = torch.empty(n, dtype=torch.int32, device=dev)
                q = torch.empty(n, dtype=torch.int16 if u16 else torch.int32, device=dev)
                c = torch.full((Q,), 9, dtype=torch.int64, device=dev)
                native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr(), q.data_ptr(),
                                   c.data_ptr(), native.FLAG_QUEUE_U16 if u16 else 0, s)
                c2 = torch.full((Q,), 9, dtype=torch.int64, device=dev)
                native.hash_device(key, tup.data_ptr(), n, H, Q, None, None, c2.data_ptr(), 0, s)
                torch.cuda.synchronize()
            np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
            qv = q.cpu().numpy().view(np.uint16 if u16 else np.uint32).astype(np.uint32)
            np.testing.assert_array_equal(qv, qo)
            np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co)
            np.testing.assert_array_equal(c2.cpu().numpy().view(np.uint64), co)


def test_byte_tables_accumulate_and_queue_column_offsets(native, oracle_lib, example_key):
    """Byte-table launches accumulate (RSS_FLAG_ACCUMULATE); a caller queue column 4 B off
    the 16-B alignment of four u32 queues makes the first pass fall back to the 12-bit tables
    and the one-tuple-per-lane body; a 16-B aligned one keeps the small tables -- same counts."""
    n, H, Q = (1 << 20) + 3, 1 << 26, 90000
    host = oracle_lib.generate(30, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    key = native.prepare_key(example_key)
    _, qo, co = oracle_lib.run(example_key, host, H, Q)
    for off in (0, 4):
        qbuf = torch.zeros(n + 4, dtype=torch.int32, device="cuda:0")
        c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
        for _ in range(2):
            native.hash_device(key, tup.data_ptr(), n, H, Q, None, qbuf.data_ptr() + off,
                               c.data_ptr(), native.FLAG_ACCUMULATE, s)
        torch.cuda.synchronize()
        got_q = qbuf.cpu().numpy().view(np.uint8)[off:off + 4 * n].view(np.uint32)
        np.testing.assert_array_equal(got_q, qo)
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), 2 * co)


def _launch(native, key, tup, n, H, Q, outputs, counts_fill=0, flags=0):
    dev = tup.device
    s = torch.cuda.current_stream(dev).cuda_stream
    h = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
    q = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
    c = torch.full((Q,), counts_fill, dtype=torch.int64, device=dev)
    native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr() if outputs else None,
                       q.data_ptr() if outputs else None, c.data_ptr(), flags, s)
    torch.cuda.synchronize()
    return h, q, c


def _with_opt(name, value, fn):
    """fn() on the hooks build with one option set (name None: the product library)"""
    if name is None:
        return fn()
    with hooks(**{name: value}):
        return fn()


@pytest.mark.parametrize("Q", [SPAN16 + 1, 131072, SPAN8, SPAN8 + 1, SPAN8 + 65535, SPAN8 + 65536,
                               262144, SPAN8 + 65536 + WIDE8 + 1, 10 ** 6,
                               SPAN8 + 9 * WIDE8, SPAN8 + 9 * WIDE8 + 1])
def test_range8_u8_bins_equal_oracle(native, oracle_lib, example_key, Q):
    """Past 80572 queues the small-table pass counts up to 161144 of them in u8 LDS bins
    (HIST_RANGE8: guard at 0x80, moves into a u32 per queue, poison-gated recount); past
    161144 it is the first range of a queue-column launch (counts only: a u16 column of
    q - 161144 up to Q = 226679, u32 beyond), whose passes over the column take 163840
    queues each in u8 bins while more than 65536 are left (one u16 pass for the rest).  On
    uniform input the bins alone (hooks build, recount=2: no gate, no recount), the recount
    alone (recount=1: every guarded pass poisoned), the default and the u16 path (range8=0)
    all give the oracle's hashes, queues and counts, with and without per-tuple outputs.
    Counts only past 161144 queues the hash pass appends the residual queues to per-wave
    lists that the wide passes read one wave per list (default), or writes the scratch column
    (resid=0, the path without memory for the lists); both with the load prefetch and with
    the static walk (prefetch=0)."""
    n, H = (1 << 21) + 5, 1 << 30
    host = oracle_lib.generate(31, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(example_key)
    ho, qo, co = oracle_lib.run(example_key, host, H, Q)
    runs = [("recount", 2), ("recount", 1), (None, None), ("range8", 0), ("resid", 0),
            ("prefetch", 0)]
    for name, value in runs:
        for outputs in (True, False):
            h, q, c = _with_opt(name, value,
                                lambda: _launch(native, key, tup, n, H, Q, outputs, counts_fill=7))
            np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co,
                                          err_msg="%s=%s outputs=%s" % (name, value, outputs))
            if outputs:
                np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
                np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), qo)


@pytest.mark.parametrize("Q", [131072, 200000])
def test_range8_guard_moves(native, oracle_lib, example_key, Q):
    """1024 distinct tuples repeated over 2^26 tuples: every workgroup adds ~256 times into
    each of their u8 bins, a few at a time, so the 0x80 guard moves 128 out of a bin into its
    u32 again and again without a bin ever wrapping.  With the gate and the recount switched
    off (hooks build, recount=2) the counts come from the u8 bins and the guard moves alone
    -- and equal the oracle's; the product launch agrees."""
    n, H, base_n = 1 << 26, 1 << 30, 1024
    base = oracle_lib.generate(32, 0, base_n)
    host = np.tile(base, (n // base_n, 1))
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    _, qb, _ = oracle_lib.run(example_key, base, H, Q)
    want = np.bincount(qb.astype(np.int64), minlength=Q).astype(np.uint64) * np.uint64(n // base_n)
    key = native.prepare_key(example_key)
    for value in (2, None):
        for outputs in (True, False):
            _, q, c = _with_opt("recount" if value else None, value,
                                lambda: _launch(native, key, tup, n, H, Q, outputs))
            np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want,
                                          err_msg="%s outputs=%s" % (value, outputs))
            if outputs:
                got = q[:base_n].cpu().numpy().view(np.uint32)
                np.testing.assert_array_equal(got, qb)


@pytest.mark.parametrize("Q,outputs,lo,hi", [(131072, True, 0, SPAN8), (131072, False, 0, SPAN8),
                                             (200000, True, 0, SPAN8), (200000, False, 0, SPAN8),
                                             (400000, True, SPAN8, SPAN8 + WIDE8),
                                             (400000, False, SPAN8, SPAN8 + WIDE8),
                                             (10 ** 6, True, SPAN8 + 2 * WIDE8, SPAN8 + 3 * WIDE8),
                                             (10 ** 6, False, SPAN8 + 2 * WIDE8, SPAN8 + 3 * WIDE8)])
def test_range8_poisoned_pass_recounts(native, oracle_lib, example_key, Q, outputs, lo, hi):
    """2^22 copies of one tuple whose queue lies in a u8 range -- the hash pass's [0, 161144),
    or (Q = 400000) the first u8 wide pass's [161144, 324984) over the queue column -- plus
    4099 random tuples: every workgroup piles thousands of in-flight adds onto one u8 bin,
    which wraps; the add that wraps it raises the poison word, the reduce skips the pass's
    rows and the recount (from the u32 queue column, or by rehashing for a counts-only hash
    pass) gives the exact counts -- also when accumulating onto the caller's counts.  Q = 10^6:
    the wrapping bin is the third u8 wide pass's (over the u32 queue column, or over the
    residual lists)."""
    n_same, n_rand, H = 1 << 22, 4099, 1 << 30
    rnd = oracle_lib.generate(33, 0, n_rand)
    _, q_rnd, _ = oracle_lib.run(example_key, rnd, H, Q)
    pick = int(np.flatnonzero((q_rnd >= lo) & (q_rnd < hi))[0])
    one = rnd[pick:pick + 1]
    host = np.concatenate([rnd[:2000], np.repeat(one, n_same, axis=0), rnd[2000:]])
    n = len(host)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    want = oracle_lib.run(example_key, rnd, H, Q, want_hash=False, want_queue=False)[2]
    want[int(q_rnd[pick])] += n_same
    key = native.prepare_key(example_key)
    _, q, c = _launch(native, key, tup, n, H, Q, outputs, counts_fill=11,
                      flags=native.FLAG_ACCUMULATE)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want + np.uint64(11))
    if outputs:
        got = q.cpu().numpy().view(np.uint32)
        assert np.all(got[2000:2000 + n_same] == q_rnd[pick])
    # the u8 bins alone are wrong here: proof that the poison gate is what kept them out
    _, _, bad = _with_opt("recount", 2, lambda: _launch(native, key, tup, n, H, Q, outputs))
    assert not np.array_equal(bad.cpu().numpy().view(np.uint64), want)


@pytest.mark.parametrize("Q,outputs", [(131072, True), (131072, False), (400000, False),
                                       (10 ** 6, True), (10 ** 6, False)])
def test_range8_zipf_flows_equal_oracle(native, oracle_lib, example_key, Q, outputs):
    """Skewed traffic: 2^22 tuples drawn Zipf(1.3) from 50000 distinct flows, shuffled -- a
    few flows hold tens of thousands of tuples spread over the batch, most hold a handful.
    Whether or not some workgroup's u8 bin wraps (the recount then takes the launch), the
    counts, and the queues, equal the oracle's."""
    n, H, flows = 1 << 22, 1 << 30, 50000
    base = oracle_lib.generate(34, 0, flows)
    rng = np.random.default_rng(34)
    pick = np.minimum(rng.zipf(1.3, n) - 1, flows - 1)
    host = np.ascontiguousarray(base[pick])
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    _, qb, _ = oracle_lib.run(example_key, base, H, Q)
    want = np.bincount(qb[pick].astype(np.int64), minlength=Q).astype(np.uint64)
    _, q, c = _launch(native, native.prepare_key(example_key), tup, n, H, Q, outputs)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want)
    if outputs:
        np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), qb[pick])


@pytest.mark.parametrize("Q", [12000, 40000, SPAN16])
@pytest.mark.parametrize("outputs", [True, False])
def test_range16_recount_and_bins_alone(native, oracle_lib, example_key, Q, outputs):
    """The hash pass's own u16 bins (HIST_RANGE16: one pass for Q = 12000 on the 12-bit
    tables, Q = 40000 and 80572 on the small tables) carry the guard (a move of 2^15 into a
    u32 per queue) and the poison word: on uniform input the bins and moves alone (hooks
    build, recount=2: no gate, no recount), the recount alone (recount=1: the pass poisoned
    -- from the caller's queue column, or by rehashing for counts only) and the product
    launch all give the oracle's counts, accumulating onto the caller's counts too."""
    n, H = (1 << 21) + 5, 1 << 30
    host = oracle_lib.generate(35, 0, n)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(example_key)
    ho, qo, co = oracle_lib.run(example_key, host, H, Q)
    for name, value in (("recount", 2), ("recount", 1), (None, None)):
        h, q, c = _with_opt(name, value, lambda: _launch(native, key, tup, n, H, Q, outputs,
                                                         counts_fill=5, flags=native.FLAG_ACCUMULATE))
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co + np.uint64(5),
                                      err_msg="%s=%s outputs=%s" % (name, value, outputs))
        if outputs:
            np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
            np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), qo)


def test_range16_recount_with_reta_and_misaligned(native, oracle_lib, example_key):
    """The u16 pass's recount by rehashing with an indirection table (QM_TABLE: the table in
    the recount's LDS beside its u32 bins) and on misaligned tuples (one tuple per lane, the
    12-bit tables), and from a caller's u16 queue column at a 2-byte offset -- each forced
    (recount=1) and as measured, against the oracle."""
    n, H = (1 << 20) + 3, 1024
    rng = np.random.default_rng(36)
    reta = rng.integers(0, 12000, H).astype(np.uint32)
    host = oracle_lib.generate(36, 0, n)
    flat = host.view(np.int32).reshape(-1)
    buf = torch.zeros(flat.size + 1, dtype=torch.int32, device="cuda:0")
    buf[1:] = torch.from_numpy(flat).to("cuda:0")
    tup = torch.from_numpy(flat).to("cuda:0")
    key = native.prepare_key(example_key)
    s = torch.cuda.current_stream().cuda_stream
    ho, _, _ = oracle_lib.run(example_key, host, 1, 1, want_queue=False)
    want_reta = np.bincount(reta[ho % H], minlength=12000).astype(np.uint64)
    Hm, Qm = 1 << 30, 20000
    _, qo, co = oracle_lib.run(example_key, host, Hm, Qm)
    for recount in (1, 0):
        with hooks(recount=recount):
            c = torch.zeros(12000, dtype=torch.int64, device="cuda:0")
            native.hash_device_reta(key, tup.data_ptr(), n, H, reta, 12000, None, None,
                                    c.data_ptr(), 0, s)
            c2 = torch.zeros(Qm, dtype=torch.int64, device="cuda:0")
            native.hash_device(key, buf.data_ptr() + 4, n, Hm, Qm, None, None, c2.data_ptr(), 0, s)
            qbuf = torch.zeros(n + 8, dtype=torch.int16, device="cuda:0")
            c3 = torch.zeros(Qm, dtype=torch.int64, device="cuda:0")
            native.hash_device(key, tup.data_ptr(), n, Hm, Qm, None, qbuf.data_ptr() + 2,
                               c3.data_ptr(), native.FLAG_QUEUE_U16, s)
            torch.cuda.synchronize()
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want_reta)
        np.testing.assert_array_equal(c2.cpu().numpy().view(np.uint64), co)
        np.testing.assert_array_equal(c3.cpu().numpy().view(np.uint64), co)
        np.testing.assert_array_equal(qbuf[1:n + 1].cpu().numpy().view(np.uint16).astype(np.uint32), qo)


@pytest.mark.parametrize("Q,outputs", [(50000, False), (50000, True), (12000, False)])
def test_range16_heavy_hitter(native, oracle_lib, example_key, Q, outputs):
    """2^24 copies of one tuple plus 4099 random ones at Q = 50000 (the small tables' u16
    pass) and 12000 (the 12-bit tables'): every workgroup piles ~65536 adds onto one u16 bin,
    which its guard empties by 2^15 again and again.  The product launch, the recount alone
    and the bins and moves alone give the oracle's counts (accumulating)."""
    n_same, n_rand, H = 1 << 24, 4099, 1 << 30
    rnd = oracle_lib.generate(37, 0, n_rand)
    _, q_rnd, _ = oracle_lib.run(example_key, rnd, H, Q)
    one = rnd[:1]
    host = np.concatenate([rnd[:2000], np.repeat(one, n_same, axis=0), rnd[2000:]])
    n = len(host)
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    want = oracle_lib.run(example_key, rnd, H, Q, want_hash=False, want_queue=False)[2]
    want[int(q_rnd[0])] += n_same
    key = native.prepare_key(example_key)
    for name, value in ((None, None), ("recount", 1), ("recount", 2)):
        _, q, c = _with_opt(name, value, lambda: _launch(native, key, tup, n, H, Q, outputs,
                                                         counts_fill=11, flags=native.FLAG_ACCUMULATE))
        np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), want + np.uint64(11),
                                      err_msg="%s=%s" % (name, value))
        if outputs:
            assert np.all(q.cpu().numpy().view(np.uint32)[2000:2000 + n_same] == q_rnd[0])


def test_guard_margin_readout(native, oracle_lib, example_key):
    """The hooks build records the adds that land on a guarded bin between its half-range add
    and the guard's subtract: after a heavy-hitter u16 launch the hash pass's margin is read
    (and is below the 2^15 that would wrap the field, or the launch's counts were recounted)
    and the read resets it."""
    import hooks as hk
    n_same, H, Q = 1 << 24, 1 << 30, 50000
    rnd = oracle_lib.generate(38, 0, 64)
    host = np.concatenate([np.repeat(rnd[:1], n_same, axis=0), rnd])
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    key = native.prepare_key(example_key)
    with hooks():
        hk.guard_margin(reset=True)
        _, _, c = _launch(native, key, tup, len(host), H, Q, False)
        m = hk.guard_margin(reset=True)
        m2 = hk.guard_margin(reset=False)
    assert int(c.sum()) == len(host)
    print("guard margin", m)
    assert m["hash16"] > 0  # the guard fired (~65536 adds per workgroup on one bin)
    assert all(v == 0 for v in m2.values())


@pytest.mark.parametrize("Q,lo,hi", [(50000, 0, 50000), (12000, 8192, 12000),
                                     (170000, SPAN8, 170000)])
def test_u16_real_wrap_is_caught(native, oracle_lib, example_key, Q, lo, hi):
    """A REAL u16 wrap, forced: with the hooks build's guard_sleep the wave of a guard that
    saw 0x7FFF sleeps (~1 ms) before its subtract while the workgroup's other waves keep
    adding 2^25 copies of one tuple onto the same bin -- the hash pass's u16 bins (small
    tables Q = 50000, 12-bit tables Q = 12000) or the u16 wide pass after the u8 hash pass
    (Q = 170000).  The bin passes 0xFFFF: without the gate and the recount (recount=2) the
    counts come out wrong -- the wrap happened -- and with them (the product's path) they
    equal the oracle's."""
    n_same, n_rand, H = 1 << 25, 4099, 1 << 30
    rnd = oracle_lib.generate(39, 0, n_rand)
    _, q_rnd, _ = oracle_lib.run(example_key, rnd, H, Q)
    pick = int(np.flatnonzero((q_rnd >= lo) & (q_rnd < hi))[0])
    host = np.concatenate([np.repeat(rnd[pick:pick + 1], n_same, axis=0), rnd])
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to("cuda:0")
    want = oracle_lib.run(example_key, rnd, H, Q, want_hash=False, want_queue=False)[2]
    want[int(q_rnd[pick])] += n_same
    key = native.prepare_key(example_key)
    with hooks(guard_sleep=300, recount=2):
        _, _, bad = _launch(native, key, tup, len(host), H, Q, False)
    with hooks(guard_sleep=300):
        _, _, good = _launch(native, key, tup, len(host), H, Q, False)
    assert not np.array_equal(bad.cpu().numpy().view(np.uint64), want), "no wrap was forced"
    np.testing.assert_array_equal(good.cpu().numpy().view(np.uint64), want)


# the hooks build's alloc_fail bits (AllocKind, csrc/rss_toeplitz.hip): which scratch blocks
# a launch is refused
AK_ROWS, AK_WIDE, AK_COLUMN, AK_LISTS = 1, 2, 4, 8


@pytest.mark.parametrize("Q,outputs,fail", [
    (50000, False, AK_ROWS),                 # the single u16 pass: no rows -> atomics
    (50000, True, AK_ROWS),
    (120000, False, AK_ROWS),                # the single u8 pass and the first range: atomics
    (300000, False, AK_LISTS),               # no residual lists -> the scratch column
    (300000, False, AK_LISTS | AK_COLUMN),   # ... and no column -> atomics
    (300000, False, AK_WIDE),                # no wide scratch -> 9 narrow passes
    (300000, True, AK_WIDE),
    (1000000, False, AK_WIDE),               # 52 narrow u32 passes > 32 -> atomics
    (1000000, True, AK_WIDE),
    (1000000, True, AK_ROWS | AK_WIDE | AK_COLUMN | AK_LISTS),
])
def test_scratch_allocation_failures_fall_back(native, oracle_lib, example_key, Q, outputs, fail):
    """A launch refused a scratch block (hooks alloc_fail) still succeeds with the oracle's
    counts, accumulated onto the caller's (the counts are untouched until the path that runs
    is chosen): the u16 / u8 rows, the residual lists, the scratch column and the wide
    passes' scratch each have a fallback, down to one global atomic per tuple."""
    n, H = (1 << 20) + 5, 1 << 30
    host = oracle_lib.generate(41, 0, n)
    dev = torch.device("cuda:0")
    tup = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    h = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
    q = torch.empty(n, dtype=torch.int32, device=dev) if outputs else None
    base = np.arange(Q, dtype=np.int64) % 7
    c = torch.from_numpy(base).to(dev)
    with hooks(alloc_fail=fail):
        native.hash_device(native.prepare_key(example_key), tup.data_ptr(), n, H, Q,
                           h.data_ptr() if outputs else None, q.data_ptr() if outputs else None,
                           c.data_ptr(), native.FLAG_ACCUMULATE,
                           torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
    ho, qo, co = oracle_lib.run(example_key, host, H, Q, threads=8)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64), co + base.astype(np.uint64))
    if outputs:
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint32), ho)
        np.testing.assert_array_equal(q.cpu().numpy().view(np.uint32), qo)


@pytest.mark.parametrize("Q,fail", [(100000, AK_WIDE), (1000000, AK_WIDE), (100000, AK_COLUMN)])
def test_ipv6_scratch_allocation_failures_fall_back(native, example_key, Q, fail):
    """IPv6 many queues without wide scratch (narrow passes, or atomics past 32 u32 passes)
    or without a scratch column: counts equal hash % H % Q of the kernel's own hashes."""
    n, H = (1 << 18) + 3, 1 << 30
    rng = np.random.default_rng(Q + fail)
    words = torch.from_numpy(rng.integers(-2**31, 2**31, 9 * n, dtype=np.int64).astype(np.int32)).to("cuda:0")
    key6 = native.prepare_key6(example_key)
    s = torch.cuda.current_stream().cuda_stream
    h = torch.empty(n, dtype=torch.int32, device="cuda:0")
    native.hash6_device(key6, words.data_ptr(), n, 1, 1, h.data_ptr(), None, None, 0, s)
    c = torch.zeros(Q, dtype=torch.int64, device="cuda:0")
    with hooks(alloc_fail=fail):
        native.hash6_device(key6, words.data_ptr(), n, H, Q, None, None, c.data_ptr(), 0, s)
        torch.cuda.synchronize()
    hv = h.cpu().numpy().view(np.uint32).astype(np.uint64)
    want_q = (hv % np.uint64(H)) % np.uint64(Q)
    np.testing.assert_array_equal(c.cpu().numpy().view(np.uint64),
                                  np.bincount(want_q.astype(np.int64), minlength=Q).astype(np.uint64))
