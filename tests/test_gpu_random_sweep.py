"""Seeded randomised parity sweep of the device API (rss_hash_device / _ws / _reta, and
rss_hash6_device / _ws / _reta) against the
C oracle: random sizes (incl. 0 and ragged tails), power-of-two and arbitrary htable /
nqueues (every modulo and histogram mode), key lengths 16..52, queue widths u8 / u16 /
u32, NULL outputs, accumulation into non-zero counts and 4-byte-misaligned tuples.
Bar: bit-exact (integer work)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# RSS_SWEEP_CASES / RSS_SWEEP_SEED0 widen the sweep for a one-off deep run
CASES = int(os.environ.get("RSS_SWEEP_CASES", "48"))
SEED0 = int(os.environ.get("RSS_SWEEP_SEED0", "0"))


@pytest.fixture(scope="module")
def native():
    from rss_simulator_nvidia_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a gfx950 device")
    return _native


def _config(seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([0, 1, 3, 4, 5, 63, 64, 65, 1023, 4097, int(rng.integers(1, 300000))]))
    if rng.random() < 0.5:
        H = 1 << int(rng.integers(0, 21))
    else:
        H = int(rng.integers(1, 1 << 20))
    Q = int(rng.choice([1, 2, 3, 24, 64, 255, 256, 257, 1000, 9000, 70000, int(rng.integers(1, 2 * H + 2))]))
    key_len = int(rng.choice([16, 40, 52, int(rng.integers(16, 53))]))
    key = [int(x) for x in rng.integers(0, 256, key_len)]
    width = "u8" if Q <= 256 and rng.random() < 0.4 else ("u16" if Q <= 65536 and rng.random() < 0.5 else "u32")
    return dict(rng=rng, n=n, H=H, Q=Q, key=key, width=width,
                want_hash=bool(rng.random() < 0.8), want_queue=bool(rng.random() < 0.8),
                accumulate=bool(rng.random() < 0.3), misaligned=bool(rng.random() < 0.3),
                reta=bool(H <= 1024 and Q <= 65536 and rng.random() < 0.25))


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + CASES))
def test_random_config_matches_oracle(native, oracle_lib, seed):
    c = _config(seed)
    rng, n, H, Q = c["rng"], c["n"], c["H"], c["Q"]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    host = oracle_lib.generate(seed * 7919 + 1, seed, n)
    # tuples at a 16-byte-aligned or a 4-byte-misaligned device address
    off = 1 if c["misaligned"] else 0
    raw = torch.zeros(3 * n + off + 1, dtype=torch.int32, device=dev)
    if n:
        raw[off:off + 3 * n] = torch.from_numpy(host.view(np.int32).reshape(-1)).to(dev)
    tup_ptr = raw.data_ptr() + 4 * off
    qbytes = {"u8": 1, "u16": 2, "u32": 4}[c["width"]]
    qflag = {"u8": native.FLAG_QUEUE_U8, "u16": native.FLAG_QUEUE_U16, "u32": 0}[c["width"]]
    guard = 64
    hbuf = torch.full((n + guard,), -1, dtype=torch.int32, device=dev)
    qbuf = torch.full((n * qbytes + guard,), 0x5A, dtype=torch.uint8, device=dev)
    base = rng.integers(0, 1000, Q).astype(np.int64)
    # count vectors are min(H, Q) long (_native.queue_modulus): no queue >= H exists; with a
    # RETA the caller's Q (entries < Q)
    qn = Q if c["reta"] else native.queue_modulus(H, Q)[1]
    base = base[:qn]
    counts = torch.from_numpy(base if c["accumulate"] else np.full(qn, 77, np.int64)).to(dev)
    flags = qflag | (native.FLAG_ACCUMULATE if c["accumulate"] else 0)
    key = native.prepare_key(c["key"])
    h_ptr = hbuf.data_ptr() if c["want_hash"] else None
    q_ptr = qbuf.data_ptr() if c["want_queue"] else None
    if c["reta"]:
        reta = rng.integers(0, Q, H).astype(np.uint32)
        native.hash_device_reta(key, tup_ptr, n, H, reta, Q, h_ptr, q_ptr, counts.data_ptr(),
                                flags, stream)
    else:
        reta = None
        # half the cases as single-pass counts (rss_hash_device_ws; own generator, so the
        # configurations above stay what they were), the workspace followed by guard words
        single_pass = bool(np.random.default_rng(5000 + seed).random() < 0.5)
        wsn = native.counts_workspace_bytes(H, Q) // 8  # spare, qn sums, tail counter
        assert wsn >= qn + 2 and wsn % (qn + 2) == 0  # spread 8 << k bytes apart
        ws = torch.zeros(wsn + 8, dtype=torch.int64, device=dev)
        ws[wsn:] = -7
        native.hash_device(key, tup_ptr, n, H, Q, h_ptr, q_ptr, counts.data_ptr(), flags, stream,
                           ws.data_ptr() if single_pass else None)
    torch.cuda.synchronize()
    if reta is None:
        wsh = ws.cpu().numpy()
        assert (wsh[:wsn] == 0).all(), "workspace not left zero"
        assert (wsh[wsn:] == -7).all(), "workspace written past its size"

    eh, eq, ec = oracle_lib.run(c["key"], host, H, Q, threads=8)
    if reta is not None:
        eq = reta[eh % H].astype(np.uint32)
        ec = np.bincount(eq, minlength=Q).astype(np.uint64)
    got_h = hbuf.cpu().numpy().view(np.uint32)
    got_q = qbuf.cpu().numpy()
    if c["want_hash"]:
        np.testing.assert_array_equal(got_h[:n], eh)
    assert (got_h[n:] == 0xFFFFFFFF).all(), "hash store past n"
    if c["want_queue"]:
        qdt = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32}[c["width"]]
        np.testing.assert_array_equal(got_q[:n * qbytes].view(qdt), eq.astype(qdt))
        assert (got_q[n * qbytes:] == 0x5A).all(), "queue store past n"
    else:
        assert (got_q == 0x5A).all()
    assert not ec[qn:].any()  # queues >= min(H, Q) never occur
    want = ec[:qn].astype(np.uint64) + (base.astype(np.uint64) if c["accumulate"] else 0)
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), want)


@pytest.mark.parametrize("seed", range(24))
def test_random_key_search_matches_oracle(native, oracle_lib, seed):
    """Key search under random (H, Q, n, key count): packed 8 / 4 keys per entry, pairs,
    partial last groups; every key's counts equal the oracle's."""
    from rss_simulator_nvidia_amd import keysearch
    rng = np.random.default_rng(5000 + seed)
    H = 1 << int(rng.integers(0, 17)) if rng.random() < 0.7 else int(rng.integers(1, 70000))
    Q = int(rng.choice([1, 7, 24, 40, 41, 64, 80, 81, 300, int(rng.integers(1, 2 * H + 2))]))
    n = int(rng.choice([0, 5, 4096, int(rng.integers(1, 200000))]))
    nkeys = int(rng.integers(1, 20))
    keys = keysearch.random_keys(nkeys, seed=seed)
    tuples = oracle_lib.generate(seed + 17, 0, n)
    counts = native.HostContext(0).key_search([native.prepare_key(k) for k in keys], tuples, H, Q)
    qn = min(H, Q)  # rows are min(H, Q) long: queues >= H never occur
    assert counts.shape == (nkeys, qn)
    for k, key in enumerate(keys):
        c = oracle_lib.run(key, tuples, H, Q)[2]
        assert not c[qn:].any()
        np.testing.assert_array_equal(counts[k], c[:qn])


def test_reta_entries_above_u16_are_refused(native):
    """Indirection-table entries travel as u16: a queue id >= 65536 is an error, not a
    silent truncation."""
    from rss_simulator_nvidia_amd.exceptions import DeviceError
    dev = torch.device("cuda:0")
    tup = torch.zeros(3 * 8, dtype=torch.int32, device=dev)
    counts = torch.zeros(70000, dtype=torch.int64, device=dev)
    reta = np.array([1, 65536, 2, 69999], dtype=np.uint32)
    with pytest.raises(DeviceError, match="exceeds 65535"):
        native.hash_device_reta(native.prepare_key(list(range(40))), tup.data_ptr(), 8, 4, reta,
                                70000, None, None, counts.data_ptr(), 0, None)


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + max(24, CASES // 2)))
def test_random_ipv6_config_matches_oracle(native, oracle_lib, seed):
    """IPv6 kernel (36-byte input) under random n / H / Q / field masks / queue widths /
    alignment / indirection tables; the numpy closed form over the oracle's 288 windows
    is the reference."""
    from oracle import oracle as o
    rng = np.random.default_rng(9000 + seed)
    n = int(rng.choice([0, 1, 5, 4097, int(rng.integers(1, 150000))]))
    H = 1 << int(rng.integers(0, 21)) if rng.random() < 0.5 else int(rng.integers(1, 1 << 20))
    Q = int(rng.choice([1, 3, 24, 256, 257, 5000, int(rng.integers(1, 2 * H + 2))]))
    width = "u8" if Q <= 256 and rng.random() < 0.5 else ("u16" if Q <= 65536 and rng.random() < 0.5 else "u32")
    key = [int(x) for x in rng.integers(0, 256, 40)]
    fields = str(rng.choice(["sdfn", "sd", "fn", "s", "sdn"]))
    words = rng.integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    k6 = native.prepare_key6(key, fields)
    full = oracle_lib.windows_n(key, 288)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    off = int(rng.integers(0, 2))
    raw = torch.zeros(9 * n + off + 1, dtype=torch.int32, device=dev)
    if n:
        raw[off:off + 9 * n] = torch.from_numpy(words.view(np.int32).reshape(-1)).to(dev)
    qbytes = {"u8": 1, "u16": 2, "u32": 4}[width]
    qflag = {"u8": native.FLAG_QUEUE_U8, "u16": native.FLAG_QUEUE_U16, "u32": 0}[width]
    hbuf = torch.full((n + 16,), -1, dtype=torch.int32, device=dev)
    qbuf = torch.full((n * qbytes + 16,), 0x5A, dtype=torch.uint8, device=dev)
    use_reta = H <= 1024 and Q <= 65536 and rng.random() < 0.4
    qn = Q if use_reta else native.queue_modulus(H, Q)[1]  # min(H, Q) counts without a table
    counts = torch.full((qn,), 3, dtype=torch.int64, device=dev)
    reta = rng.integers(0, Q, H).astype(np.uint32) if use_reta else None
    if use_reta:
        native.hash6_device_reta(k6, raw.data_ptr() + 4 * off, n, H, reta, Q, hbuf.data_ptr(),
                                 qbuf.data_ptr(), counts.data_ptr(), qflag, stream)
    else:
        # half the cases as single-pass counts (rss_hash6_device_ws; own generator, as the
        # IPv4 sweep), the workspace followed by guard words
        single_pass = bool(np.random.default_rng(6000 + seed).random() < 0.5)
        wsn = native.counts_workspace_bytes(H, Q) // 8
        ws = torch.zeros(wsn + 8, dtype=torch.int64, device=dev)
        ws[wsn:] = -7
        native.hash6_device(k6, raw.data_ptr() + 4 * off, n, H, Q, hbuf.data_ptr(),
                            qbuf.data_ptr(), counts.data_ptr(), qflag, stream,
                            ws.data_ptr() if single_pass else None)
    torch.cuda.synchronize()
    if not use_reta:
        wsh = ws.cpu().numpy()
        assert (wsh[:wsn] == 0).all(), "workspace not left zero"
        assert (wsh[wsn:] == -7).all(), "workspace written past its size"
    if fields == "sdfn":
        want = o.hash_words_np(full, words)
    else:
        # field selection = the concatenated selected fields hashed from key bit 0
        sel = []
        for f, (a, b) in zip("sdfn", [(0, 128), (128, 256), (256, 272), (272, 288)]):
            if f in fields:
                sel.extend(range(a, b))
        w = np.zeros(288, dtype=np.uint32)
        w[sel] = oracle_lib.windows_n(key, len(sel))
        want = o.hash_words_np(w, words)
    np.testing.assert_array_equal(hbuf.cpu().numpy().view(np.uint32)[:n], want)
    assert (hbuf.cpu().numpy()[n:] == -1).all()
    qo, co = o.queue_and_counts(want, H, Q)
    if use_reta:
        qo = reta[want % H]
        co = np.bincount(qo, minlength=Q).astype(np.uint64)
    qdt = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32}[width]
    got_q = qbuf.cpu().numpy()
    np.testing.assert_array_equal(got_q[:n * qbytes].view(qdt), qo.astype(qdt))
    assert (got_q[n * qbytes:] == 0x5A).all()
    assert not np.asarray(co)[qn:].any()
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64), np.asarray(co)[:qn])
