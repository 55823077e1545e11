"""``htable`` / ``nqueues`` beyond the C ABI's ``uint32_t``: ctypes would
truncate 4294967297 to 1 silently, so ``_native.queue_modulus`` rewrites such values into
ones that give the same ``hash % htable % nqueues`` (``simulator.py:96-98``) for every
32-bit hash.  Checked here against Python's arbitrary-precision ``%`` -- the reference's
own arithmetic -- on edge and random hashes, and through the CLI (device call replaced by
the oracle, which applies the rewritten arguments exactly as the kernel does)."""
import os

import numpy as np
import pytest

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.main import main

U32 = 2 ** 32
HASHES = [0, 1, 2, 12345, U32 // 2, U32 - 2, U32 - 1] + \
    [int(x) for x in np.random.default_rng(7).integers(0, U32, 2000, dtype=np.uint64)]


@pytest.mark.parametrize("H,Q", [(U32 + 1, 24), (U32, 24), (U32 + 1, 1), (U32 * 5 + 3, 7),
                                 (2 ** 40, U32 - 1), (2 ** 40, 3 * 2 ** 30), (128, U32 + 1),
                                 (U32 - 1, U32), (5, 2 ** 70), (U32 - 1, U32 - 1), (128, 24)])
def test_rewritten_modulus_gives_the_reference_queue(H, Q):
    h2, q2 = _native.queue_modulus(H, Q)
    assert 1 <= h2 <= U32 - 1 and 1 <= q2 <= U32 - 1
    for h in HASHES:
        assert h % h2 % q2 == h % H % Q, (h, H, Q, h2, q2)


def test_both_beyond_u32_is_refused():
    with pytest.raises(ValueError, match="both >= 2"):
        _native.queue_modulus(U32, U32)
    with pytest.raises(ValueError):
        _native.queue_modulus(-1, 5)
    assert _native.queue_modulus(0, 5) == (0, 5)  # passed on: the library refuses it


def test_reta_bounds_only_the_count_length():
    assert _native.queue_modulus(16, U32 + 9, reta=True) == (16, 65536)
    assert _native.queue_modulus(16, 4, reta=True) == (16, 4)


class RecordingContext:
    """Oracle stand-in that records the (htable, nqueues) the kernel would receive."""

    def __init__(self, oracle_lib):
        from test_cli_host import OracleContext
        self.inner = OracleContext(oracle_lib)
        self.seen = []

    def csv_hash_file(self, *a, **k):
        return None

    def csv_hash_text(self, *a, **k):
        return None

    def hash(self, key, tuples, htable, nqueues, **kw):
        htable, nqueues = _native.queue_modulus(htable, nqueues, kw.get("reta") is not None)
        self.seen.append((htable, nqueues))
        return self.inner.hash(key, tuples, htable, nqueues, **kw)


@pytest.mark.parametrize("fast", ["1", "0"])
@pytest.mark.parametrize("H", [U32 + 1, U32, 2 ** 40 + 12345])
def test_cli_htable_beyond_u32(fast, H, golden_dir, tmp_path, capsys, monkeypatch, oracle_lib):
    """--htable-size >= 2**32: queue = hash % num_queues, as the reference computes."""
    import pandas as pd
    ctx = RecordingContext(oracle_lib)
    monkeypatch.setattr(_native, "default_context", lambda: ctx)
    monkeypatch.setenv("RSS_CSV_FASTPATH", fast)
    out = tmp_path / "o.csv"
    main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
          "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", str(H), "--num-queues", "24", "--csv", str(out)])
    assert ctx.seen and all(h < U32 and q == 24 for h, q in ctx.seen)
    text = out.read_text().splitlines()
    start = text.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number")
    body = pd.read_csv(out, skiprows=start)
    assert (body.queue_number == body.hash_result % H % 24).all()
    # the hashes themselves are the example's (htable does not enter the hash)
    ref = pd.read_csv(os.path.join(golden_dir, "example", "out_h128_q24.csv"),
                      skiprows=open(os.path.join(golden_dir, "example", "out_h128_q24.csv"))
                      .read().splitlines().index(text[start]))
    assert (body.hash_result == ref.hash_result).all()
    counts = pd.read_csv(out, nrows=start - 1)
    want = body.queue_number.value_counts().sort_index()
    assert list(counts.queue_number) == list(want.index)
    assert list(counts.counts) == list(want.values)


def test_cli_both_beyond_u32_is_a_usage_error(golden_dir, capsys):
    with pytest.raises(SystemExit) as exc:
        main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
              "--ips-file", "x.csv", "--htable-size", str(U32), "--num-queues", str(U32)])
    assert exc.value.code == 2
    assert "both >= 2**32" in capsys.readouterr().err


@pytest.mark.parametrize("H,Q,want", [(128, 129, (128, 128)), (128, 20000, (128, 128)),
                                      (128, 300000, (128, 128)), (128, 4 * 10 ** 9, (128, 128)),
                                      (128, U32 + 1, (128, 128)), (128, 24, (128, 24)),
                                      (128, 128, (128, 128)), (U32 - 1, U32, (U32 - 1, U32 - 1))])
def test_counts_sized_by_min_of_htable_and_queues(H, Q, want):
    """VERDICT r02 "Fix the Q >= H path": queue = bucket % Q < min(H, Q) (simulator.py:96-98),
    so every count vector is min(H, Q) long -- not 32 GB for --num-queues 4e9."""
    assert _native.queue_modulus(H, Q) == want
    h2, q2 = want
    for h in HASHES[:200]:
        assert h % h2 % q2 == h % H % Q


def test_cli_both_beyond_u32_csv_counts_hashes(golden_dir, tmp_path, monkeypatch, oracle_lib):
    """--csv with htable and num-queues both >= 2**32: queue = hash (the reference's pandas
    arithmetic), counted sparsely on the host (no usage error in CSV mode)."""
    import pandas as pd
    ctx = RecordingContext(oracle_lib)
    monkeypatch.setattr(_native, "default_context", lambda: ctx)
    out = tmp_path / "o.csv"
    main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
          "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", str(U32 + 5), "--num-queues", str(2 ** 40), "--csv", str(out)])
    text = out.read_text().splitlines()
    start = text.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number")
    body = pd.read_csv(out, skiprows=start)
    assert (body.queue_number == body.hash_result).all()
    ref_path = os.path.join(golden_dir, "example", "out_h128_q24.csv")
    ref = pd.read_csv(ref_path, skiprows=open(ref_path).read().splitlines().index(text[start]))
    assert (body.hash_result == ref.hash_result).all()
    counts = pd.read_csv(out, nrows=start - 1)
    want = body.hash_result.value_counts().sort_index()
    assert list(counts.queue_number) == list(want.index)
    assert list(counts.counts) == list(want.values)
