"""``--htable-size`` / ``--num-queues`` >= 2**32 on the device: before the fix,
ctypes truncated 4294967297 to 1 and every row went to queue 0.  Every ingest path (device
CSV, host CSV, pandas) must now write ``queue_number = hash_result % htable % num_queues``
with the hashes of the reference's own example output, and the device-pointer API must
agree with the oracle on 1M synthetic tuples."""
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

U32 = 2 ** 32
PATHS = {"device": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "1"},
         "host": {"RSS_CSV_FASTPATH": "1", "RSS_CSV_DEVICE": "0"},
         "pandas": {"RSS_CSV_FASTPATH": "0", "RSS_CSV_DEVICE": "1"}}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("H,Q", [(U32 + 1, 24), (U32, 7), (128, U32 + 1), (2 ** 45 + 3, 100003)])
def test_cli_beyond_u32(path, H, Q, golden_dir, tmp_path, monkeypatch):
    from rss_simulator_nvidia_amd.main import main
    for k, v in PATHS[path].items():
        monkeypatch.setenv(k, v)
    out = tmp_path / "o.csv"
    main(["--key-file", os.path.join(golden_dir, "example_input", "hash_key.txt"),
          "--ips-file", os.path.join(golden_dir, "example_input", "ips.csv"),
          "--htable-size", str(H), "--num-queues", str(Q), "--csv", str(out)])
    lines = out.read_text().splitlines()
    header = "src_ip,dst_ip,src_port,dst_port,hash_result,queue_number"
    start = lines.index(header)
    body = pd.read_csv(out, skiprows=start)
    ref_path = os.path.join(golden_dir, "example", "out_h128_q24.csv")
    ref = pd.read_csv(ref_path, skiprows=open(ref_path).read().splitlines().index(header))
    assert (body.hash_result == ref.hash_result).all()
    want_q = [int(h) % H % Q for h in body.hash_result]
    assert list(body.queue_number) == want_q
    vc = pd.Series(want_q).value_counts().sort_index()
    counts = pd.read_csv(out, nrows=start - 1)
    assert list(counts.queue_number) == list(vc.index) and list(counts.counts) == list(vc.values)


@pytest.mark.parametrize("H,Q", [(U32 + 1, 24), (U32 * 3, 1000), (100, U32 + 5)])
def test_device_api_beyond_u32(H, Q, oracle_lib, example_key):
    from rss_simulator_nvidia_amd import _native
    n = 1 << 20
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev).cuda_stream
    h2, q2 = _native.queue_modulus(H, Q)
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(q2, dtype=torch.int64, device=dev)
    _native.generate_device(11, 0, n, tuples.data_ptr(), s)
    _native.hash_device(_native.prepare_key(example_key), tuples.data_ptr(), n, H, Q,
                        hashes.data_ptr(), queues.data_ptr(), counts.data_ptr(), 0, s)
    torch.cuda.synchronize()
    ho, _, _ = oracle_lib.run(example_key, oracle_lib.generate(11, 0, n), 128, 24)
    h = hashes.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(h, ho)
    want = (h.astype(object) % H % Q).astype(np.uint64)
    np.testing.assert_array_equal(queues.cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(counts.cpu().numpy().view(np.uint64),
                                  np.bincount(want.astype(np.int64), minlength=q2))
