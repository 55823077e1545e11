"""The INTEGRATION.md ctypes stub on the GPU: ``hash_frame`` over the reference's
example_input reproduces the hash_result / queue_number columns and the counts the
reference itself wrote (tests/golden/example/out_h128_q24.csv), twice on one context."""
import io
import os

import numpy as np
import pytest

from integration_stub import load_stub

pytestmark = pytest.mark.gpu
pd = pytest.importorskip("pandas")


def test_stub_hash_frame_matches_reference_csv(golden_dir, example_key):
    stub = load_stub()
    df = pd.read_csv(os.path.join(golden_dir, "example_input", "ips.csv"))
    with open(os.path.join(golden_dir, "example", "out_h128_q24.csv")) as f:
        text = f.read()
    head, table = text.split("src_ip,", 1)
    ref = pd.read_csv(io.StringIO("src_ip," + table))
    counts = pd.read_csv(io.StringIO(head))
    for _ in range(2):  # the second call reuses the process's context
        h, q, c = stub.hash_frame(bytes(example_key), df, 128, 24)
        np.testing.assert_array_equal(h.astype(np.int64), ref["hash_result"].to_numpy())
        np.testing.assert_array_equal(q.astype(np.int64), ref["queue_number"].to_numpy())
        full = np.zeros(24, dtype=np.int64)
        full[counts["queue_number"].to_numpy()] = counts["counts"].to_numpy()
        np.testing.assert_array_equal(c.astype(np.int64), full)
    assert stub._CTX is not None
