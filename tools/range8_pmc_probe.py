"""One many-queues mode, 3 launches (tool, not product): python tools/range8_pmc_probe.py Q
full|counts -- 2^28 uniform tuples, H = 2^30, run under rocprofv3 --pmc by
tools/range8_pmc.sh (every kernel of the 3 launches is summed; the input generator is not)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import EXAMPLE_KEY, SEED  # noqa: E402
from rss_simulator_nvidia_amd import _native  # noqa: E402

Q, mode = int(sys.argv[1]), sys.argv[2]
n, H = 1 << 28, 1 << 30
dev = torch.device("cuda:0")
s = torch.cuda.current_stream(dev).cuda_stream
key = _native.prepare_key([int(x, 16) for x in EXAMPLE_KEY.split(":")])
tup = torch.empty(3 * n, dtype=torch.int32, device=dev)
_native.generate_device(SEED, 0, n, tup.data_ptr(), s)
full = mode == "full"
h = torch.empty(n, dtype=torch.int32, device=dev) if full else None
q = torch.empty(n, dtype=torch.int32, device=dev) if full else None
c = torch.zeros(Q, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
for _ in range(3):
    _native.hash_device(key, tup.data_ptr(), n, H, Q, h.data_ptr() if full else None,
                        q.data_ptr() if full else None, c.data_ptr(), 0, s)
torch.cuda.synchronize()
assert int(c.sum()) == n
