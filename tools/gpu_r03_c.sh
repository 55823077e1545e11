#!/bin/bash
# GPU box, round 3 (c): the tests that changed with the min(H, Q) count contract and the
# wide histogram, the (H, Q) sweep and the single-pass variant A/B (incl. counts only).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03_c}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_keysearch.py tests/test_gpu_parity.py tests/test_gpu_fields_ipv6.py \
    tests/test_gpu_random_sweep.py tests/test_gpu_range_hist.py tests/test_gpu_single_pass.py \
    > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 300 python tools/config_sweep_probe.py > $OUT/config_sweep.jsonl 2> $OUT/config_sweep.err
echo "sweep ok"
timeout -k 10 200 python tools/ws_order_ab.py 6 > $OUT/ab.json 2> $OUT/ab.err
echo "ab ok"
