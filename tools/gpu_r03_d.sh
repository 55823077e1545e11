#!/bin/bash
# GPU box, round 3 (d): wide-histogram tests + the (H, Q) sweep after the issue-all-adds change.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03_d}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_range_hist.py tests/test_gpu_single_pass.py tests/test_gpu_random_sweep.py tests/test_gpu_queues_ge_htable.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
echo "pytest ok"
timeout -k 10 300 python tools/config_sweep_probe.py > $OUT/config_sweep.jsonl 2> $OUT/config_sweep.err
echo "sweep ok"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mqprof -o run -- \
    python3 $R/tools/many_queues_prof.py > $OUT/mqprof.log 2>&1
echo "mqprof ok"
