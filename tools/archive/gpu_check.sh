#!/bin/bash
# GPU box: the changed paths' GPU tests (TESTS, 2nd argument), the single-pass variant A/B and one bench
# line.  Every step has its own time limit; the first failure ends the script.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03_check}
TESTS=${2:-"tests/test_gpu_single_pass.py tests/test_gpu_queues_ge_htable.py tests/test_gpu_bench_launch.py tests/test_gpu_modulus.py tests/test_gpu_pipeline.py tests/test_gpu_placement.py tests/test_gpu_rccl.py"}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1
echo "pytest ok"
for p in 1 2; do
    timeout -k 10 120 python tools/ws_order_ab.py 6 > $OUT/ab_$p.json 2> $OUT/ab_$p.err
done
echo "ab ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"
