# nine 11/10-bit tables + QM_FAST8 in the product kernel: full GPU suite, bench, kbench side by side
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r44
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r44/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r44/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r44/bench.json 2> gpurun_out/r44/bench.err || { tail gpurun_out/r44/bench.err; exit 1; }
cat gpurun_out/r44/bench.json
timeout -k 10 300 tools/kbench 268435456 20 T9 > gpurun_out/r44/kbench_t9.log 2>&1 || exit $?
cat gpurun_out/r44/kbench_t9.log
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r44/kbench_policy.log 2>&1 || exit $?
tail -3 gpurun_out/r44/kbench_policy.log
