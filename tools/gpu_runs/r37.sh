# full GPU suite, smoke, bench + rocprofv3 stats (tag r01i) after the multi-context host API, RETA range check and bench timing changes
# smoke, bench + rocprofv3 stats (tag r01i), key search and IPv6 throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r37
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r37/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r37/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r37/smoke.log 2>&1 || exit $?
cat gpurun_out/r37/smoke.log
bash tools/gpu_bench_prof.sh r01i > gpurun_out/r37/bench_prof.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r37/bench_prof.log
