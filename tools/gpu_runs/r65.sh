# full GPU suite, smoke, bench + rocprofv3 stats (tag r01l) after the pooled-block CSV file path,
# e2e IPv4 and IPv6 CSV rates
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r65
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r65/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r65/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r65/smoke.log 2>&1 || exit $?
cat gpurun_out/r65/smoke.log
bash tools/gpu_bench_prof.sh r01l > gpurun_out/r65/bench_prof.log 2>&1 || exit $?
cat gpurun_out/r01l/bench.json
timeout -k 10 600 python tools/e2e_ipv6_bench.py > gpurun_out/r65/e2e6.out 2> gpurun_out/r65/e2e6.err || { tail gpurun_out/r65/e2e6.err; exit 1; }
tail -1 gpurun_out/r65/e2e6.out
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/r65/e2e.out 2> gpurun_out/r65/e2e.err || { tail gpurun_out/r65/e2e.err; exit 1; }
tail -1 gpurun_out/r65/e2e.out
