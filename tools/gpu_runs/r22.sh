# Session re-entry check of the committed tree: full pytest -m gpu, smoke(), bench + rocprofv3
# kernel stats (tag r01g), then the work-distribution probe of tools/kbench ("dyn").
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r22
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r22/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r22/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r22/smoke.log 2>&1 || exit $?
cat gpurun_out/r22/smoke.log
bash tools/gpu_bench_prof.sh r01g > gpurun_out/r22/bench_prof.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r22/bench_prof.log
timeout -k 10 300 tools/kbench 268435456 20 dyn > gpurun_out/r22/kbench_dyn.log 2>&1 || exit $?
cat gpurun_out/r22/kbench_dyn.log
