# full GPU suite, smoke, bench + rocprofv3 stats (tag r01j), PMC traffic of the current kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r41
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r41/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r41/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r41/smoke.log 2>&1 || exit $?
cat gpurun_out/r41/smoke.log
bash tools/gpu_bench_prof.sh r01j > gpurun_out/r41/bench_prof.log 2>&1 || exit $?
cat gpurun_out/r01j/bench.json
bash tools/pmc_traffic.sh r01j_pmc > gpurun_out/r41/pmc.log 2>&1 || exit $?
python tools/pmc_summarize.py gpurun_out/r01j_pmc gpurun_out/r41/pmc_traffic.json && cat gpurun_out/r41/pmc_traffic.json | head -40
