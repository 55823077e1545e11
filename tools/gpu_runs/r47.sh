# QM_FAST8 (24-bit queue step for H <= 256): full GPU suite + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r47
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r47/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r47/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r47/smoke.log 2>&1 || exit $?
cat gpurun_out/r47/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r47/bench.json 2> gpurun_out/r47/bench.err || { tail gpurun_out/r47/bench.err; exit 1; }
cat gpurun_out/r47/bench.json
