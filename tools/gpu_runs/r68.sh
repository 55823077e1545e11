# final check: full GPU suite (incl. test_gpu_1g.py and the restated CLI helper modules) + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r68
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r68/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r68/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r68/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/r68/smoke.log; exit $rc
