# randomised parity sweep incl. IPv6
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r30
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_sweep.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r30/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r30/pytest.log; exit $rc
