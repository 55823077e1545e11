# randomised parity sweep (device API + key search) and the RETA u16 range check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r29
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_sweep.py tests/test_gpu_reta.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r29/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r29/pytest.log; exit $rc
