# IPv6 indirection tables (device, host, CLI) + the random sweep incl. IPv6 RETAs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r39
timeout -k 10 600 python -u -m pytest tests/test_gpu_reta.py tests/test_gpu_random_sweep.py tests/test_gpu_fields_ipv6.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r39/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r39/pytest.log; exit $rc
