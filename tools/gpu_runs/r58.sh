# IPv6 device CSV path: new parity suite + the IPv4 device CSV and IPv6 CLI suites it touches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r58
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_csv6_device.py tests/test_gpu_csv_device.py tests/test_gpu_fields_ipv6.py \
    tests/test_gpu_reta.py tests/test_gpu_cli.py > gpurun_out/r58/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r58/pytest.log; exit $rc
