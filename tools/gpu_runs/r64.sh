# pooled device blocks in the CSV device path: device CSV suites, then phase times again
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r64
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_csv6_device.py tests/test_gpu_csv_device.py > gpurun_out/r64/pytest.log 2>&1 &&
RSS_CSV_TIMING=1 timeout -k 10 300 python tools/e2e_ipv6_bench.py 8388608 16384 /tmp/rss_e2e6 > gpurun_out/r64/e2e6.log 2>&1 &&
RSS_CSV_TIMING=1 timeout -k 10 300 python tools/e2e_bench.py 16777216 16384 /tmp/rss_e2e > gpurun_out/r64/e2e4.log 2>&1; rc=$?
tail -2 gpurun_out/r64/pytest.log; grep "hash_file:" gpurun_out/r64/*.log; exit $rc
