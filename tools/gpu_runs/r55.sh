# segmented rss_csv_hash_file: device CSV + CLI suites, then a 5.3 GB file end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r55
timeout -k 10 900 python -u -m pytest tests/test_gpu_csv_device.py tests/test_gpu_cli.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r55/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r55/pytest.log
[ $rc -eq 0 ] || exit $rc
df -h /tmp | tail -1
