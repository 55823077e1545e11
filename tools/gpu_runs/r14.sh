set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_csv_device.py tests/test_gpu_cli.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest14.log 2>&1; rc=$?
tail -5 gpurun_out/gputest14.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/e2e14.json 2> gpurun_out/e2e14.err; rc=$?
tail -c 3000 gpurun_out/e2e14.json; tail -5 gpurun_out/e2e14.err; exit $rc
