set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_fields_ipv6.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest12.log 2>&1; rc=$?
tail -5 gpurun_out/gputest12.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ipv6_bench.py > gpurun_out/v6_12.json 2>&1; rc=$?; tail -2 gpurun_out/v6_12.json; exit $rc
