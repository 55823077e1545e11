set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest6.log 2>&1; rc=$?
tail -15 gpurun_out/gputest6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ipv6_bench.py > gpurun_out/v6.json 2>&1; rc=$?; tail -1 gpurun_out/v6.json; exit $rc
