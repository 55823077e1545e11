set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest5.log 2>&1; rc=$?
tail -5 gpurun_out/gputest5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/keysearch_bench.py 4096 1048576 > gpurun_out/ks1.json 2>&1; rc=$?; cat gpurun_out/ks1.json | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/keysearch_bench.py 64 16777216 > gpurun_out/ks2.json 2>&1; rc=$?; cat gpurun_out/ks2.json | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/e2e_bench.py 16777216 262144 /tmp/rss_e2e > gpurun_out/e2e2.json 2> gpurun_out/e2e2.err; rc=$?; cat gpurun_out/e2e2.json; exit $rc
