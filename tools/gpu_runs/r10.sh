set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest10.log 2>&1; rc=$?
tail -5 gpurun_out/gputest10.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dist_probe.py > gpurun_out/dist10.log 2>&1 || exit $?
cat gpurun_out/dist10.log
timeout -k 10 200 python tools/keysearch_bench.py 1024 1048576 uniform > gpurun_out/ks10_u.json || exit $?
timeout -k 10 200 python tools/keysearch_bench.py 1024 1048576 flow > gpurun_out/ks10_f.json || exit $?
cat gpurun_out/ks10_u.json gpurun_out/ks10_f.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench10.json 2> gpurun_out/bench10.err || exit $?
cat gpurun_out/bench10.json
