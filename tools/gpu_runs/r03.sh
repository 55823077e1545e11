set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest3.log 2>&1; rc=$?
tail -5 gpurun_out/gputest3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/e2e_bench.py 16777216 262144 /tmp/rss_e2e > gpurun_out/e2e1.json 2> gpurun_out/e2e1.err; rc=$?
tail -3 gpurun_out/e2e1.err; cat gpurun_out/e2e1.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_prof.sh r01c --steps 50 --warmup 5
