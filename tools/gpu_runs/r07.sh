set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest7.log 2>&1; rc=$?
tail -15 gpurun_out/gputest7.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_prof.sh r01d --steps 50 --warmup 10
