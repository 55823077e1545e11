set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest2.log 2>&1; rc=$?
tail -5 gpurun_out/gputest2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/kbench 268435456 20 "product" > gpurun_out/kbench3.log 2>&1 && cat gpurun_out/kbench3.log
bash tools/gpu_bench_prof.sh r01b --steps 50 --warmup 5
