# sharded GPU test, CLI GPU tests, bench (flow_like field), e2e with CLI-process timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_sharding.py tests/test_gpu_cli.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest17.log 2>&1; rc=$?
tail -4 gpurun_out/gputest17.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench17.json 2> gpurun_out/bench17.err || exit $?
cat gpurun_out/bench17.json
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/e2e17.json 2> gpurun_out/e2e17.err; rc=$?
tail -c 1800 gpurun_out/e2e17.json; tail -3 gpurun_out/e2e17.err; exit $rc
