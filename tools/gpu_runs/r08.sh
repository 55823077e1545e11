set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "flow" > gpurun_out/gputest8.log 2>&1; rc=$?
tail -5 gpurun_out/gputest8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --distribution flow --steps 50 --warmup 10 > gpurun_out/bench_flow.json 2> gpurun_out/bench_flow.err; rc=$?
cat gpurun_out/bench_flow.json; exit $rc
