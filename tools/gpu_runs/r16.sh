# full GPU suite, bench + rocprofv3 kernel stats, PMC HBM traffic, e2e, world-2 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest16.log 2>&1; rc=$?
tail -4 gpurun_out/gputest16.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_prof.sh r01e --steps 50 --warmup 10 > gpurun_out/r01e.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r01e.log
bash tools/pmc_traffic.sh pmc16 > gpurun_out/pmc16.log 2>&1 || exit $?
tail -2 gpurun_out/pmc16.log
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/e2e16.json 2> gpurun_out/e2e16.err || exit $?
tail -c 1200 gpurun_out/e2e16.json
RSS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --tuples-per-gpu 67108864 > gpurun_out/w2_16.json 2> gpurun_out/w2_16.err; rc=$?
cat gpurun_out/w2_16.json; tail -3 gpurun_out/w2_16.err; exit $rc
