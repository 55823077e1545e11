set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/e2e15.json 2> gpurun_out/e2e15.err || exit $?
tail -c 2500 gpurun_out/e2e15.json
RSS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --tuples-per-gpu 67108864 > gpurun_out/w2_15.json 2> gpurun_out/w2_15.err; rc=$?
cat gpurun_out/w2_15.json; tail -3 gpurun_out/w2_15.err; exit $rc
