# bench: per-launch HIP events inside the timed region; N=1 and a world-2 gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r27
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 2000 > gpurun_out/r27/bench.json 2> gpurun_out/r27/bench.err || { tail gpurun_out/r27/bench.err; exit 1; }
cat gpurun_out/r27/bench.json
RSS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --tuples-per-gpu 67108864 > gpurun_out/r27/w2.json 2> gpurun_out/r27/w2.err; rc=$?
cat gpurun_out/r27/w2.json; tail -3 gpurun_out/r27/w2.err; exit $rc
