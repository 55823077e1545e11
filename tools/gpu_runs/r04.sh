set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/b4_graph.json 2> gpurun_out/b4_graph.err; rc=$?; cat gpurun_out/b4_graph.json; tail -3 gpurun_out/b4_graph.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-graph --no-cpu-baseline > gpurun_out/b4_eager.json 2> gpurun_out/b4_eager.err; rc=$?; cat gpurun_out/b4_eager.json; [ $rc -eq 0 ] || exit $rc
RSS_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 --tuples-per-gpu 67108864 --dist-backend gloo > gpurun_out/b4_w2.json 2> gpurun_out/b4_w2.err; rc=$?; cat gpurun_out/b4_w2.json; tail -5 gpurun_out/b4_w2.err; exit $rc
