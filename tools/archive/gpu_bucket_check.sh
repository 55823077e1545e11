set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_pipeline.py tests/test_gpu_placement.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
RSS_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 3 --tuples-per-gpu 67108864 --no-extras --cpu-sample 2000 --cpu-procs 4 > $O/w4_gloo.json 2> $O/w4_gloo.err || { tail -30 $O/w4_gloo.err; exit 1; }
grep '^{' $O/w4_gloo.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['config']['parallelism'])"
