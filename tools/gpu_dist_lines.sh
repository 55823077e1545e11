#!/bin/bash
# GPU box: the distributed bench lines on one GPU -- the world-1 RCCL run under torchrun and
# the 8-rank gloo rehearsal (all ranks on cuda:0; its value is meaningless, its blocks are
# what tests/test_bench_host.py parses).  usage: tools/gpu_dist_lines.sh TAG
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dist_lines}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 20 --warmup 5 \
    > $OUT/torchrun_w1_rccl.json 2> $OUT/w1.err
echo "w1 ok"
RSS_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 \
    --dist-backend gloo --tuples-per-gpu 67108864 --placement-probe 2 --steps 5 --warmup 2 \
    --settle-ms 0 --no-extras > $OUT/w8_gloo_rehearsal_1gpu.json 2> $OUT/w8.err
echo "w8 ok"
