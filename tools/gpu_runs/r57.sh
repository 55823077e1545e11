# rehearse the N=8 bench path on one GPU: 8 ranks (gloo), every rank on cuda:0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r57
RSS_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 10 --warmup 3 \
    --dist-backend gloo --tuples-per-gpu 16777216 > gpurun_out/r57/w8.json 2> gpurun_out/r57/w8.err; rc=$?
cat gpurun_out/r57/w8.json; grep -v Gloo gpurun_out/r57/w8.err | tail -3; exit $rc
