#!/bin/bash
# GPU box, round 3 (b): the full -m gpu suite (test failures do not stop the script; a
# crash, abort or time limit does), the (H, Q) sweep, the ballast placement experiment, the
# world-1 RCCL bench under torchrun and the 8-rank gloo rehearsal on this one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03_b}
mkdir -p $OUT $OUT/bench_lines
cd $R
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests \
    > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python tools/config_sweep_probe.py > $OUT/config_sweep.jsonl 2> $OUT/config_sweep.err
echo "sweep ok"
for g in 0 16 64 0 16 64 0 16 64; do
    timeout -k 10 120 ./tools/place_pmc 6 5 268435456 ballast $g >> $OUT/ballast.txt 2>&1
done
for g in 16 64 16 64; do
    timeout -k 10 120 ./tools/place_pmc 6 5 268435456 ballast $g free >> $OUT/ballast.txt 2>&1
done
echo "ballast ok"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 20 --warmup 5 \
    > $OUT/bench_lines/torchrun_w1_rccl.json 2> $OUT/w1.err
echo "w1 ok"
RSS_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 \
    --dist-backend gloo --tuples-per-gpu 67108864 --placement-probe 2 --steps 5 --warmup 2 \
    --settle-ms 0 --no-extras > $OUT/bench_lines/w8_gloo_rehearsal_1gpu.json 2> $OUT/w8.err
echo "w8 ok"
