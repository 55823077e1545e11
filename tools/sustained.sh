# The bench step 50,000 times back to back (no extras): sustained rate, per-launch spread.
# GPU box: bash tools/sustained.sh  (writes gpurun_out/sustained/; a heartbeat file while it runs)
mkdir -p gpurun_out/sustained || exit 1
python -c "import torch; print('torch', torch.__version__, flush=True)" || exit 1
( for i in $(seq 1 22); do sleep 20; echo "bench running $((i*20)) s" >> gpurun_out/sustained/heartbeat.txt; done ) &
hb=$!
timeout -k 10 420 python -u bench.py --steps 50000 --warmup 100 --no-cpu-baseline --no-extras --configs3-steps 20 > gpurun_out/sustained/bench_50k.json 2> gpurun_out/sustained/bench_50k.err
rc=$?
kill $hb 2>/dev/null
tail -c 400 gpurun_out/sustained/bench_50k.json
exit $rc
