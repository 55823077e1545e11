# IPv6 narrow queues: parity + throughput; bench step count stability (50 vs 200 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_fields_ipv6.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest21.log 2>&1; rc=$?
tail -3 gpurun_out/gputest21.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ipv6_bench.py > gpurun_out/v6_21.json 2>&1 || exit $?
tail -1 gpurun_out/v6_21.json
for k in 50 200 50 200; do
  timeout -k 10 300 python bench.py --steps $k --warmup 20 --no-cpu-baseline > gpurun_out/b21_$k.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b21_$k.json'));print($k, round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done
