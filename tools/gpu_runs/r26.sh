# xor3 (v_bitop3) hash trees + packed key search with SDWA byte buckets: full GPU suite,
# smoke, bench + rocprofv3 stats (tag r01h), key search and IPv6 throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r26
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/r26/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r26/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r26/smoke.log 2>&1 || exit $?
cat gpurun_out/r26/smoke.log
bash tools/gpu_bench_prof.sh r01h > gpurun_out/r26/bench_prof.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r26/bench_prof.log
for args in "4096 1048576 uniform" "4096 1048576 flow" "4096 1048576 uniform 128 64" \
            "4096 1048576 uniform 512 24" "4096 1048576 uniform 100 24"; do
  timeout -k 10 120 python tools/keysearch_bench.py $args >> gpurun_out/r26/ks.jsonl || exit $?
done
cat gpurun_out/r26/ks.jsonl
timeout -k 10 120 python tools/ipv6_bench.py > gpurun_out/r26/ipv6.json 2>&1 || exit $?
cat gpurun_out/r26/ipv6.json
