# packed-bucket key search: parity + throughput (H=128 packed8, H=512 packed16, H=100 pair)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r24
timeout -k 10 600 python -u -m pytest tests/test_gpu_keysearch.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r24/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r24/pytest.log
[ $rc -eq 0 ] || exit $rc
for args in "4096 1048576 uniform" "4096 1048576 flow" "1024 1048576 uniform" "64 16777216 uniform" \
            "4096 1048576 uniform 512 24" "4096 1048576 uniform 100 24" "4096 1048576 uniform 128 64"; do
  timeout -k 10 120 python tools/keysearch_bench.py $args >> gpurun_out/r24/ks.jsonl || exit $?
done
cat gpurun_out/r24/ks.jsonl
