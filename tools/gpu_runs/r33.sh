# rss_hash_host_multi (several contexts on cuda:0) + bench secondary lines with 3 warm launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r33
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_path.py tests/test_native_abi.py -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r33/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r33/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 2000 > gpurun_out/r33/bench.json 2> gpurun_out/r33/bench.err || { tail gpurun_out/r33/bench.err; exit 1; }
cat gpurun_out/r33/bench.json
