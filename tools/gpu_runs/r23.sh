# rss_hash_host direct-DMA path for page-locked buffers: parity + e2e host_path rates
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r23
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_parity.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r23/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r23/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/r23/e2e.json 2> gpurun_out/r23/e2e.err; rc=$?
tail -5 gpurun_out/r23/e2e.err
python -c "import json;d=json.load(open('gpurun_out/r23/e2e.json'));print(json.dumps({k:d[k] for k in ('host_path','host_path_pinned','host_path_pinned_4x','csv_fastpath_device')}))"; exit $rc
