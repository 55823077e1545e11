# IPv6 CSV fast path: GPU tests + e2e rates against the pandas path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r40
timeout -k 10 600 python -u -m pytest tests/test_gpu_fields_ipv6.py tests/test_gpu_reta.py tests/test_fastcsv6.py -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r40/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r40/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/e2e_ipv6_bench.py > gpurun_out/r40/e2e6.out 2> gpurun_out/r40/e2e6.err || { tail gpurun_out/r40/e2e6.err; exit 1; }
tail -1 gpurun_out/r40/e2e6.out
