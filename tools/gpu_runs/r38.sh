# pcapng + IPv6 pcap on the GPU (CLI) and the IPv6 / fields suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r38
timeout -k 10 600 python -u -m pytest tests/test_gpu_fields_ipv6.py tests/test_pcap.py -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r38/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r38/pytest.log; exit $rc
