# IPv6 CSV end to end: device text path vs host text path (8M rows) + pandas (128K rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r59
timeout -k 10 300 python tools/e2e_ipv6_bench.py 8388608 131072 /tmp/rss_e2e6 > gpurun_out/r59/e2e6.log 2>&1; rc=$?
tail -1 gpurun_out/r59/e2e6.log > gpurun_out/r59/e2e6.json; tail -c 1500 gpurun_out/r59/e2e6.log; exit $rc
