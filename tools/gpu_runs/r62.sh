# phase times of rss_csv_hash_file / rss_csv6_hash_file (RSS_CSV_TIMING=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r62
export RSS_CSV_TIMING=1
timeout -k 10 300 python tools/e2e_ipv6_bench.py 8388608 16384 /tmp/rss_e2e6 > gpurun_out/r62/e2e6.log 2>&1 &&
timeout -k 10 300 python tools/e2e_bench.py 16777216 16384 /tmp/rss_e2e > gpurun_out/r62/e2e4.log 2>&1; rc=$?
grep "hash_file:" gpurun_out/r62/*.log; exit $rc
