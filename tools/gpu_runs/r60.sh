# kernel times of the IPv6 device CSV path (rocprofv3 kernel trace of the e2e tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r60
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r60/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/e2e_ipv6_bench.py 8388608 16384 /tmp/rss_e2e6 > $GRAFT_REPO_ROOT/gpurun_out/r60/e2e6.log 2>&1; rc=$?
find $GRAFT_REPO_ROOT/gpurun_out/r60/prof -name "*kernel_stats.csv" | head -3; exit $rc
