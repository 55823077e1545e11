# CSV -> CSV above 4 GiB: device file path in segments vs the host text path, identical files
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r56
timeout -k 10 900 python tools/e2e_big.py 120000000 > gpurun_out/r56/big.json 2> gpurun_out/r56/big.err; rc=$?
tail -5 gpurun_out/r56/big.err; cat gpurun_out/r56/big.json; rm -rf /tmp/rss_big; exit $rc
