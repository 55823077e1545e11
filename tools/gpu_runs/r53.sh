# bench with the row-f secondary lines (IPv6 hash, key search)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r53
timeout -k 10 300 python bench.py > gpurun_out/r53/bench.json 2> gpurun_out/r53/bench.err || { tail gpurun_out/r53/bench.err; exit 1; }
cat gpurun_out/r53/bench.json
