# bench twice on one box: --steps 20 and the default 50 (secondary-line spreads recorded)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r36
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 2000 > gpurun_out/r36/bench20.json 2> gpurun_out/r36/bench20.err || { tail gpurun_out/r36/bench20.err; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r36/bench50.json 2> gpurun_out/r36/bench50.err || { tail gpurun_out/r36/bench50.err; exit 1; }
cat gpurun_out/r36/bench20.json gpurun_out/r36/bench50.json
