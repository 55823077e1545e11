# fixed-cost probe (kernel time vs n) + bench with the hbm_read_roofline object
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r31
timeout -k 10 120 python tools/fixed_cost_probe.py > gpurun_out/r31/fixed.json 2> gpurun_out/r31/fixed.err || { tail gpurun_out/r31/fixed.err; exit 1; }
cat gpurun_out/r31/fixed.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 2000 > gpurun_out/r31/bench.json 2> gpurun_out/r31/bench.err || { tail gpurun_out/r31/bench.err; exit 1; }
cat gpurun_out/r31/bench.json
