# fixed-cost probe + the bench step shape (zero counts then hash) vs back-to-back launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r32
timeout -k 10 120 python tools/fixed_cost_probe.py > gpurun_out/r32/fixed.json 2> gpurun_out/r32/fixed.err || { tail gpurun_out/r32/fixed.err; exit 1; }
cat gpurun_out/r32/fixed.json
true
true
