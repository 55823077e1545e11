# kbench policy probe: store cache-policy bits, XCD-contiguous mapping, 2-iteration loads (12R+5W)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r42
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r42/kbench_policy.log 2>&1; rc=$?
cat gpurun_out/r42/kbench_policy.log; exit $rc
