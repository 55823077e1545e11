# box sampling 2: kbench T9 (kbench-local kernels) beside the library's product launch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r51
timeout -k 10 300 tools/kbench 268435456 20 T9 > gpurun_out/r51/kbench_t9.log 2>&1 || exit $?
cat gpurun_out/r51/kbench_t9.log
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r51/kbench_policy.log 2>&1 || exit $?
grep -E "as product\)" gpurun_out/r51/kbench_policy.log
timeout -k 10 120 python tools/ab_kernel.py
