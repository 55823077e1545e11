# kbench T9: nine 11/10-bit tables (60 KiB) at 2 workgroups / CU vs the product's 12-bit x1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r43
timeout -k 10 300 tools/kbench 268435456 20 T9 > gpurun_out/r43/kbench_t9.log 2>&1; rc=$?
cat gpurun_out/r43/kbench_t9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r43/kbench_policy.log 2>&1; rc=$?
tail -9 gpurun_out/r43/kbench_policy.log; exit $rc
