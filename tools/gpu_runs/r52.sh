# software-pipelined hash loop (next group's loads ahead of this group's stores): A/B vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r52
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r52/kbench_policy.log 2>&1 || exit $?
grep -E "as product\)" gpurun_out/r52/kbench_policy.log
for k in 1 2 3; do
  RSS_TOEPLITZ_LIB=$GRAFT_REPO_ROOT/tools/ab/librss_toeplitz_head.so timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r52/ab.jsonl 2>> gpurun_out/r52/ab.err || exit $?
  timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r52/ab.jsonl 2>> gpurun_out/r52/ab.err || exit $?
done
cat gpurun_out/r52/ab.jsonl
