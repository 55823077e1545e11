# box sampling: stream ceiling (kbench) + product (current) vs the T9 build, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r50
timeout -k 10 300 tools/kbench 268435456 20 policy > gpurun_out/r50/kbench_policy.log 2>&1 || exit $?
grep -E "product full u8|as product\)" gpurun_out/r50/kbench_policy.log
for k in 1 2; do
  timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r50/ab.jsonl 2>> gpurun_out/r50/ab.err || exit $?
  RSS_TOEPLITZ_LIB=$GRAFT_REPO_ROOT/tools/ab/librss_toeplitz_t9.so timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r50/ab.jsonl 2>> gpurun_out/r50/ab.err || exit $?
done
cat gpurun_out/r50/ab.jsonl
