# same-box A/B/C: previous kernel (12-bit tables, FAST16) / current (12-bit, FAST8) / nine 11-bit tables + FAST8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r46
for k in 1 2 3; do
  RSS_TOEPLITZ_LIB=$GRAFT_REPO_ROOT/tools/ab/librss_toeplitz_prev.so timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r46/ab.jsonl 2>> gpurun_out/r46/ab.err || exit $?
  timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r46/ab.jsonl 2>> gpurun_out/r46/ab.err || exit $?
  RSS_TOEPLITZ_LIB=$GRAFT_REPO_ROOT/tools/ab/librss_toeplitz_t9.so timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r46/ab.jsonl 2>> gpurun_out/r46/ab.err || exit $?
done
cat gpurun_out/r46/ab.jsonl
