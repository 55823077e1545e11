# same-box A/B: previous product kernel (8 x 12-bit tables, FAST16) vs current (9 x 11/10-bit, FAST8)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r45
for k in 1 2 3; do
  RSS_TOEPLITZ_LIB=$GRAFT_REPO_ROOT/tools/ab/librss_toeplitz_prev.so timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r45/ab.jsonl 2>> gpurun_out/r45/ab.err || exit $?
  timeout -k 10 120 python tools/ab_kernel.py >> gpurun_out/r45/ab.jsonl 2>> gpurun_out/r45/ab.err || exit $?
done
cat gpurun_out/r45/ab.jsonl
