set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02e
mkdir -p $O
for i in 1 2; do echo "== process $i" >> $O/offsets.log; timeout -k 10 150 $R/tools/kbench 268435456 15 offsets >> $O/offsets.log 2>&1 || exit 1; done
echo done
