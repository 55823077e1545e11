set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02c
mkdir -p $O
for i in 1 2 3; do echo "== process $i" >> $O/contig.log; timeout -k 10 120 $R/tools/kbench 268435456 20 contig >> $O/contig.log 2>&1 || exit 1; done
echo contig-done
bash $R/tools/gpu_bench_prof.sh r02c > $O/gbp.log 2>&1
echo bench-done
