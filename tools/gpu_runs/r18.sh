# device CSV kernels under rocprofv3 (kernel trace + stats); bench --gpus 2 self-relaunch (gloo)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python tools/csv_device_prof.py > gpurun_out/csvprof_plain.log 2>&1 || exit $?
cat gpurun_out/csvprof_plain.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/csvprof -o run -- python3 $R/tools/csv_device_prof.py > $R/gpurun_out/csvprof.log 2>&1 || exit $?
cd $R
cat gpurun_out/csvprof/run_kernel_stats.csv 2>/dev/null || find gpurun_out/csvprof -name '*kernel_stats.csv' -exec cat {} \;
RSS_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --tuples-per-gpu 67108864 > gpurun_out/w2_18.json 2> gpurun_out/w2_18.err; rc=$?
cat gpurun_out/w2_18.json; tail -2 gpurun_out/w2_18.err; exit $rc
