# device CSV parity after the LDS-staged parse / write kernels + their rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_csv_device.py tests/test_gpu_cli.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest19.log 2>&1; rc=$?
tail -4 gpurun_out/gputest19.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/csvprof19 -o run -- python3 $R/tools/csv_device_prof.py > $R/gpurun_out/csvprof19.log 2>&1 || exit $?
cd $R
tail -3 gpurun_out/csvprof19.log
cut -d, -f1-4 gpurun_out/csvprof19/run_kernel_stats.csv
