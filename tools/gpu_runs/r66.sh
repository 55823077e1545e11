# PMC traffic of the current rss_toeplitz_kernel (after QM_FAST8): FETCH_SIZE / WRITE_SIZE /
# TCC_EA0 request passes (tag r01l_pmc), each pass its own rocprofv3 run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r66
timeout -k 10 900 bash tools/pmc_traffic.sh r01l_pmc > gpurun_out/r66/pmc.log 2>&1; rc=$?
tail -3 gpurun_out/r66/pmc.log
[ $rc -eq 0 ] || exit $rc
python tools/pmc_summarize.py gpurun_out/r01l_pmc gpurun_out/r66/pmc_traffic.json && cat gpurun_out/r66/pmc_traffic.json
