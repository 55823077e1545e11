# rss_hash_host with threaded staging copies: parity + e2e host_path rate
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_reta.py tests/test_gpu_cli.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gputest20.log 2>&1; rc=$?
tail -3 gpurun_out/gputest20.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/e2e_bench.py > gpurun_out/e2e20.json 2> gpurun_out/e2e20.err; rc=$?
python -c "import json;d=json.load(open('gpurun_out/e2e20.json'));print(json.dumps({k:d[k] for k in ('host_path','csv_fastpath_host','csv_fastpath_device','cli_process')}))"; exit $rc
