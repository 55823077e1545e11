# packed-bucket key search: 4-key fallback for 40 < Q <= 80 (H <= 256); parity, throughput,
# rocprofv3 kernel stats and one PMC pass (LDS / VALU instruction mix, bank conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r25
timeout -k 10 600 python -u -m pytest tests/test_gpu_keysearch.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r25/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r25/pytest.log
[ $rc -eq 0 ] || exit $rc
for args in "4096 1048576 uniform" "4096 1048576 flow" "4096 1048576 uniform 128 64" \
            "4096 1048576 uniform 256 80" "4096 1048576 uniform 512 24"; do
  timeout -k 10 120 python tools/keysearch_bench.py $args >> gpurun_out/r25/ks.jsonl || exit $?
done
cat gpurun_out/r25/ks.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r25/prof -o ks \
    -- python3 $R/tools/keysearch_bench.py 4096 1048576 uniform > $R/gpurun_out/r25/prof.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/r25/pmc -o ks \
    -- python3 $R/tools/keysearch_bench.py 4096 1048576 uniform > $R/gpurun_out/r25/pmc.log 2>&1 || exit $?
echo ok
