#!/bin/bash
# GPU box: HBM bytes of many-queues launches (tools/range8_pmc_probe.py: 3 launches of one
# (Q, mode) per process), FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes,
# summarised by tools/range8_pmc_summarize.py (every kernel but the input generator).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-range8_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for Q in 131072 262144; do
  for M in full counts; do
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_${Q}_$M -o run -- python3 $R/tools/range8_pmc_probe.py $Q $M > $OUT/fetch_${Q}_$M.log 2>&1
    timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_${Q}_$M -o run -- python3 $R/tools/range8_pmc_probe.py $Q $M > $OUT/write_${Q}_$M.log 2>&1
  done
done
python3 $R/tools/range8_pmc_summarize.py $OUT > $OUT/summary.json
cat $OUT/summary.json
