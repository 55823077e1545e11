#!/bin/bash
# GPU box: SQ / LDS counter passes over the key search (tools/keysearch_bench.py: 1024 random
# keys x 2^20 uniform tuples, H = 128, Q = 24 -- the bench's row_f_kernels.key_search line;
# 6 launches of rss_key_search_packed_kernel), one rocprofv3 --pmc run per pass (at most 8 SQ
# + 2 GRBM counters each), summarised by tools/pmc_keysearch_summarize.py.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_keysearch}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq1 -o run -- python3 $R/tools/keysearch_bench.py > $OUT/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 $R/tools/keysearch_bench.py > $OUT/sq2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/keysearch_bench.py > $OUT/trace.log 2>&1
python3 $R/tools/pmc_keysearch_summarize.py $OUT > $OUT/summary.json
cat $OUT/summary.json
