#!/bin/bash
# GPU box: SQ / LDS counter passes over tools/pmc_probe.py (3 x full-u8, 3 x counts-only,
# 3 x full-u32 launches on 2^28 tuples), one rocprofv3 --pmc run per pass (at most 8 SQ +
# 2 GRBM counters each), summarised per tuple by tools/pmc_summarize.py --sq.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_sq}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq1 -o run -- python3 $R/tools/pmc_probe.py > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d $OUT/sq2 -o run -- python3 $R/tools/pmc_probe.py > $OUT/sq2.log 2>&1
echo done
