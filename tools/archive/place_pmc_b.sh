#!/bin/bash
# GPU box: second set of placement-tier counter passes (after tools/place_pmc.sh ruled out
# translation and memory-side latency): where the slow tier's requests wait -- TA/TCP/TD
# stalls, SQ vector-memory latency, and per-channel (non-summed) L2 counters.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-place_pmc_b}
K=${2:-12}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
pass() {
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run \
        -- $R/tools/place_pmc $K 5 > $OUT/$name.txt 2>&1
    echo "pass $name done"
}
pass tccch TCC_REQ TCC_TAG_STALL TCC_EA0_RDREQ TCC_EA0_WRREQ
pass tastall TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_RDRET_STALL_sum TD_TC_STALL_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE
pass sqlat SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU
pass tcclevel TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL
echo all passes done
