#!/bin/bash
# GPU box: the placement tier under PMC counters (DESIGN.md §3 "Placement").
# One plain run of tools/place_pmc, then one rocprofv3 --pmc pass per counter group, each
# its own process (each re-measures its own candidates: tools/place_pmc.hip).
# Summarise with: python3 tools/place_pmc_summarize.py gpurun_out/<tag>
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-place_pmc}
K=${2:-12}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $R/tools/place_pmc $K 5 > $OUT/plain.txt 2>&1
pass() {
    local name=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run \
        -- $R/tools/place_pmc $K 5 > $OUT/$name.txt 2>&1
    echo "pass $name done"
}
pass utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
pass tcplat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE GRBM_EA_BUSY
pass ealevel TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum
pass eastall TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum
pass eadram TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_64B_sum
echo all passes done
