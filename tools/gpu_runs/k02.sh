set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 tools/kbench 268435456 20 > gpurun_out/kbench2.log 2>&1 && cat gpurun_out/kbench2.log
cd /tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run -- $GRAFT_REPO_ROOT/tools/kbench 268435456 2 counts > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1
echo pmc1 rc=$?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o run -- $GRAFT_REPO_ROOT/tools/kbench 268435456 2 counts > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1
echo pmc2 rc=$?
