#!/bin/bash
# GPU box: the full -m gpu suite, smoke(), the driver's bench command and a rocprofv3
# --kernel-trace --stats of the same command (+ its timed-launch summary) -- the final
# validation without the PMC passes, A/B and sweep of gpu_validate.sh.  Every GPU step has
# its own time limit and the first failure ends the call.
# usage: tools/archive/gpu_suite_prof.sh TAG     (outputs under gpurun_out/TAG/)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-suite_prof}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
head -c 400 $O/bench.json; echo
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1
python3 $R/tools/prof_timed.py $O/prof/run_kernel_trace.csv $O/prof.log > $O/prof_timed.json
cat $O/prof_timed.json
echo "suite_prof done"
