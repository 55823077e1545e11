#!/bin/bash
# GPU box: the round's one final validation of the last tree, in two stages that each fit one
# call -- `tests`: the full -m gpu suite and smoke(); `perf`: the driver's bench command, a
# rocprofv3 kernel trace of the same command (+ its timed-launch summary), the FETCH_SIZE /
# WRITE_SIZE passes of the bench's step and the distributed bench lines (world-1 RCCL,
# 8-rank gloo rehearsal).
# usage: tools/gpu_validate.sh TAG [tests|perf|all]     (outputs under gpurun_out/TAG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-validate}
STAGE=${2:-all}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$STAGE" = tests ] || [ "$STAGE" = all ]; then
  RSS_MARGIN_LOG=$O/guard_margin.jsonl timeout -k 10 1000 python -u -m pytest -q -m gpu \
      --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
  rc=$?
  tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -2 $O/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "$STAGE" = perf ] || [ "$STAGE" = all ]; then
  set -e
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
      python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1
  python3 $R/tools/prof_timed.py $O/prof/run_kernel_trace.csv $O/prof.log > $O/prof_timed.json
  cat $O/prof_timed.json
  mkdir -p $O/pmc && bash $R/tools/pmc_traffic.sh $TAG/pmc > $O/pmc.log 2>&1
  cd $R
  bash tools/gpu_dist_lines.sh $TAG/dist > $O/dist.log 2>&1
fi
echo "validate done"
