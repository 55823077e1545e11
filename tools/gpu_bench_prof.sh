#!/bin/bash
# Run on the GPU box: bench (N=1) + rocprofv3 kernel-trace stats of the same command.
# usage: tools/gpu_bench_prof.sh TAG [bench args...]
set -eo pipefail
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python $R/bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python $R/bench.py --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
python3 $R/tools/prof_timed.py $OUT/prof/run_kernel_trace.csv $OUT/prof.log > $OUT/prof_timed.json
cat $OUT/prof_timed.json
