#!/bin/bash
# GPU box: per-kernel breakdown of many-queues launches (tools/many_queues_trace.py) under
# rocprofv3 --kernel-trace --stats, one profiled process per (Q, mode).
# usage: tools/many_queues_trace.sh TAG "Q:mode[:option=value] ..."   (outputs under gpurun_out/TAG/)
# (option=value: a tests/hooks.py path option, run on the hooks build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for spec in $2; do
  IFS=: read -r q m opt <<< "$spec"
  tag=${q}_$m${opt:+_${opt//[=]/-}}
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 $R/tools/many_queues_trace.py $q $m 20 $opt > $O/$tag.log 2>&1 || exit $?
  tail -1 $O/$tag.log
done
echo "trace done"
