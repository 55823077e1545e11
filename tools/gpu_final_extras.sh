#!/bin/bash
# GPU box: the -m gpu suite with per-test durations, and the end-to-end CSV rates (tools/e2e_bench.py)
# on the final tree.  usage: tools/gpu_final_extras.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-extras}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu --durations=30 tests > $O/pytest_durations.log 2>&1 || { tail -30 $O/pytest_durations.log; exit 1; }
tail -40 $O/pytest_durations.log | grep -E "s (call|setup)|passed" | head -35
gcc -O2 -o /tmp/gen_csv tools/gen_csv.c 2>/dev/null || true
timeout -k 10 300 python -u tools/e2e_bench.py 16777216 262144 /tmp/rss_e2e > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
tail -c 1500 $O/e2e.json
