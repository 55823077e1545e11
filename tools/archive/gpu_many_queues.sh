#!/bin/bash
# GPU box: many queues -- the range-hist, bench-launch and single-pass tests, the many-queues
# rows of the config sweep (byte vs 12-bit tables), and the same-buffer A/B of the bench's
# step incl. RSS_OFF32=0.  usage: tools/archive/gpu_many_queues.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03/e}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_range_hist.py tests/test_gpu_bench_launch.py tests/test_gpu_single_pass.py \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python tools/config_sweep_probe.py many > $O/config_sweep_many.jsonl 2> $O/sweep.err || exit 1
cat $O/config_sweep_many.jsonl
for p in 1 2; do
    timeout -k 10 200 python tools/ws_order_ab.py 6 > $O/ab_$p.json 2> $O/ab_$p.err || exit 1
done
python -c "
import json
for p in (1, 2):
    d = json.load(open('$O/ab_%d.json' % p))
    print({k: (v['median'] if isinstance(v, dict) and 'median' in v else v) for k, v in d.items()})
"
