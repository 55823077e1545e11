#!/bin/bash
# GPU box: the round's validation in one call -- the -m gpu suite, smoke(), the bench and a
# rocprofv3 kernel-trace of the bench with its timed-launch summary (tools/gpu_bench_prof.sh).
# usage: tools/gpu_validate.sh TAG     (outputs under gpurun_out/TAG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-validate}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
bash $R/tools/gpu_bench_prof.sh $TAG > $O/gbp.log 2>&1 || { tail $O/gbp.log; exit 1; }
python3 - "$O" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read())
print(round(d["value"] / 1e9, 1), "G tuples/s, frac", round(d["roofline"]["frac"], 4),
      "placement", d["placement"]["chosen"], round(d["placement"]["chosen_ms"], 4),
      "first", round(d["placement"]["first_allocation_ms"], 4))
PY
