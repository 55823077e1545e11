set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_placement.py tests/test_gpu_integration_stub.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2 3; do timeout -k 10 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit 1; done
python - <<'PY'
import json
for l in open("gpurun_out/r02d/bench.jsonl"):
    d=json.loads(l); p=d["placement"]
    print(round(d["value"]/1e9,1), round(d["roofline"]["frac"],4), p["chosen"], round(p["chosen_ms"],4), round(p["first_allocation_ms"],4))
PY
