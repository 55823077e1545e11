# configs[3] shape on one GPU: 2^30 tuples, one launch + eight shards (tests/test_gpu_1g.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r67
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_1g.py > gpurun_out/r67/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r67/pytest.log; exit $rc
