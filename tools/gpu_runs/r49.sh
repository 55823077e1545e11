# start-up costs: bare HIP init (C) vs the library's first calls from Python
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r49
for k in 1 2; do
  hipcc --offload-arch=gfx950 -O2 -x hip tools/hipinit_probe.c -o tools/hipinit_probe 2>/dev/null; timeout -k 10 60 tools/hipinit_probe >> gpurun_out/r49/init.jsonl || exit $?
  timeout -k 10 60 python tools/init_probe.py >> gpurun_out/r49/init.jsonl || exit $?
done
HIP_ENABLE_DEFERRED_LOADING=1 timeout -k 10 60 python tools/init_probe.py >> gpurun_out/r49/init.jsonl || exit $?
cat gpurun_out/r49/init.jsonl
