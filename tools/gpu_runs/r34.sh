# mode-switch probe: counts-only launch times before / after full-output launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r34
timeout -k 10 120 python tools/mode_switch_probe.py > gpurun_out/r34/probe.json 2> gpurun_out/r34/probe.err || { tail gpurun_out/r34/probe.err; exit 1; }
cat gpurun_out/r34/probe.json
