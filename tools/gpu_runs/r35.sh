# mode-switch probe from a fresh process, full-output launches first (ramp-up at start?)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r35
(rocm-smi --showclocks > gpurun_out/r35/clocks_before.txt 2>&1 || true)
timeout -k 10 120 python tools/mode_switch_probe.py full-first > gpurun_out/r35/probe.json 2> gpurun_out/r35/probe.err || { tail gpurun_out/r35/probe.err; exit 1; }
cat gpurun_out/r35/probe.json
timeout -k 10 120 python tools/mode_switch_probe.py full-first > gpurun_out/r35/probe2.json 2> gpurun_out/r35/probe2.err || { tail gpurun_out/r35/probe2.err; exit 1; }
cat gpurun_out/r35/probe2.json
(rocm-smi --showclocks > gpurun_out/r35/clocks_after.txt 2>&1 || true)
