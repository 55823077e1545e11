# PCIe probe: pinned H2D, D2H and both at once (ceiling for the direct-DMA host path)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r28
timeout -k 10 120 python tools/pcie_probe.py > gpurun_out/r28/pcie.json 2> gpurun_out/r28/pcie.err || { tail gpurun_out/r28/pcie.err; exit 1; }
cat gpurun_out/r28/pcie.json
