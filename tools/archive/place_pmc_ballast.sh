#!/bin/bash
# GPU box: the ballast placement recipes (DESIGN §3 "Placement"): hold 0 / 16 / 64 GiB, or
# allocate and free it, before the bench's buffers; three processes each.  Needs tools/place_pmc
# (hipcc --offload-arch=gfx950 -O3 -o tools/place_pmc tools/place_pmc.hip).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ballast}
mkdir -p $OUT
cd $R
for g in 0 16 64 0 16 64 0 16 64; do
    timeout -k 10 120 ./tools/place_pmc 6 5 268435456 ballast $g >> $OUT/ballast.txt 2>&1
done
for g in 16 64 16 64; do
    timeout -k 10 120 ./tools/place_pmc 6 5 268435456 ballast $g free >> $OUT/ballast.txt 2>&1
done
echo "ballast ok"
