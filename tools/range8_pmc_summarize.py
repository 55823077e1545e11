"""Summarise tools/range8_pmc.sh: per launch HBM bytes of a many-queues launch (all its
kernels: the hash pass, wide passes, reduces, recount gates) against its algorithmic bytes
(full: 12 B read + 4 B hash + 4 B queue per tuple; counts only: 12 B read).  Read bytes =
2 x FETCH_SIZE x 1024 (the gfx950 half count of 16-B/lane streams, MI355X_MICROARCH.md HBM
section), write bytes = WRITE_SIZE x 1024.

usage: python tools/range8_pmc_summarize.py OUTDIR > summary.json"""
import csv
import json
import os
import sys

N = 1 << 28
src = sys.argv[1]


def total(name, counter):
    path = None
    for root, _, files in os.walk(os.path.join(src, name)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(root, f)
    kernels = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        # the launch's own kernels and its hipMemsetAsync fill; not the input generator nor
        # the probe's torch zeros / sum
        if r["Counter_Name"] != counter or "generate" in name or not (
                name.startswith("rss_") or "fillBuffer" in name):
            continue
        k = name.split("(")[0][:90]
        kernels[k] = kernels.get(k, 0.0) + float(r["Counter_Value"])
    return kernels


out = {"tuples": N, "htable": 1 << 30, "launches_per_process": 3, "modes": {}}
for Q in (131072, 262144):
    for m in ("full", "counts"):
        f = total("fetch_%d_%s" % (Q, m), "FETCH_SIZE")
        w = total("write_%d_%s" % (Q, m), "WRITE_SIZE")
        rd = 2 * sum(f.values()) * 1024 / 3
        wr = sum(w.values()) * 1024 / 3
        algo = N * (20 if m == "full" else 12)
        out["modes"]["%d_%s" % (Q, m)] = {
            "read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
            "algorithmic_bytes": algo, "traffic_over_algorithmic": (rd + wr) / algo,
            "fetch_kib_by_kernel": {k: v / 3 for k, v in f.items()},
            "write_kib_by_kernel": {k: v / 3 for k, v in w.items()}}
json.dump(out, sys.stdout, indent=1)
print()
