"""Summarise the rocprofv3 --pmc passes of tools/pmc_traffic.sh into profiles/pmc_traffic.json.

Dispatch attribution follows tools/pmc_probe.py's fixed order: 3 x full_u8, 3 x
counts_only, 3 x full_u32 Toeplitz launches.  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE (KiB) reads exactly half the bytes of a 16-B/lane coalesced stream on
gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.  TCC_EA0_RDREQ x 128 B
is recorded as an independent cross-check of the corrected read bytes.
"""
import csv
import collections
import json
import sys

src, out = sys.argv[1], sys.argv[2]
N, H, Q = 1 << 28, 128, 24
MODES = ["full_u8"] * 3 + ["counts_only"] * 3 + ["full_u32"] * 3
ALGO = {"full_u8": 17, "counts_only": 12, "full_u32": 20}


def per_dispatch(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if not any(k in r["Kernel_Name"] for k in ("rss_toeplitz_kernel", "rss_counts_perm_kernel")):
            continue
        agg.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += \
            float(r["Counter_Value"])
    return list(agg.values())


def pass_csv(name):
    """A pass's counter CSV: flattened (profiles/) or as rocprofv3 wrote it (gpurun_out/)."""
    import os
    flat = "%s/%s_counter_collection.csv" % (src, name)
    return flat if os.path.exists(flat) else "%s/%s/run_counter_collection.csv" % (src, name)


fetch = per_dispatch(pass_csv("fetch"))
write = per_dispatch(pass_csv("write"))
req = per_dispatch(pass_csv("req"))
modes = {}
for i, m in enumerate(MODES):
    rd = 2 * fetch[i]["FETCH_SIZE"] * 1024
    wr = write[i]["WRITE_SIZE"] * 1024
    rec = modes.setdefault(m, {"fetch_size_kib": [], "write_size_kib": [], "rdreq_x128_bytes": [],
                               "hbm_bytes": []})
    rec["fetch_size_kib"].append(fetch[i]["FETCH_SIZE"])
    rec["write_size_kib"].append(write[i]["WRITE_SIZE"])
    rec["rdreq_x128_bytes"].append(req[i].get("TCC_EA0_RDREQ_sum", 0) * 128)
    rec["hbm_bytes"].append(rd + wr)
for m, rec in modes.items():
    rec["hbm_bytes_per_launch"] = sum(rec["hbm_bytes"]) / len(rec["hbm_bytes"])
    rec["algorithmic_bytes_per_launch"] = ALGO[m] * N
    rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"]
summary = {
    "tuples": N, "htable": H, "queues": Q,
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum in "
              "three separate passes over tools/pmc_probe.py (tools/pmc_traffic.sh)",
    "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count for 16-B/lane streams, "
                  "MI355X_MICROARCH.md HBM section); write bytes = WRITE_SIZE x 1024",
    "modes": modes,
    # the bench configuration (u8 queue outputs) -- read by bench.py as roofline.traffic
    "queue_width": "u8",
    "hbm_bytes_per_launch": modes["full_u8"]["hbm_bytes_per_launch"],
}
json.dump(summary, open(out, "w"), indent=1)
for m, rec in modes.items():
    print(m, "%.4e B/launch" % rec["hbm_bytes_per_launch"], "x%.5f of algorithmic"
          % rec["traffic_over_algorithmic"])
