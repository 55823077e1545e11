"""Summarise tools/pmc_keysearch.sh's passes: per launch of rss_key_search_packed_kernel (the
first, warm-up launch dropped), the SQ counters per wave-step (64 tuples x 8 keys = 512 key x
tuple evaluations), the launch duration from the kernel trace, and the unit loads the bench's
key_search `frac` is stated against.

usage: python tools/pmc_keysearch_summarize.py OUTDIR > summary.json
"""
import collections
import csv
import json
import os
import sys

KEYS, TUPLES = 1024, 1 << 20
EVALS = KEYS * TUPLES
STEPS = EVALS / 512          # wave-steps: 64 lanes x 8 packed keys
CUS = 256


def counters(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "rss_key_search" not in r["Kernel_Name"]:
            continue
        agg.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += \
            float(r["Counter_Value"])
    return list(agg.values())[1:]  # drop the warm-up launch


def durations(path):
    out = []
    for r in csv.DictReader(open(path)):
        if "rss_key_search" in r["Kernel_Name"]:
            out.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return out[1:]


def find(d, name):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(name):
                return os.path.join(root, f)
    raise FileNotFoundError("%s under %s" % (name, d))


def mean(xs):
    return sum(xs) / len(xs)


src = sys.argv[1]
c1 = counters(find(os.path.join(src, "sq1"), "counter_collection.csv"))
c2 = counters(find(os.path.join(src, "sq2"), "counter_collection.csv"))
ms = durations(find(os.path.join(src, "trace"), "kernel_trace.csv"))
k = {}
for rows in (c1, c2):
    for name in rows[0]:
        k[name] = mean([r[name] for r in rows])
dur_ms = mean(ms)
# GRBM_GUI_ACTIVE counts GPU-busy clocks summed over the 8 XCDs
clock_ghz = k["GRBM_GUI_ACTIVE"] / 8 / (dur_ms * 1e6)
cu_cycles = CUS * dur_ms * 1e6 * clock_ghz
out = {
    "kernel": "rss_key_search_packed_kernel (8 keys per 8-byte table entry)",
    "keys": KEYS, "tuples": TUPLES, "launches": len(ms),
    "kernel_ms_trace": dur_ms,
    "key_tuple_evals_per_s": EVALS / (dur_ms / 1e3),
    "clock_ghz_from_grbm": clock_ghz,
    "per_wave_step": {  # 64 tuples x 8 keys
        "valu_insts": k["SQ_INSTS_VALU"] / STEPS,
        "lds_insts": k["SQ_INSTS_LDS"] / STEPS,
        "salu_insts": k["SQ_INSTS_SALU"] / STEPS,
        "lds_bank_conflict_cycles": k["SQ_LDS_BANK_CONFLICT"] / STEPS,
        "lds_idx_active_cycles": k["SQ_LDS_IDX_ACTIVE"] / STEPS,
    },
    "raw_means": k,
}
# unit loads over the launch: LDS array cycles per CU-cycle; VALU issue (quad-cycle counter)
# per SIMD-cycle
out["lds_array_busy_frac"] = k["SQ_LDS_IDX_ACTIVE"] / cu_cycles
out["valu_active_frac"] = 4 * k["SQ_ACTIVE_INST_VALU"] / (4 * cu_cycles)
out["lds_active_frac"] = 4 * k["SQ_ACTIVE_INST_LDS"] / (4 * cu_cycles)
json.dump(out, sys.stdout, indent=1)
print()
