"""Join tools/place_pmc.sh's per-dispatch PMC counters to the placement candidates.

Each pass is its own process with its own allocations (so its own tiers): per pass, the
rss_toeplitz_kernel dispatches are assigned to candidates by tools/place_pmc.hip's fixed
launch order (per candidate: 2 warm full, R full, R hash-only, R queue-only), and each
candidate's full-mode counters (mean over its R launches) are printed beside its duration
in that same pass (the trace's own End - Start).  Writes <dir>/summary.json and prints,
per pass and counter, the correlation of the counter (per launch) with the duration.

    python3 tools/place_pmc_summarize.py gpurun_out/<tag>
"""
import collections
import csv
import json
import os
import re
import sys

MODES = ("full", "hash_only", "queue_only")


def parse_plain(path):
    cands = []
    head = None
    for line in open(path):
        if line.startswith("place_pmc "):
            head = dict(re.findall(r"(\w+)=(\d+)", line))
        m = re.match(r"cand (\d+) in=(\d+) out=(\d+) order in=(\d+) h=(\d+) q=(\d+) "
                     r"va in=(\S+) h=(\S+) q=(\S+) full_ms=(\S+) hash_only_ms=(\S+) "
                     r"queue_only_ms=(\S+)", line)
        if m:
            g = m.groups()
            cands.append({"cand": int(g[0]), "in": int(g[1]), "out": int(g[2]),
                          "order": [int(g[3]), int(g[4]), int(g[5])],
                          "va": {"in": g[6], "h": g[7], "q": g[8]},
                          "event_ms": {"full": float(g[9]), "hash_only": float(g[10]),
                                       "queue_only": float(g[11])}})
    return head, cands


def dispatches(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "rss_toeplitz_kernel" not in r["Kernel_Name"]:
            continue
        d = agg.setdefault(int(r["Dispatch_Id"]), {"ns": int(r["End_Timestamp"]) -
                                                   int(r["Start_Timestamp"]),
                                                   "c": collections.Counter()})
        d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [agg[k] for k in sorted(agg)]


def corr(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxy = sum((x - mx) * (y - my) for x, y in zip(xs, ys))
    sxx = sum((x - mx) ** 2 for x in xs)
    syy = sum((y - my) ** 2 for y in ys)
    return sxy / (sxx * syy) ** 0.5 if sxx > 0 and syy > 0 else float("nan")


def main(root):
    out = {"passes": {}}
    for name in sorted(os.listdir(root)):
        csv_path = os.path.join(root, name, "run_counter_collection.csv")
        txt = os.path.join(root, name + ".txt")
        if not (os.path.exists(csv_path) and os.path.exists(txt)):
            continue
        head, cands = parse_plain(txt)
        R = int(head["R"])
        per = 2 + 3 * R
        ds = dispatches(csv_path)
        if len(ds) != per * len(cands):
            print("%s: %d dispatches, expected %d -- skipped" % (name, len(ds), per * len(cands)))
            continue
        rows = []
        for c in cands:
            block = ds[per * c["cand"]: per * (c["cand"] + 1)]
            rec = dict(c)
            for mi, mode in enumerate(MODES):
                part = block[2 + mi * R: 2 + (mi + 1) * R]
                rec[mode + "_trace_ms"] = sum(d["ns"] for d in part) / len(part) / 1e6
                keys = sorted(set().union(*[d["c"].keys() for d in part]))
                rec[mode + "_counters"] = {k: sum(d["c"][k] for d in part) / len(part) for k in keys}
            rows.append(rec)
        ms = [r["full_trace_ms"] for r in rows]
        corrs = {k: corr([r["full_counters"][k] for r in rows], ms)
                 for k in rows[0]["full_counters"]}
        out["passes"][name] = {"candidates": rows, "corr_with_full_ms": corrs}
        print("== pass %s  (%d candidates; full-mode trace ms %.4f .. %.4f)" %
              (name, len(rows), min(ms), max(ms)))
        fast = min(rows, key=lambda r: r["full_trace_ms"])
        slow = max(rows, key=lambda r: r["full_trace_ms"])
        for k in sorted(corrs):
            print("  %-48s corr %+.3f   fastest %.4g   slowest %.4g   ratio %.3f" %
                  (k, corrs[k], fast["full_counters"][k], slow["full_counters"][k],
                   slow["full_counters"][k] / fast["full_counters"][k]
                   if fast["full_counters"][k] else float("nan")))
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
