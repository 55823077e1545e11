"""Summarise a ``rocprofv3 --kernel-trace`` of ``bench.py`` over its TIMED launches only
(tool, not product).

``run_kernel_stats.csv`` averages every launch of the kernel in the process: the placement
probe's launches on all candidate buffers, the warmup, the timed steps and the secondary
lines.  The bench's ``roofline.kernel_ms`` is the mean over the K timed launches, so the
comparable profiler figure is the mean duration of exactly those dispatches.  With the bench
line of the same profiled run (``prof.log``), the full-output kernel's dispatches are, in
order: the probe (inputs x outputs x (3 warm + 5 timed)), the clock-settle launches
(``settle.launches``), W warmup steps, K timed steps -- or, since the probe and the settle
carry RSS_FLAG_ADDR64 (``placement.probe_addr64``; the spread and flow-like launches too),
W warmup steps and K timed steps only.

    python tools/prof_timed.py TRACE_CSV PROF_LOG > summary.json
"""
import csv
import json
import sys

PROBE_LAUNCHES = 3 + 5  # placement.choose_stream_buffers: probe_warm + probe_reps


def main(trace_path, log_path):
    line = None
    with open(log_path) as f:
        for raw in f:
            if raw.startswith("{") and '"metric"' in raw:
                line = json.loads(raw)
    if line is None:
        raise SystemExit("no bench line in %s" % log_path)
    cand = line["placement"]["candidates"]
    probe = cand["inputs"] * cand["outputs"] * PROBE_LAUNCHES
    w, k = line["warmup"], line["steps"]
    probe += line.get("settle", {}).get("launches", 0)
    if line["placement"].get("probe_addr64"):
        # round 3 on: the probe and the settle launch the 64-bit instance (RSS_FLAG_ADDR64),
        # so this kernel's row starts with the warmup steps
        probe = 0
    name = "rss_toeplitz_kernel<true, 4, 0, 2, true, true, false>"  # full output, u8 queues, 32-bit offsets
    durs = []
    with open(trace_path) as f:
        for row in csv.DictReader(f):
            if name in row["Kernel_Name"]:
                durs.append((int(row["Dispatch_Id"]),
                             int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    durs = [d for _, d in sorted(durs)]
    timed = durs[probe + w: probe + w + k]
    if len(timed) != k:
        raise SystemExit("expected %d timed launches, found %d" % (k, len(timed)))
    mean_ms = sum(timed) / k / 1e6
    out = {
        "kernel": name,
        "launches_in_trace": len(durs),
        "probe_and_settle_launches": probe, "warmup": w, "timed": k,
        "rocprof_timed_mean_ms": mean_ms,
        "rocprof_timed_min_max_ms": [min(timed) / 1e6, max(timed) / 1e6],
        "bench_kernel_ms_same_run": line["roofline"]["kernel_ms"],
        "rel_diff": mean_ms / line["roofline"]["kernel_ms"] - 1,
        "rocprof_all_launches_mean_ms": sum(durs) / len(durs) / 1e6,
        "placement_chosen": line["placement"]["chosen"],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
