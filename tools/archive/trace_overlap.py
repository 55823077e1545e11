"""Print the kernels of a rocprofv3 kernel trace in start order around the bench's timed
region (tool, not product): name, start offset, duration, gap to the previous kernel's end,
and which queue -- to see whether the collective's kernel overlaps the next hash launch.

    python tools/trace_overlap.py TRACE_CSV [LAST_N]
"""
import csv
import sys


def main(path, last_n=60):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                         r.get("Queue_Id", r.get("Stream_Id", "?")), r.get("Grid_Size", "?"),
                         r.get("Workgroup_Size", "?"), r.get("LDS_Block_Size", r.get("Lds_Size", "?"))))
    rows.sort()
    hash_idx = [i for i, r in enumerate(rows) if "rss_toeplitz_kernel" in r[2]]
    end = hash_idx[-1] + 1 if hash_idx else len(rows)
    sel = rows[max(0, end - last_n): end]
    t0 = sel[0][0]
    prev_end = None
    for s, e, name, q, grid, wg, lds in sel:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print("%10.1f us  dur %8.1f us  gap %7.1f us  q=%s grid=%s wg=%s lds=%s  %s"
              % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, grid, wg, lds, name))
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
