"""Convert a rocprofv3 SQLite output (run_results.db) into kernel_trace.csv / kernel_stats.csv
with the columns of rocprofv3's own CSV output (the subset tools/*.py read).

usage: python tools/rocpd_to_csv.py <run_results.db> <out_prefix>"""
import collections
import csv
import sqlite3
import sys


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, lds_size "
                     "from kernels order by start").fetchall()
    with open(prefix + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y",
                    "Grid_Size_Z", "Workgroup_Size_X", "VGPR_Count", "LDS_Block_Size"])
        w.writerows(rows)
    agg = collections.OrderedDict()
    for name, s, e, *_ in rows:
        a = agg.setdefault(name, [0, 0, None, 0])
        d = e - s
        a[0] += 1; a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(v[1] for v in agg.values())
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (n, t, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, n, t, t / n, 100.0 * t / tot, mn, mx])


if __name__ == "__main__":
    main()
