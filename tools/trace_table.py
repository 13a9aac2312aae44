"""Per (kernel, grid) launch counts and average durations from a rocprofv3 kernel trace: a
*kernel_trace.csv or the default rocpd SQLite database (*.db, its `kernels` view).

    python tools/trace_table.py <trace.csv | results.db> [name filter] [skip first N launches]
"""
import collections
import csv
import sqlite3
import sys


def rows_of(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = "select name, grid_x, grid_y, workgroup_x, start, end from kernels order by start"
        for name, gx, gy, wx, s, e in c.execute(q):
            yield name, str(gx), str(gy), str(wx), (e - s) / 1000.0
    else:
        for r in csv.DictReader(open(path)):
            yield (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"],
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    d = collections.defaultdict(list)
    for name, gx, gy, wx, us in rows_of(path):
        if filt and filt not in name:
            continue
        d[(name.split("(")[0][:60], gx, gy, wx)].append(us)
    tot = sum(sum(v) for v in d.values())
    print(f"{'kernel':60s} {'grid':>14s} {'wg':>5s} {'n':>4s} {'avg us':>9s} {'sum us':>9s} {'%':>5s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[0]:60s} {k[1] + 'x' + k[2]:>14s} {k[3]:>5s} {len(v):4d} {sum(v) / len(v):9.2f} {sum(v):9.1f} "
              f"{100 * sum(v) / tot:5.1f}")


if __name__ == "__main__":
    main()
