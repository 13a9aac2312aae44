"""Per (kernel, grid) launch counts and average durations from a rocprofv3 kernel trace CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0][:56], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
tot = sum(sum(v) for v in d.values())
print(f"{'kernel':56s} {'grid':>14s} {'wg':>5s} {'n':>4s} {'avg us':>9s} {'sum us':>9s} {'%':>5s}")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:56s} {k[1] + 'x' + k[2]:>14s} {k[3]:>5s} {len(v):4d} {sum(v) / len(v):9.2f} {sum(v):9.1f} {100 * sum(v) / tot:5.1f}")
