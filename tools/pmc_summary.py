"""Summarise rocprofv3 --pmc passes: per kernel name, mean counter value per dispatch."""
import csv, glob, os, sys, collections
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("KernelName", "?"))
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    if "igemm" not in name and "wgrad" not in name:
        continue
    print(name)
    for c, v in sorted(cs.items()):
        print("   %-28s %.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
