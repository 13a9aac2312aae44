"""Summarise rocprofv3 --pmc passes (tools/pmc.sh): per kernel, counters summed over their
instances (XCD / SE / ...) per dispatch, then averaged over dispatches; plus derived ratios.

    python tools/pmc_summary.py [dir]

Derived: per-wave instruction counts (SQ_INSTS_* / SQ_WAVES), MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), effective clock = GRBM_GUI_ACTIVE / 8 / duration,
wait fractions of SQ_WAVE_CYCLES (quad-cycle units for both)."""
import collections
import csv
import glob
import os
import sys


def load(out):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", r.get("KernelName", "?"))
            disp = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[name][r["Counter_Name"]][disp] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(out, "p*", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    res = {}
    for name, cs in per.items():
        res[name] = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    return res, dur


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    res, dur = load(out)
    for name, c in sorted(res.items()):
        if not any(k in name for k in ("igemm", "wgrad", "head", "trace", "wino", "smallconv")):
            continue
        print(name[:150])
        for k, v in sorted(c.items()):
            print("   %-30s %.6g" % (k, v))
        w = c.get("SQ_WAVES")
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_INSTS_VMEM",
                      "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if k in c:
                    print("   per wave %-21s %.1f" % (k, c[k] / w))
        g = c.get("GRBM_GUI_ACTIVE")
        ds = dur.get(name)
        if g and ds:
            print("   effective clock GHz          %.3f" % (g / 8.0 / (sum(ds) / len(ds))))
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            print("   MFMA busy                    %.3f" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8.0 * 1024)))
        if g and "SQ_LDS_IDX_ACTIVE" in c:
            # per CU and GPU cycle (x4 if the counter runs in quad-cycles like SQ_WAVE_CYCLES)
            print("   LDS active / CU-cycle        %.3f" % (c["SQ_LDS_IDX_ACTIVE"] / (g / 8.0 * 256)))
        if g and "TA_TA_BUSY_sum" in c:
            print("   TA busy / CU-cycle           %.3f" % (c["TA_TA_BUSY_sum"] / (g / 8.0 * 256)))
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
                if k in c:
                    print("   %-28s %.3f of wave cycles" % (k, c[k] / wc))


if __name__ == "__main__":
    main()
