"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).
usage: python tools/pmc_summary.py gpurun_out/pmc1 [kernel-substring ...]"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
keep = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(root + "/p*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0].replace("void ", "")
        # template arguments dropped (k_blend_fwd<false, true> -> k_blend_fwd), except the
        # measurement-only counting forward, kept apart
        # and the projection backward with the Adam update fused in (the replayed step's) apart from the plain one
        k = ("k_blend_fwd_counting" if k.startswith("k_blend_fwd<true") else
             "k_project_bwd_adam" if k.startswith("k_project_bwd<true, true>") else re.sub(r"<.*", "", k))
        if keep and not any(s in k for s in keep):
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, d in sorted(agg.items()):
    print(k)
    for c, v in sorted(d.items()):
        print("   %-26s %.5g" % (c, sum(v) / len(v)))
