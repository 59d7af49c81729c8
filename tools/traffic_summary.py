"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (one directory per counter) into KiB per launch of
each step kernel (launches after the first three dropped).  usage: traffic_summary.py DIR [DIR...]"""
import csv
import os
import sys

for d in sys.argv[1:]:
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    by = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        by.setdefault((k, r["Counter_Name"]), []).append((float(r["Counter_Value"]), r["Scratch_Size"]))
    for (k, c), v in by.items():
        vals = [x[0] for x in v][3:] or [x[0] for x in v]
        print(f"{os.path.basename(d):36s} {c:10s} {sum(vals) / len(vals):10.1f} KiB/launch  scratch {v[0][1]:>4}  {k}")
