"""Shrink rocprofv3 CSVs on the GPU box before they are copied back: keep only the rows of the step
kernels (w_env_step*, w_env_step_list*) in counter-collection / kernel-trace files.
usage: filter_csv.py FILE..."""
import csv
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        rows = list(csv.reader(f))
    if not rows:
        continue
    hdr = rows[0]
    key = "Kernel_Name" if "Kernel_Name" in hdr else ("Name" if "Name" in hdr else None)
    if key is None:
        continue
    k = hdr.index(key)
    keep = [hdr] + [r for r in rows[1:] if "w_env_step" in r[k]]
    with open(path, "w", newline="") as f:
        csv.writer(f).writerows(keep)
    print(path, len(rows) - 1, "->", len(keep) - 1)
