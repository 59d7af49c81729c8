"""Summarise tools/stall_pmc.sh: per-dispatch averages of the compact-tier queue kernel's SQ counters
(rocprofv3 csv, one row per counter per dispatch), as per-wave cycle shares."""
import csv, glob, json, os, sys
from collections import defaultdict

D = sys.argv[1]
KERNEL = "w_env_step_q<64"
vals = defaultdict(list)
dur = []
for f in sorted(glob.glob(os.path.join(D, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(lambda: defaultdict(float))
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if KERNEL not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d in per.values():
        for k, v in d.items():
            vals[k].append(v)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
w = avg.get("SQ_WAVES", 1.0)
out = {"dispatches": len(vals.get("SQ_WAVES", [])), "waves": w}
q = 4.0  # SQ_WAVE_CYCLES / WAIT / ACTIVE count quad-cycles
wc = avg.get("SQ_WAVE_CYCLES", 0) * q
out["wave_cycles_per_wave"] = wc / w
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
          "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_FLAT",
          "SQ_ACTIVE_INST_VMEM"):
    if k in avg and wc:
        out[k + "_share"] = round(avg[k] * q / wc, 4)
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM",
          "SQ_LDS_BANK_CONFLICT", "SQ_INST_CYCLES_SMEM"):
    if k in avg:
        out[k + "_per_wave"] = round(avg[k] / w, 1)
for k, n in (("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"), ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM"),
             ("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"), ("SQ_IFETCH_LEVEL", "SQ_IFETCH")):
    if k in avg and avg.get(n):
        out[k.replace("SQ_INST_LEVEL_", "latency_").replace("SQ_IFETCH_LEVEL", "latency_IFETCH")] = round(avg[k] / avg[n], 1)
for k in ("SQ_IFETCH", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQC_DCACHE_HITS",
          "SQC_DCACHE_MISSES"):
    if k in avg:
        out[k + "_per_wave"] = round(avg[k] / w, 1)
if "GRBM_GUI_ACTIVE" in avg:
    out["GRBM_GUI_ACTIVE"] = avg["GRBM_GUI_ACTIVE"]
for k in ("SQ_BUSY_CYCLES", "SQ_CYCLES"):
    if k in avg:
        out[k] = avg[k]
print(json.dumps(out, indent=1))
