"""Per-launch averages of every counter collected by tools/gpu_calls/r05_j.sh for the compact step kernel."""
import csv, glob, json, os, sys

KEYS = ("w_env_step<64", "w_env_step_q<64")
src = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    vals = {}
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in KEYS):
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        v = v[1:] if len(v) > 1 else v
        res[k] = sum(v) / len(v)
w = res.get("SQ_WAVES", 1.0)
per_wave = {k + "/wave": v / w for k, v in res.items() if k.startswith("SQ_INSTS") or k.startswith("SQ_ACTIVE")}
res.update(per_wave)
json.dump(res, open(os.path.join(src, "breakdown.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
