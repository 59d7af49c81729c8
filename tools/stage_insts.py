"""Per-stage instruction counts and marginal step time of the compact tier, from -DUR3E_DOUBLE_STAGE=k
builds (stage k runs twice; it is idempotent, so the results are unchanged): the difference against
the normal build of SQ_INSTS_* per wave and of the queue kernel's duration is stage k's share.
usage: stage_insts.py <rocprof out dir> (reads <dir>/<variant>/run_counter_collection.csv)"""
import csv, json, os, sys
NAMES = {"base": "normal build", "dbl0": "kinematics", "dbl6": "com_vel + cacc (r_vel_acc)",
         "dbl7": "RNE + passive + actuation", "dbl4": "collision", "dbl5": "constraint rows",
         "dbl8": "M^-1 qfrc_smooth (tree solve)", "dbl15": "Newton solver",
         "dbl20": "Newton: direction (H, Cholesky, solves)", "dbl21": "Newton: line search",
         "dbl22": "Newton: constraint-state evaluation", "dbl23": "Newton: gradient"}
root = sys.argv[1]
res = {}
for v in NAMES:
    p = os.path.join(root, v, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    per = {}
    for r in csv.DictReader(open(p)):
        if "w_env_step_q<64" not in r["Kernel_Name"]:
            continue
        d = per.setdefault(r["Dispatch_Id"], {"dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = list(per.values())[2:]  # skip the first launches (warm-up)
    if not rows:
        continue
    keys = [k for k in rows[0] if k.startswith("SQ_")]
    avg = {k: sum(x[k] for x in rows) / len(rows) for k in keys + ["dur"]}
    w = avg.get("SQ_WAVES", 2048.0)
    res[v] = {"dur_us": avg["dur"] / 1e3, **{k + "_per_wave": avg[k] / w for k in keys if k != "SQ_WAVES"}}
base = res.get("base")
out = {}
for v, r in res.items():
    row = {"stage": NAMES[v], **{k: round(x, 1) for k, x in r.items()}}
    if base and v != "base":
        row["delta"] = {k: round(r[k] - base[k], 1) for k in r}
    out[v] = row
print(json.dumps(out, indent=1))
