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
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def classes(r):
    """VALU wave-instructions per wave by class: FP64 arithmetic, int32, and the rest (moves, readlanes,
    selects, compares, conversions: data movement and control)"""
    g = lambda k: r.get(k + "_per_wave")
    if g("SQ_INSTS_VALU") is None or any(g(k) is None for k in F64 + ("SQ_INSTS_VALU_INT32",)):
        return None
    f64 = sum(g(k) for k in F64)
    i32 = g("SQ_INSTS_VALU_INT32")
    return {"valu": g("SQ_INSTS_VALU"), "f64": f64, "int32": i32, "other": g("SQ_INSTS_VALU") - f64 - i32}


base = res.get("base")
out = {}
for v, r in res.items():
    row = {"stage": NAMES[v], **{k: round(x, 1) for k, x in r.items()}}
    c = classes(r)
    if base and v != "base":
        row["delta"] = {k: round(r[k] - base[k], 1) for k in r}
        cb = classes(base)
        if c and cb:
            row["delta_classes"] = {k: round(c[k] - cb[k], 1) for k in c}
    elif c:
        row["classes"] = {k: round(x, 1) for k, x in c.items()}
    out[v] = row
if base and classes(base):
    # useful FP64 flops per FP64 wave-instruction: the oracle's counted flops of the env-steps one wave
    # runs (4,096 env-steps over SQ_WAVES waves) over the wave's FP64 VALU instructions
    fl = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "flops_r01.json")))
    fps = fl.get("flops_per_env_step") or fl.get("gym_v2", {}).get("flops_per_env_step")
    w = base.get("SQ_WAVES_per_wave") or 1.0
    steps_per_wave = 4096 / (res["base"].get("SQ_WAVES", 2048.0) if "SQ_WAVES" in res["base"] else 2048.0)
    if fps:
        out["flops_per_f64_instruction"] = round(fps * steps_per_wave / classes(base)["f64"], 2)
print(json.dumps(out, indent=1))
