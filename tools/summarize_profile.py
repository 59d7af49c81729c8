"""Summarise a tools/profile_round.sh run into profiles/<name>/ (kernel stats, HBM and SQ counters).

HBM bytes per launch follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE are
collected in separate passes, both in KiB; on gfx950 FETCH_SIZE counts one half of each wide
coalesced read, so the fetch figure is doubled.
usage: summarize_profile.py gpurun_out/<run> <name> [round] [kind: traffic | traffic_mesh]
(bench.py reads profiles/<kind>_<round>.json: `traffic` for the headline model, `traffic_mesh` for
--model main_mesh)"""
import csv, json, os, shutil, sys

src, name = sys.argv[1], sys.argv[2]
rnd = sys.argv[3] if len(sys.argv) > 3 else "r05"
kind = sys.argv[4] if len(sys.argv) > 4 else "traffic"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(REPO, "profiles", name)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
KEYS = ("w_env_step<64", "w_env_step_q<64")  # the dominant step kernel (env-step launch or substep queue)


def counters(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if not any(k in r["Kernel_Name"] for k in KEYS):
            continue
        out.setdefault(r["Counter_Name"], []).append(
            dict(value=float(r["Counter_Value"]), dispatch=int(r["Dispatch_Id"]),
                 dur_ns=int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                 lds=int(r["LDS_Block_Size"]), scratch=int(r["Scratch_Size"]),
                 vgpr=int(r["VGPR_Count"]), agpr=int(r.get("Accum_VGPR_Count", 0) or 0)))
    return out


def per_launch(vals):
    v = [x["value"] for x in vals]
    v = v[1:] if len(v) > 1 else v  # first timed launch after warmup is kept out
    return sum(v) / len(v)


fe = counters(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))["FETCH_SIZE"]
wr = counters(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))["WRITE_SIZE"]
fkb, wkb = per_launch(fe), per_launch(wr)
kname = next(r["Kernel_Name"] for r in csv.DictReader(open(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv")))
             if any(k in r["Kernel_Name"] for k in KEYS))
hbm = dict(kernel=kname.split("(")[0], envs_per_launch=4096,
           fetch_kib_per_launch=fkb, write_kib_per_launch=wkb,
           hbm_bytes_per_launch=(2 * fkb + wkb) * 1024,
           launch_resources=dict(lds_bytes=fe[0]["lds"], scratch_bytes_per_lane=fe[0]["scratch"],
                                 vgpr=fe[0]["vgpr"], agpr=fe[0]["agpr"]),
           note="FETCH_SIZE doubled (gfx950 wide-read correction); KiB units from rocprofv3. launch_resources are "
                "rocprofv3's dispatch fields: lds_bytes is the STATIC group segment rounded to its 512 B granule "
                "(the working set is dynamic LDS, w_dyn_lds, which the dispatch record leaves out) and vgpr is "
                "the descriptor's VGPR granule count x 4 (gfx950 wave64 allocates VGPRs in granules of 8), so "
                "the code object's figures (tools/kinfo.py, bench kernel_resources) are the ones to quote")
json.dump(hbm, open(os.path.join(dst, "pmc_hbm.json"), "w"), indent=1)
sq = counters(os.path.join(src, "pmc_sq", "run_counter_collection.csv"))
sqs = {k: per_launch(v) for k, v in sq.items()}
if "SQ_WAVE_CYCLES" in sqs:
    wc = sqs["SQ_WAVE_CYCLES"]
    sqs["frac_wait_any"] = sqs.get("SQ_WAIT_ANY", 0) / wc
    sqs["frac_active_inst"] = sqs.get("SQ_ACTIVE_INST_ANY", 0) / wc
    sqs["valu_insts_per_wave"] = sqs.get("SQ_INSTS_VALU", 0) / sqs["SQ_WAVES"]
sq2p = os.path.join(src, "pmc_sq2", "run_counter_collection.csv")
if os.path.exists(sq2p):
    sq2 = {k: per_launch(v) for k, v in counters(sq2p).items()}
    # SQ_ACTIVE_INST_VALU is in quad-cycles; SQ_THREAD_CYCLES_VALU in thread-cycles: active lanes per
    # VALU-busy cycle out of 64
    if sq2.get("SQ_ACTIVE_INST_VALU"):
        sq2["valu_lane_utilisation"] = sq2["SQ_THREAD_CYCLES_VALU"] / (4.0 * sq2["SQ_ACTIVE_INST_VALU"] * 64.0)
    sqs.update({k: v for k, v in sq2.items() if k != "SQ_WAVES"})
json.dump(sqs, open(os.path.join(dst, "pmc_sq.json"), "w"), indent=1)
import subprocess
head = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
dirty = subprocess.run(["git", "-C", REPO, "status", "--porcelain", "--untracked-files=no", "--", "ur3e_amd/csrc",
                        "include"], capture_output=True, text=True).stdout.strip()
json.dump({"hbm_bytes_per_launch": hbm["hbm_bytes_per_launch"], "source": f"profiles/{name}/pmc_hbm.json",
           "head": head + ("+dirty-csrc" if dirty else ""), "kernel": hbm["kernel"]},
          open(os.path.join(REPO, "profiles", f"{kind}_{rnd}.json"), "w"))
stats = list(csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))))
for r in stats[:4]:
    print(r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6, "ms")
print(json.dumps(hbm, indent=1))
print(json.dumps(sqs, indent=1))
