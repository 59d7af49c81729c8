"""Benchmark: env-steps/sec of the batched UR3e gym step on MI355X.

Workload (BASELINE.json configs[3], per GPU): `assets/main.xml` (arm + 2F-85 +
mug, contacts on), gymnasium `ur3e-v2` step semantics (pid_task_ctrl + 2
physics substeps + obs/reward/termination + auto-reset at T=2500), uniformly
random task-space actions in the v2 action Box, 4096 envs per GPU.  One
"step" = one env-step of all resident envs = one ur3e_batch_step call: the
compact-tier kernel (w_env_step_q: a substep work queue, one wavefront per
env-substep, working set in LDS) plus the full-capacity fallback kernel over
the envs it queued.

Multi-GPU: one process per GPU, envs sharded by contiguous global id (weak
scaling: 4096 per GPU), per-step RCCL gather of (obs, reward, done) to rank 0
(the policy rank) as the north_star's C4 prescribes.  Under torchrun the ranks
come from its environment; `python bench.py --gpus N` without it starts the N
rank processes itself (`launch_workers`, before this process touches a GPU)
and fails when fewer than N GPUs are visible.

Model: `--model main_mesh` (the default) is main.xml with convex hulls for its
mesh geoms -- the reference's collision set (24 geoms, 234 candidate pairs);
`--model main` is the box surrogate, measured beside it in `other_configs`.

Prints ONE JSON line on rank 0 (see the contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
# algorithmic HBM bytes per env-step for main.xml (nq 21, nv 20, n_a 4, n_obs 24)
ALGO_BYTES_PER_ENV_STEP = 1898
# MI355X vector FP64 (AMD public spec): the path's real bound is FP64 latency at one
# wavefront per SIMD, so the algorithmic FP64 rate is reported beside the HBM roofline
FP64_VECTOR_PEAK_TFLOPS = 78.6


# the two compiles of the reference's assets/main.xml (ur3e_amd/model/compiler.py): its mesh files are
# git-ignored upstream: main_mesh (the headline) has SURVEY §2.3's collision set, with synthetic convex stand-in
# hulls for every mesh file (tools/make_main_meshes.py); main is the documented box surrogate
MODEL_VARIANT = {"main": "model variant: box surrogate for the mesh geoms (15 colliding geoms, 92 candidate pairs)",
                 "main_mesh": "model variant: convex stand-in hulls for the mesh geoms (24 colliding geoms, 17 meshes, "
                              "234 candidate pairs)"}


def shard_offset(rank: int, envs_per_gpu: int) -> int:
    """first global env id of a rank's shard (contiguous ranges, weak scaling)"""
    return rank * envs_per_gpu


def launch_mode(gpus: int, environ) -> str:
    """"rank": this process is one rank of a launched job (WORLD_SIZE set, by torchrun or launch_workers);
    "spawn": start `gpus` rank processes (launch_workers); "single": one GPU, this process."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if gpus != 1 and int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}")
        return "rank"
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    return "spawn" if gpus > 1 else "single"


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(n: int, argv, script: str | None = None, check_devices: bool = True, stdout=None,
                   timeout: float | None = None) -> int:
    """Start `n` rank processes of `script` (default: this file) with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set, one GPU each, and return the job's exit status (the first non-zero
    one; the other ranks are then terminated).  This process only counts the devices -- no HIP call --
    so the ranks start from a GPU-clean parent; more ranks than visible GPUs fail before any start."""
    import signal
    import subprocess
    if check_devices:
        import torch
        have = torch.cuda.device_count()  # counts devices without initialising one (no HIP context)
        if n > have:
            print(f"bench.py: --gpus {n} needs {n} GPUs, {have} visible", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv),
                                      env=env, stdout=stdout))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"bench.py: ranks still running after {timeout} s", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:  # only these exact children
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc < 0:  # a rank died of a signal: report it as the shell would
        rc = 128 - rc
    return rc


def _kinfo(batch, tier="step"):
    """kernel_info of one tier, or None when the handle does not launch that tier (e.g. a build without the mid
    tier)"""
    try:
        return batch.kernel_info(tier)
    except RuntimeError:
        return None


def _profile_file(kind: str):
    """profiles/<kind>_rNN.json of the newest round that has one (traffic: PMC HBM bytes per launch of
    the step kernel; flops: the oracle-counted FP64 flops per env-step), or None.  Each file records the
    commit it was measured at (`head`); the GPU box has no .git, so the newest round is the selector."""
    import re
    best, best_r = None, -1
    d = os.path.join(REPO, "profiles")
    for f in os.listdir(d) if os.path.isdir(d) else ():
        m = re.fullmatch(rf"{kind}_r(\d+)\.json", f)
        if m and int(m.group(1)) > best_r:
            best, best_r = os.path.join(d, f), int(m.group(1))
    return best


def _state_diff(gb, ob):
    """max |qpos - ref|, max |qvel - ref| and contact-count mismatches, GPU handle vs oracle batch"""
    qp, qv, _ = gb.get_state()
    oqp, oqv, _, onc = ob.get_state()
    ncon = gb.get_info()["ncon"].cpu().numpy()
    return dict(max_abs_qpos=float(np.abs(qp.cpu().numpy() - oqp).max()),
                max_abs_qvel=float(np.abs(qv.cpu().numpy() - oqv).max()),
                ncon_mismatch_envs=int((ncon != onc).sum()))


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _host_threads() -> int:
    """The CPU share of this process: OMP_NUM_THREADS when set (16 per GPU on the box), else the
    affinity mask (os.cpu_count() reports the whole machine there)."""
    if os.environ.get("OMP_NUM_THREADS"):
        return int(os.environ["OMP_NUM_THREADS"])
    return len(os.sched_getaffinity(0))


def _host_info() -> dict:
    """The machine the CPU baseline ran on: logical CPUs of the machine, of this process's affinity mask,
    and lscpu's model / socket / core / thread counts."""
    info = {"machine_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:  # the cgroup's CPU bandwidth limit (cgroup v2 cpu.max: "quota period" or "max period")
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpu_quota"] = "unavailable"
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        want = {"Model name": "lscpu_model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "CPU(s)": "lscpu_cpus"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in want:
                info[want[k.strip()]] = v.strip()
    except Exception as e:  # lscpu missing: the cpuinfo model is still reported
        info["lscpu"] = f"unavailable: {e}"
    return info


def _time_oracle(ob, actions_fn, steps):
    """seconds of oracle stepping over `steps` batches of actions_fn(i) (action generation untimed)"""
    dt = 0.0
    for i in range(steps):
        a = actions_fn(i)
        t0 = time.perf_counter()
        ob.step(a)
        dt += time.perf_counter() - t0
    return dt


def cpu_other_configs(L, threads, c2_envs=4096, c2_steps=200, c3_envs=1024, c3_rows=(1500, 1800)):
    """Oracle CPU figures for the other single-GPU configs, on `threads` host threads:
    C2 -- ur3e_2f85, random joint targets through move_j's PD (as other_configs);
    C3 -- main.xml move_l_mug scripted pick, the rows c3_rows of the grasp window (reached untimed), on
    both compiles of main.xml (the box surrogate and the convex hulls)."""
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.controller.move_l_mug import MoveLMug
    L.ur3o_set_threads(threads)
    out = {}
    md, mc = rt.load_model("ur3e_2f85")
    cfg = rt.make_config(task=rt.TASK_MOVE_J, frame_skip=1, model=md, seed=3, reset_noise=False,
                         reset_key=md["id_key_down"])
    ob = po.OracleBatch(mc, po.config_from(cfg), c2_envs, L=L)
    q0 = np.array(md["key_qpos"][md["id_key_down"]][:6])
    rng = np.random.default_rng(3)

    def act(_):
        a = np.empty((c2_envs, 7))
        a[:, :6] = q0 + rng.uniform(-0.5, 0.5, size=(c2_envs, 6))
        a[:, 6] = rng.uniform(0, 1, size=c2_envs)
        return a
    dt = _time_oracle(ob, act, c2_steps)
    out["C2_ur3e_2f85_move_j"] = {"value": c2_envs * c2_steps / dt, "unit": "env-steps/s", "cores": threads,
                                  "sample": f"{c2_envs} envs x {c2_steps} move_j env-steps, {dt:.1f} s"}
    for model in ("main", "main_mesh"):
        drv = MoveLMug(c3_envs, reset_mode="low", seed=0, model=model)  # trajectory rows only (GPU-evaluated)
        ob = po.OracleBatch(drv.batch.model_c, po.config_from(drv.batch.cfg), c3_envs, L=L)
        g0, g1 = c3_rows
        for t in range(g0):
            ob.step(drv.traj.row(t).cpu().numpy())
        rows = [drv.traj.row(t).cpu().numpy() for t in range(g0, g1)]
        dt = _time_oracle(ob, lambda i: rows[i], g1 - g0)
        drv.close()
        out[f"C3_{model}_move_l_mug"] = {
            "value": c3_envs * (g1 - g0) / dt, "unit": "env-steps/s", "cores": threads,
            "sample": f"{c3_envs} envs x rows {g0}-{g1} of the scripted pick (grasp window, reached untimed), "
                      f"{dt:.1f} s", "model": MODEL_VARIANT[model]}
    return out


def cpu_baseline(n_envs_sample=4096, steps=1000, seed=0, one_core_envs=256, one_core_steps=400,
                 all_cores_steps=100, model="main_mesh"):
    """The cpu_baseline leg.  The oracle (oracle/, the same algorithm in C) is compiled for this host
    (-O3 -march=native -ffp-contract=off, OpenMP over envs) and timed on a bounded sample of the bench
    workload: (1) this process's CPU share (OMP_NUM_THREADS, 16 per GPU on the box): n_envs_sample gym
    ur3e-v2 envs x `steps` env-steps; (2) every core of the affinity mask: n_envs_sample x all_cores_steps;
    (3) one thread: one_core_envs x one_core_steps; (4) C2 and C3 on the CPU share.  As the checker, the
    same seeded actions of (1) are replayed through a fresh GPU handle, giving the metric's second half,
    max |qpos - ref| after `steps` env-steps (the oracle is the reference here: MuJoCo is absent).
    `model`: the compile of main.xml the headline runs (main_mesh: convex hulls; main: box surrogate)."""
    import tempfile

    import torch
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    L = po.load_native(os.path.join(tempfile.gettempdir(), f"ur3e_oracle_native_{os.getpid()}"))
    threads = _host_threads()
    md, mc = rt.load_model(model)
    c = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, model=md, seed=seed)
    lo = np.array([0.04799994, -0.11650084, 0.0, 0.0])
    hi = np.array([0.54799994, 0.38349916, 0.5, 1.0])
    # (1) all threads, with the GPU replaying the same actions for the parity figure
    L.ur3o_set_threads(threads)
    ob = po.OracleBatch(mc, po.config_from(c), n_envs_sample, L=L)
    gb = rt.Batch(mc, c, n_envs_sample)
    rng = np.random.default_rng(seed)
    dt = 0.0
    for _ in range(steps):
        a = rng.uniform(lo, hi, size=(n_envs_sample, 4))
        t0 = time.perf_counter()
        ob.step(a)
        dt += time.perf_counter() - t0
        gb.step(torch.from_numpy(a))
    torch.cuda.synchronize()
    parity = dict(workload="gym ur3e-v2, uniform random actions", model=MODEL_VARIANT[model], envs=n_envs_sample,
                  steps=steps, **_state_diff(gb, ob))
    gb.close()
    # (2) one thread
    L.ur3o_set_threads(1)
    ob1 = po.OracleBatch(mc, po.config_from(c), one_core_envs, L=L)
    rng = np.random.default_rng(seed + 1)
    dt1 = 0.0
    for _ in range(one_core_steps):
        a = rng.uniform(lo, hi, size=(one_core_envs, 4))
        t0 = time.perf_counter()
        ob1.step(a)
        dt1 += time.perf_counter() - t0
    # (3) every core of the affinity mask (the machine's cores the process may run on)
    host = _host_info()
    n_all = min(host["affinity_cpus"], 512)  # threads count against the box's task limit
    quota = host.get("cgroup_cpu_quota")
    if isinstance(quota, float) and quota < n_all:
        # the cgroup's CPU bandwidth limit, not the affinity mask, is what the threads can use: more threads
        # than the quota only time-share it (round 4 measured 256 threads 28x slower than 16)
        n_all = max(int(quota), 1)
    all_cores = None
    capped = isinstance(quota, float) and quota < host["affinity_cpus"]
    if n_all != threads:
        L.ur3o_set_threads(n_all)
        oba = po.OracleBatch(mc, po.config_from(c), n_envs_sample, L=L)
        rng = np.random.default_rng(seed + 2)
        dta = _time_oracle(oba, lambda _: rng.uniform(lo, hi, size=(n_envs_sample, 4)), all_cores_steps)
        del oba
        all_cores = {"value": n_envs_sample * all_cores_steps / dta, "unit": "env-steps/s", "cores": n_all,
                     "sample": f"{n_envs_sample} envs x {all_cores_steps} env-steps from reset, OpenMP {n_all} "
                               f"threads (the affinity mask's CPUs"
                               + (f", capped at the cgroup's CPU quota {quota}" if capped else "")
                               + f"), {dta:.1f} s"}
    L.ur3o_set_threads(threads)
    try:
        others = cpu_other_configs(L, threads)
    except Exception as e:  # secondary figures never fail the baseline
        others = {"error": repr(e)}
    cpu = _cpu_model()
    build = "gcc -O3 -march=native -ffp-contract=off -fopenmp (compiled on this host)"
    base = dict(value=n_envs_sample * steps / dt, unit="env-steps/s", cores=threads, kind="port",
                sample=f"{n_envs_sample} envs x {steps} gym ur3e-v2 env-steps (main.xml, {MODEL_VARIANT[model]}; "
                       f"2 substeps) from reset, oracle/ C restatement, OpenMP {threads} threads (this process's "
                       f"CPU share), {dt:.1f} s",
                cpu_model=cpu, build=build, host=host,
                all_cores=all_cores,
                one_core={"value": one_core_envs * one_core_steps / dt1, "unit": "env-steps/s", "cores": 1,
                          "sample": f"{one_core_envs} envs x {one_core_steps} env-steps, 1 thread, {dt1:.1f} s"},
                other_configs=others)
    return base, parity


def other_configs(n_envs=4096, steps=50, warmup=5, pre_steps=500, headline_model="main_mesh"):
    """Throughput of the BASELINE configs other than the headline one, on one GPU (rank 0, N=1):
    the headline workload on the other compile of main.xml (the box surrogate beside the mesh headline);
    C2 -- ur3e_2f85, random joint targets through move_j's PD (one mj_step per control step);
    C3 -- main.xml move_l_mug scripted pick (pid_task_ctrl along build_traj_l_pick_place rows,
    one mj_step per row).  Timed with HIP events on the library's stream, inputs resident."""
    import torch
    from ur3e_amd import runtime as rt
    from ur3e_amd.controller.move_l_mug import MoveLMug
    out = {}
    md, mc = rt.load_model("ur3e_2f85")
    cfg = rt.make_config(task=rt.TASK_MOVE_J, frame_skip=1, model=md, seed=3, reset_noise=False,
                         reset_key=md["id_key_down"])
    b = rt.Batch(mc, cfg, n_envs)
    dev = b.obs.device
    q0 = torch.tensor(md["key_qpos"][md["id_key_down"]][:6], dtype=torch.float64, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(3)

    def act():
        a = torch.empty((n_envs, 7), dtype=torch.float64, device=dev)
        a[:, :6] = q0 + (torch.rand((n_envs, 6), dtype=torch.float64, device=dev, generator=g) - 0.5)
        a[:, 6] = torch.rand(n_envs, dtype=torch.float64, device=dev, generator=g)
        return a

    def timed(step_fn):
        for _ in range(warmup):
            step_fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            step_fn()
        e1.record()
        torch.cuda.synchronize()
        return n_envs * steps / (e0.elapsed_time(e1) * 1e-3)

    acts = [act() for _ in range(warmup + steps)]
    it = iter(acts)
    out["C2_ur3e_2f85_move_j"] = {"value": timed(lambda: b.step(next(it))), "unit": "env-steps/s",
                                  "envs": n_envs, "substeps_per_env_step": 1}
    b.close()
    # the headline workload on the other compile of main.xml: the box surrogate beside the convex-hull headline
    # (or the hulls -- the mesh-capable tier set, GJK/EPA in the wavefront -- beside a box-surrogate headline)
    other = "main" if headline_model == "main_mesh" else "main_mesh"
    md_m, mc_m = rt.load_model(other)
    cfg_m = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, max_episode_steps=2500, model=md_m, seed=1234)
    bm = rt.Batch(mc_m, cfg_m, n_envs)
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device=dev)
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device=dev)
    acts_m = lo + (hi - lo) * torch.rand((pre_steps + warmup + steps, n_envs, 4), dtype=torch.float64, device=dev,
                                         generator=g)
    for t in range(pre_steps):  # the headline's window (--pre-steps untimed env-steps since reset)
        bm.step(acts_m[t])
    tc0 = bm.tier_counts()
    it = iter(acts_m[pre_steps:])
    val = timed(lambda: bm.step(next(it)))
    tc = [x - y for x, y in zip(bm.tier_counts(), tc0)]
    tot = float(n_envs * (warmup + steps))
    out[f"{other}_gym_v2"] = {"value": val, "unit": "env-steps/s", "envs": n_envs, "substeps_per_env_step": 2,
                               "pre_steps_untimed": pre_steps,
                               "model": MODEL_VARIANT[other],
                               "kernel_resources": bm.kernel_info(),
                               "compact_bail_frac": tc[0] / tot, "full_tier_frac": tc[1] / tot,
                               "grasp_tier_routed_frac": tc[2] / tot}
    bm.close()
    # C3 is timed over the grasp: rows 1500-2600 of build_traj_l_pick_place (build_traj.py:28-59: the
    # descent to the mug ends at row 1800, the gripper closes and the lift starts), reached untimed
    drv = MoveLMug(n_envs, reset_mode="low", seed=0)
    g0, g1 = 1500, 2600
    for t in range(g0):
        drv.batch.step(drv.traj.row(t))
    rows = [drv.traj.row(t) for t in range(g0, g1)]
    tc0 = drv.batch.tier_counts()
    m0 = drv.batch.mid_count()
    it = iter(rows)
    steps_c3 = g1 - g0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps_c3):
        drv.batch.step(next(it))
    e1.record()
    torch.cuda.synchronize()
    tc = [x - y for x, y in zip(drv.batch.tier_counts(), tc0)]
    mid = drv.batch.mid_count() - m0
    tot = float(n_envs * steps_c3)
    out["C3_main_move_l_mug"] = {"value": n_envs * steps_c3 / (e0.elapsed_time(e1) * 1e-3), "unit": "env-steps/s",
                                 "envs": n_envs, "substeps_per_env_step": 1, "rows": [g0, g1],
                                 "mid_tier_routed_frac": mid / tot,
                                 # env-steps beyond the compact tier's capacity: routed to the grasp tier by
                                 # the previous step's contact count, or handed on mid-step (and beyond it)
                                 "grasp_tier_routed_frac": tc[2] / tot, "compact_bail_frac": tc[0] / tot,
                                 "full_tier_frac": tc[1] / tot}
    drv.close()
    # C3 as the reference's loop runs it (controller/move_l_mug.py:67-81): the same rows, and after every
    # mj_step traj_true[t] = get_task_space_state and actuator_frc[t] = get_jnt_torques recorded into
    # device buffers [rows, N, 7] (two small kernels per row on the same stream)
    from ur3e_amd.controller.move_l_mug import task_space_state
    drv = MoveLMug(n_envs, reset_mode="low", seed=0)
    for t in range(g0):
        drv.batch.step(drv.traj.row(t))
    it = iter(rows)
    tt = torch.empty((steps_c3, n_envs, 7), dtype=torch.float64, device=drv.batch.device)
    af = torch.empty((steps_c3, n_envs, drv.batch.nu), dtype=torch.float64, device=drv.batch.device)
    torch.cuda.synchronize()
    e0.record()
    for i in range(steps_c3):
        drv.batch.step(next(it))
        task_space_state(drv.batch, tt[i])
        drv.batch.get_actuator_force(af[i])
    e1.record()
    torch.cuda.synchronize()
    out["C3_main_move_l_mug_recording"] = {
        "value": n_envs * steps_c3 / (e0.elapsed_time(e1) * 1e-3), "unit": "env-steps/s", "envs": n_envs,
        "substeps_per_env_step": 1, "rows": [g0, g1],
        "records": "traj_true [rows, N, 7] and actuator_frc [rows, N, 7] every row, on the device",
        "grasp_rows_recorded_frac": float(tt[:, :, 6].mean().item())}
    drv.close()
    # C3 on main.xml with its convex meshes (the reference's collision set): the whole grasp and carry, tier
    # fractions included (the closed gripper's linkage meshes touch every carry row: EPA in the wavefront)
    out["C3_main_mesh_move_l_mug"] = c3_mesh(n_envs)
    try:
        out["C5_ppo_rollout"] = c5_ppo_rollout(n_envs)
    except Exception as e:  # secondary numbers never fail the headline line
        out["C5_ppo_rollout"] = {"error": repr(e)}
    return out


def c3_mesh(n_envs=4096, rows=(1500, 5000)):
    """C3 (move_l_mug scripted pick) on main.xml compiled with convex stand-in hulls for its mesh files: rows
    rows[0]..rows[1] (descent, grasp, lift and carry; the approach untimed), HIP events on the library
    stream, with the tier fractions (full_tier_frac: env-steps that needed the full-capacity tier)"""
    import torch
    from ur3e_amd.controller.move_l_mug import MoveLMug
    drv = MoveLMug(n_envs, reset_mode="low", seed=0, model="main_mesh")
    g0, g1 = rows
    for t in range(g0):
        drv.batch.step(drv.traj.row(t))
    rows_t = [drv.traj.row(t) for t in range(g0, g1)]
    tc0 = drv.batch.tier_counts()
    m0 = drv.batch.mid_count()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in rows_t:
        drv.batch.step(r)
    e1.record()
    torch.cuda.synchronize()
    tc = [x - y for x, y in zip(drv.batch.tier_counts(), tc0)]
    mid = drv.batch.mid_count() - m0
    tot = float(n_envs * (g1 - g0))
    res = {"value": tot / (e0.elapsed_time(e1) * 1e-3), "unit": "env-steps/s", "envs": n_envs,
           "substeps_per_env_step": 1, "rows": [g0, g1], "model": MODEL_VARIANT["main_mesh"],
           "kernel_resources": drv.batch.kernel_info(), "mid_kernel_resources": _kinfo(drv.batch, "mid"),
           "grasp_kernel_resources": _kinfo(drv.batch, "grasp"),
           "mid_tier_routed_frac": mid / tot,
           "grasp_tier_routed_frac": tc[2] / tot, "compact_bail_frac": tc[0] / tot, "full_tier_frac": tc[1] / tot,
           "tier_note": "routed env-steps run in the mid tier (16 contacts / 64 rows) when their last forward fits "
                        "it, else in the grasp tier; the mid tier's bails are counted again in the grasp fraction"}
    drv.close()
    return res



def c5_ppo_rollout(n_envs=4096, n_steps=16, iterations=3):
    """BASELINE config C5 on one GPU: SB3 PPO as gymnasium_src/scripts/regular_rl/rl/train_rl.py:38-90 runs it
    (config_rl.yml: n_steps 16, batch 256, 30 epochs, net_arch [256, 256]; VecNormalize(norm_obs, clip 10),
    train_rl.py:57), restated on the device (ur3e_amd/rl/ppo.py: SB3 is not installed): the UR3eVecEnv
    (this library) -> on-device VecNormalize -> the actor-critic's forward, no host round trip.  Reported:
    `value`, BASELINE's C5 metric -- wall-clock env-steps/s of whole PPO iterations (rollout plus update) --;
    the rollout's env-steps/s alone (env + normalisation + policy), the same env-steps through the env and
    VecNormalize alone with resident actions (the env's share), and the PPO update per iteration."""
    import torch
    from ur3e_amd.envs.vec_env import UR3eVecEnv
    from ur3e_amd.envs.vec_normalize import VecNormalize
    from ur3e_amd.rl.ppo import PPO
    venv = UR3eVecEnv(num_envs=n_envs, device=0, seed=0)
    env = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10.0)
    algo = PPO(env, n_steps=n_steps, batch_size=256, n_epochs=30, device="cuda:0", seed=0)
    algo.learn(1)  # warm-up: allocations, graph capture, first kernels
    times = algo.learn(iterations)
    roll = sum(t["rollout_s"] for t in times) / iterations
    train = sum(t["train_s"] for t in times) / iterations
    lo = torch.as_tensor(env.action_space.low, dtype=torch.float64, device="cuda")
    hi = torch.as_tensor(env.action_space.high, dtype=torch.float64, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    acts = lo + (hi - lo) * torch.rand((n_steps * iterations, n_envs, lo.numel()), dtype=torch.float64, device="cuda",
                                       generator=g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts:
        env.step_torch(a)
    torch.cuda.synchronize()
    env_s = (time.perf_counter() - t0) / iterations
    venv.close()
    k = n_steps * n_envs
    return {"value": k / (roll + train), "unit": "env-steps/s", "envs": n_envs,
            "what": "wall-clock PPO iterations: rollout (env + on-device VecNormalize + policy inference, "
                    "[256, 256] tanh MLP, f32) plus the PPO update (out of scope: DESIGN.md §8)",
            "rollout_env_steps_per_s": {"value": k / roll, "unit": "env-steps/s",
                                        "what": "the rollout alone: env + VecNormalize + policy inference"},
            "env_and_vecnormalize_only": {"value": k / env_s, "unit": "env-steps/s"},
            "policy_share_of_rollout": 1.0 - env_s / roll,
            "rollout_ms_per_env_step": 1e3 * roll / n_steps,
            "ppo_update_s_per_iteration": train,
            "iteration_env_steps_per_s": k / (roll + train),
            "config": {"n_steps": n_steps, "batch_size": 256, "n_epochs": 30, "iterations_timed": iterations,
                       "source": "ur3e_amd/rl/ppo.py (SB3 PPO restated; SB3 absent)"}}


def move_l_mug_parity(n_envs=512, steps=1000, seed=0, model="main_mesh"):
    """Checker for the north_star's parity clause: the move_l_mug scripted grasp (C3 semantics:
    pid_task_ctrl along per-env build_traj_l_pick_place rows, one mj_step per row, 'low' mug noise)
    for `steps` rows on the GPU and on the oracle; max |qpos - ref| and ncon mismatches at the end."""
    import torch
    from oracle import pyoracle as po
    from ur3e_amd.controller.move_l_mug import MoveLMug
    drv = MoveLMug(n_envs, reset_mode="low", seed=seed, model=model)
    gb = drv.batch
    ob = po.OracleBatch(gb.model_c, po.config_from(gb.cfg), n_envs)
    for _ in range(steps):
        row = drv.step()
        ob.step(row.cpu().numpy())
    torch.cuda.synchronize()
    out = dict(workload="move_l_mug scripted pick (main.xml, pid_task_ctrl, 1 substep)", model=MODEL_VARIANT[model],
               envs=n_envs,
               steps=steps, **_state_diff(gb, ob))
    drv.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--envs-per-block", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-envs", type=int, default=4096)
    ap.add_argument("--cpu-sample-steps", type=int, default=1000)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C2/C3 secondary throughput numbers")
    ap.add_argument("--queue-split", type=int, default=None,
                    help="A/B knob: percent of each unit queue's envs whose last substep runs as two half units "
                         "(default: the library's)")
    ap.add_argument("--pre-steps", type=int, default=500,
                    help="untimed env-steps after reset, so the timed window is mid-episode (contact regime)")
    ap.add_argument("--model", default="main_mesh", choices=["main", "main_mesh"],
                    help="main_mesh (the headline): main.xml with convex stand-in hulls for its mesh files (the "
                         "reference's collision set); main: main.xml's box-surrogate compile")
    ap.add_argument("--gather-self", action="store_true",
                    help="init RCCL and run the gather path even at one rank (exercises the overlap logic)")
    ap.add_argument("--env-priority", choices=["auto", "normal", "high"], default="auto",
                    help="priority of the stream the env steps run on; auto: high when the RCCL gather runs beside "
                         "them (its kernels then take the slots the env kernel's tail leaves), else normal")
    ap.add_argument("--launch-timeout", type=float, default=None,
                    help="--gpus N without torchrun: seconds before the rank processes are stopped")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="REHEARSAL ONLY (not a scaling number): let --gpus N ranks share the visible GPUs "
                         "(rank r on GPU r mod count) over gloo, without the RCCL gather -- exercises the launcher "
                         "and the multi-rank timing path on a box with fewer GPUs than ranks")
    args = ap.parse_args()
    if launch_mode(args.gpus, os.environ) == "spawn":
        # one process per GPU, started before anything here touches a GPU (this process only counts them)
        sys.exit(launch_workers(args.gpus, sys.argv[1:], timeout=args.launch_timeout,
                                check_devices=not args.rehearse_shared_gpu))
    if args.rehearse_shared_gpu:
        args.no_gather = True  # RCCL needs one GPU per rank; gloo has no device gather

    import torch
    import torch.distributed as dist
    from ur3e_amd import runtime as rt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_shared_gpu:
        local = local % max(torch.cuda.device_count(), 1)
    use_dist = world > 1 or args.gather_self
    if use_dist:
        torch.cuda.set_device(local)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # RCCL prints a version banner on stdout when the communicator comes up; keep stdout for
        # the one JSON line by pointing fd 1 at stderr until the first collective has run
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if args.rehearse_shared_gpu:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()
            torch.cuda.synchronize()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    n = args.envs_per_gpu
    md, mc = rt.load_model(args.model)
    cfg = rt.make_config(task=rt.TASK_GYM_V2, frame_skip=2, max_episode_steps=2500, model=md, seed=1234,
                         env_id_offset=shard_offset(rank, n), envs_per_block=args.envs_per_block)
    batch = rt.Batch(mc, cfg, n, device=local)
    if args.queue_split is not None:
        batch.set_queue_split(args.queue_split)
    batch_kinfo = batch.kernel_info()
    full_kinfo = _kinfo(batch, "full") or {}  # an untiered layout has no fallback tier
    lo = torch.tensor([0.04799994, -0.11650084, 0.0, 0.0], dtype=torch.float64, device=dev)
    hi = torch.tensor([0.54799994, 0.38349916, 0.5, 1.0], dtype=torch.float64, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)

    gather = use_dist and not args.no_gather
    if gather:
        # double-buffered payload: step t's gather runs on its own stream while step t+1 computes.  The env step
        # writes its outputs straight into the payload (obs [n, 24], reward [n], then terminated and truncated as
        # bytes), so one gather sends it whole with no packing kernels on the env stream; buffer k is rewritten
        # only after the gather that last read it (two steps earlier) has completed (its event)
        comm = torch.cuda.Stream(device=dev)
        od = batch.obs_dim
        plen = n * od + n + (2 * n + 7) // 8
        payloads = [torch.empty(plen, dtype=torch.float64, device=dev) for _ in range(2)]
        outs = []
        for p_ in payloads:
            fl = p_[n * od + n:].view(torch.uint8)
            outs.append((p_[:n * od].view(n, od), p_[n * od:n * od + n], fl[:n], fl[n:2 * n]))
        glists = [[torch.empty_like(payloads[0]) for _ in range(world)] if rank == 0 else None for _ in range(2)]
        gdone = [None, None]
        nstep = [0]

    env_priority = args.env_priority if args.env_priority != "auto" else ("high" if gather else "normal")
    if env_priority == "high":
        # the env steps on a high-priority stream: the dispatcher then places the env kernel's workgroups ahead
        # of the gather's, which runs in the slots the env kernel's tail frees
        torch.cuda.synchronize()
        lo_p, hi_p = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=min(lo_p, hi_p)))
    step_events = []
    # synthetic inputs are generated before the timed regions and stay resident in HBM (one [n, 4]
    # action batch per step); the timed loops run only the env step (and the gather)
    n_fresh = min(args.steps, args.pre_steps)

    def draw(k):
        return lo + (hi - lo) * torch.rand((k, n, 4), dtype=torch.float64, device=dev, generator=gen)

    def one_step(a, timed=False):
        if timed:  # HIP events on the stream the library launches on (torch's current stream)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if gather:
            k = nstep[0] & 1
            nstep[0] += 1
            if gdone[k] is not None:  # the gather that last read this buffer (two steps ago)
                torch.cuda.current_stream().wait_event(gdone[k])
            batch.step(a, out=outs[k])
        else:
            batch.step(a)
        if timed:
            e1.record()
            step_events.append((e0, e1))
        if gather:
            comm.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(comm):
                dist.gather(payloads[k], glists[k], dst=0)
                ev = torch.cuda.Event()
                ev.record()
            gdone[k] = ev

    # (1) fresh-reset window (secondary figure): the first n_fresh env-steps after reset, timed on the
    # stream; (2) the rest of the --pre-steps, untimed, so the headline window is mid-episode
    acts_fresh = draw(n_fresh)
    torch.cuda.synchronize()
    fe0, fe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fe0.record()
    for i in range(n_fresh):
        one_step(acts_fresh[i])
    fe1.record()
    for _ in range(args.pre_steps - n_fresh):
        one_step(draw(1)[0])
    torch.cuda.synchronize()
    fresh_ms = fe0.elapsed_time(fe1) / max(n_fresh, 1)
    del acts_fresh
    acts = draw(args.warmup + 2 * args.steps)
    for i in range(args.warmup):
        one_step(acts[i])
    ovf0 = batch.overflow_count()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        one_step(acts[args.warmup + i])
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    fallback = batch.overflow_count() - ovf0
    # the timed region carries no per-step events: each timing-event pair on the stream costs ~10 us of
    # GPU time per step (a marker's release between the launches, profiles/r05_l), 2 % of the step.  The
    # per-launch durations come from an instrumented window of as many steps right after it
    for i in range(args.steps):
        one_step(acts[args.warmup + args.steps + i], timed=True)
    torch.cuda.synchronize()
    step_kernel_ms_instr = sum(a.elapsed_time(b) for a, b in step_events) / len(step_events)
    gather_check = None
    if gather and rank == 0:
        # the last gathered payload's rank-0 slot is this rank's payload, bit for bit, and decodes to the step's
        # outputs (obs rows, reward, terminated / truncated bytes) -- the layout the policy rank reads
        torch.cuda.synchronize()
        kl = (nstep[0] - 1) & 1
        got = glists[kl][0]
        o_, r_, te_, tr_ = outs[kl]
        fl = got[n * od + n:].view(torch.uint8)
        gather_check = bool(torch.equal(got, payloads[kl]) and torch.equal(got[:n * od].view(n, od), o_)
                            and torch.equal(got[n * od:n * od + n], r_) and torch.equal(fl[:n], te_)
                            and torch.equal(fl[n:2 * n], tr_))
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    # per-step average over the timed region from the stream events (the step's launches and the gaps
    # between them): the dominant kernel's duration the roofline divides by (an upper bound on it)
    kernel_avg_ms = ev_ms / args.steps
    step_kernel_ms = kernel_avg_ms
    ms_per_step = wall * 1000.0 / args.steps
    total_env_steps = n * world * args.steps
    value = total_env_steps / wall

    if rank == 0:
        achieved = ALGO_BYTES_PER_ENV_STEP * n / (step_kernel_ms * 1e-3) / 1e9
        prof_traffic, traffic_src = None, None
        sfx = "" if args.model == "main" else "_mesh"   # profiles of the model variant that ran
        tf = _profile_file("traffic" + sfx)
        if tf:
            try:
                with open(tf) as f:
                    tj = json.load(f)
                prof_traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = {"file": os.path.relpath(tf, REPO), "pmc": tj.get("source"), "head": tj.get("head")}
            except Exception:
                prof_traffic = None
        fp64 = None
        ff = _profile_file("flops" + sfx)
        if ff:
            try:
                with open(ff) as f:
                    fj = json.load(f)
                fpe = fj["flops_per_env_step"]
                ach = fpe * n / (step_kernel_ms * 1e-3) / 1e12
                fp64 = {"bound": "fp64-vector", "achieved": ach, "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": ach / FP64_VECTOR_PEAK_TFLOPS, "flops_per_env_step": fpe,
                        "source": os.path.relpath(ff, REPO) + " (tools/count_flops.py: counting build of the oracle)",
                        "head": fj.get("head")}
            except Exception:
                fp64 = None
        cpu, parity = None, None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu, p_gym = cpu_baseline(args.cpu_sample_envs, args.cpu_sample_steps, model=args.model)
                parity = {"gym_v2": p_gym,
                          "move_l_mug": move_l_mug_parity(steps=args.cpu_sample_steps, model=args.model),
                          "reference": "oracle/ (CPU restatement; MuJoCo 3.3.3 absent: parity vs MuJoCo unpinned)",
                          "tolerance": 1e-5}
            except Exception as e:  # the oracle is only the checker; never fail the bench on it
                cpu = dict(value=None, unit="env-steps/s", cores=None, kind="port", sample=f"failed: {e}")
        extra = None
        if world == 1 and not args.no_extra:
            try:
                extra = other_configs(n_envs=n, pre_steps=args.pre_steps, headline_model=args.model)
            except Exception as e:  # secondary numbers never fail the headline line
                extra = {"error": repr(e)}
        line = {
            "metric": "env-steps/sec at N parallel envs, 1/2/4/8 MI355X; max |qpos-ref| @1k steps",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform random actions in the ur3e-v2 action Box, generated into HBM before the timed region; stochastic 'high' mug resets; timed window starts after --pre-steps untimed env-steps, mid-episode)",
            "config": {"workload": "main.xml gym ur3e-v2 step (pid_task_ctrl + 2 substeps + obs/reward/auto-reset), "
                                   + MODEL_VARIANT[args.model],
                       "envs_per_gpu": n, "global_envs": n * world, "frame_skip": 2,
                       "kernel_layout": {0: f"two-tier: compact 64-lane wavefront per env ({batch_kinfo.get('lds_bytes')} B lifetime-overlaid LDS working set,"
                                               f" {batch_kinfo.get('regs')} VGPRs: {batch_kinfo.get('envs_per_cu')} envs/CU)"
                                            " + full-capacity fallback; above the resident slot count the compact tier runs as a"
                                            " substep work queue", -128: "full-capacity, 128 lanes per env",
                                            -64: "full-capacity, 64 lanes per env"}.get(
                           batch.cfg.envs_per_block, f"v1 lane-per-env, {batch.cfg.envs_per_block} envs/wave"),
                       "kernel_resources": batch_kinfo,
                       "fallback_kernel_resources": full_kinfo,
                       "queue_split_percent": args.queue_split if args.queue_split is not None else "library default",
                       "env_stream_priority": env_priority,
                       "parallelism": f"env-shard{world}" + ("+rccl-gather" if gather else "")
                                      + (" (REHEARSAL: ranks share GPUs over gloo; not a scaling figure)"
                                         if args.rehearse_shared_gpu else "")},
            "fallback_env_steps_frac": fallback / float(n * args.steps),
            "gather": ({"payload_doubles_per_rank": plen, "layout": "obs [n, obs_dim] | reward [n] | terminated, "
                        "truncated bytes [2n], written by the env step in place", "rank0_slot_check": gather_check}
                       if gather else None),
            "window": {"pre_steps_untimed": args.pre_steps,
                       "timed_env_steps_since_reset": [args.pre_steps + args.warmup,
                                                       args.pre_steps + args.warmup + args.steps],
                       "fresh_reset": {"value": n * world / (fresh_ms * 1e-3), "unit": "env-steps/s",
                                       "env_steps_since_reset": [0, n_fresh],
                                       "note": "rank-0 stream time of the first env-steps after reset"}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": prof_traffic, "traffic_source": traffic_src,
                         "kernel": batch_kinfo["kernel"] + " + " + full_kinfo.get("kernel", "?") + " fallback",
                         "kernel_ms": step_kernel_ms,
                         "stream_avg_ms": kernel_avg_ms,
                         "kernel_ms_source": "HIP events around the timed region on the library's stream, per "
                                             "step (the step's launches and the gaps between them)",
                         "kernel_ms_note": "per-step stream time: an upper bound on the dominant kernel's launch "
                                           "duration, so `achieved` is a lower bound; kernel_ms_instrumented is "
                                           "the per-step event pair of a window right after (rounds 1-4 divided "
                                           "by that figure)",
                         "kernel_ms_instrumented": step_kernel_ms_instr,
                         "algo_bytes_per_env_step": ALGO_BYTES_PER_ENV_STEP,
                         "note": "path is FP64-latency-bound (SURVEY.md §8d); HBM fraction reported as required"},
            "roofline_fp64": fp64,
            "cpu_baseline": cpu,
            "parity": parity,
            "other_configs": extra,
        }
        print(json.dumps(line), flush=True)
    batch.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
