"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: `make -C oracle asan`
builds a standalone driver of the oracle's batch step with -fsanitize=address,undefined
(-fno-sanitize-recover: any report aborts).  It runs the gym ur3e-v2 (with auto-resets), ur3e-v0,
scripted task-space, move_j and raw-control workloads, and its results must equal the normal build's
(pyoracle), so the sanitized run is the same computation.  CPU only."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "oracle", "_build", "ur3e_oracle_asan")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return EXE


def _actions(task, md, n, steps, rng):
    from ur3e_amd import runtime as rt
    if task in (rt.TASK_GYM_V2, rt.TASK_IMIT_INDIRECT):
        return rng.uniform([0.048, -0.1165, 0.0, 0.0], [0.548, 0.3835, 0.5, 1.0], size=(steps, n, 4))
    if task == rt.TASK_GYM_V0:
        return rng.uniform([0.288, 0.1335, 0.005, 0.0], [0.358, 0.3535, 0.165, 1.0], size=(steps, n, 4))
    if task == rt.TASK_TRAJ_L:  # task-space rows around the tcp at `down`, rotation held, grip closing
        a = np.zeros((steps, n, 7))
        a[..., 0:3] = [0.298, 0.1335, 0.17] + rng.normal(size=(steps, n, 3)) * 0.02
        a[..., 3:6] = [-1.209, -1.209, 1.209]
        a[..., 6] = rng.uniform(0, 1, size=(steps, n))
        return a
    if task == rt.TASK_MOVE_J:
        q0 = np.asarray(md["key_qpos"][md["id_key_down"]][:6]) if md.get("id_key_down", -1) >= 0 else np.zeros(6)
        a = np.zeros((steps, n, 7))
        a[..., :6] = q0 + rng.uniform(-0.5, 0.5, size=(steps, n, 6))
        a[..., 6] = rng.uniform(0, 1, size=(steps, n))
        return a
    return rng.uniform(-1, 1, size=(steps, n, md["nu"]))  # raw ctrl


CASES = [("main", 0, 2, 20), ("main", 4, 2, 20), ("main", 1, 1, 0), ("ur3e_2f85", 2, 1, 0), ("ur3e_raw", 3, 1, 0)]


@pytest.mark.parametrize("model,task,fs,T", CASES)
def test_oracle_under_asan_ubsan(exe, tmp_path, model, task, fs, T):
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    md, mc = rt.load_model(model)
    n, steps = 12, 30
    key = md["id_key_down"] if md.get("id_key_down", -1) >= 0 else -1
    cfg = rt.make_config(task=task, frame_skip=fs, max_episode_steps=T, model=md, seed=3, reset_key=key,
                         reset_noise=task in (0, 4))
    a = np.ascontiguousarray(_actions(task, md, n, steps, np.random.default_rng(task)))
    adim = a.shape[2]
    (tmp_path / "m.bin").write_bytes(bytes(mc))
    (tmp_path / "c.bin").write_bytes(bytes(cfg))
    a.tofile(tmp_path / "a.bin")
    out = tmp_path / "out.bin"
    r = subprocess.run([exe, str(tmp_path / "m.bin"), str(tmp_path / "c.bin"), str(tmp_path / "a.bin"), str(n),
                        str(steps), str(adim), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    rews = []
    for t in range(steps):
        rews.append(ob.step(a[t])[1])
    qp, qv, _, _ = ob.get_state()
    od = ob.od
    got = np.fromfile(out, dtype=np.float64)
    sizes = [n * od, n * mc.nq, n * mc.nv, steps * n]
    parts = np.split(got, np.cumsum(sizes)[:-1])
    assert len(got) == sum(sizes)
    assert np.array_equal(parts[0].reshape(n, od), ob.obs)
    assert np.array_equal(parts[1].reshape(n, mc.nq), qp)
    assert np.array_equal(parts[2].reshape(n, mc.nv), qv)
    assert np.array_equal(parts[3].reshape(steps, n), np.stack(rews))
