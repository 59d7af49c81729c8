"""The reference's SB3 scripts drop in unchanged (north_star; SURVEY.md §7.3 H6 option a).

A synthetic script with train_rl.py's import order -- SB3 names bound first
(gymnasium_src/scripts/regular_rl/rl/train_rl.py:5-7), then `import register_envs`
(:9), then make_vec_env(..., env_kwargs={"render_mode": "human"}, vec_env_cls=
SubprocVecEnv) (:38-44) and VecNormalize(venv, ...) (:57) -- runs in a fresh
interpreter with this repository on the path and minimal stand-ins for the SB3
modules (SB3 is not installed in this image).  Without any edit to the script it
must get the batched UR3eVecEnv (stepping, 24-d obs, 4-d actions), the dispatching
VecNormalize, and unchanged SB3 behaviour for ids that are not gymnasium_env/*.

CPU: the stepper is swapped for the oracle-backed test stepper by a test-only
bootstrap (runpy); GPU: the same script runs on the real Batch and VecNormalize.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SB3_STUBS = {
    "stable_baselines3/__init__.py": "class PPO:\n    pass\n",
    "stable_baselines3/common/__init__.py": "",
    "stable_baselines3/common/env_util.py": textwrap.dedent("""
        def make_vec_env(env_id, n_envs=1, **kwargs):
            if str(env_id).startswith("gymnasium_env/"):
                raise RuntimeError("SB3 make_vec_env reached: would fork SubprocVecEnv workers")
            return ("sb3-make_vec_env", env_id, n_envs)
    """),
    "stable_baselines3/common/vec_env/__init__.py": textwrap.dedent("""
        from .base_vec_env import VecEnv
        class SubprocVecEnv:
            pass
        class VecNormalize:
            def __init__(self, venv, **kwargs):
                self.venv = venv
                self.sb3 = True
            @classmethod
            def load(cls, path, venv):
                return cls(venv)
    """),
    "stable_baselines3/common/vec_env/base_vec_env.py": "class VecEnv:\n    pass\n",
}

# the reference script's shape, written for this test (train_rl.py:1-9, 38-44, 57)
SCRIPT = textwrap.dedent("""
    import json
    import os
    import numpy as np
    import yaml
    from stable_baselines3 import PPO
    from stable_baselines3.common.env_util import make_vec_env
    from stable_baselines3.common.vec_env import SubprocVecEnv, VecNormalize
    import register_envs

    visualize = True
    n_envs = 5
    venv = make_vec_env(env_id="gymnasium_env/ur3e-v2", n_envs=n_envs,
                        env_kwargs={"render_mode": "human" if visualize else "rgb_array"},
                        vec_env_cls=SubprocVecEnv)
    out = {"venv": type(venv).__name__, "num_envs": venv.num_envs,
           "obs_shape": list(venv.observation_space.shape), "act_shape": list(venv.action_space.shape),
           "vec_env_base": [c.__name__ for c in type(venv).__mro__],
           "VecNormalize": type(VecNormalize).__name__}
    obs0 = venv.reset()
    rng = np.random.default_rng(0)
    ends = 0
    for _ in range(6):
        a = rng.uniform(venv.action_space.low, venv.action_space.high, size=(n_envs, 4))
        obs, rew, dones, infos = venv.step(a)
        ends += int(dones.sum())
    out.update(obs=list(obs.shape), rew=list(rew.shape), ends=ends)
    if os.environ.get("DROPIN_GPU"):
        # train_rl.py:20 names the statistics file; :46-57 resume or start; :90 saves
        save_dir = "policies/rl_policies"
        os.makedirs(save_dir, exist_ok=True)
        vecnormalize_fpath = f"{save_dir}/rl_vecnormalize_l.pkl"
        resume_training = bool(os.environ.get("DROPIN_RESUME"))
        if resume_training and os.path.exists(vecnormalize_fpath):
            vn = VecNormalize.load(vecnormalize_fpath, venv)
        else:
            vn = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10)
        out["rms_loaded"] = [float(vn.obs_rms.count)] + [float(x) for x in vn.obs_rms.mean]
        o = vn.reset()
        o, r, d, i = vn.step(np.tile(venv.action_space.low, (n_envs, 1)))
        out.update(vecnormalize=type(vn).__module__, vn_obs_dtype=str(o.dtype))
        vn.save(vecnormalize_fpath)
        out["saved_files"] = sorted(os.listdir(save_dir))
        out["rms_saved"] = [float(vn.obs_rms.count)] + [float(x) for x in vn.obs_rms.mean]
    out["other_id"] = list(make_vec_env("CartPole-v1", n_envs=2))
    print("RESULT " + json.dumps(out))
""")

# test-only bootstrap: the GPU stepper -> the oracle-backed stepper, then run the script as __main__
BOOT_CPU = textwrap.dedent("""
    import runpy, sys
    sys.path.insert(0, {repo!r})
    import ur3e_amd.envs.vec_env as ve
    from tests.helpers import OracleStepper
    ve._default_stepper = lambda env_id, n, device, seed, off, epb, T, cfg_yaml=None: OracleStepper(
        n, seed=seed, env_id_offset=off, max_episode_steps=3 if T is None else T, env_id=env_id)
    runpy.run_path({script!r}, run_name="__main__")
""")


def _run(tmp_path, gpu: bool, resume: bool = False):
    for rel, txt in SB3_STUBS.items():
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(txt)
    script = tmp_path / "train_rl_like.py"
    script.write_text(SCRIPT)
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([str(tmp_path), REPO])
    if gpu:
        env["DROPIN_GPU"] = "1"
        if resume:
            env["DROPIN_RESUME"] = "1"
        cmd = [sys.executable, str(script)]
    else:
        boot = tmp_path / "boot.py"
        boot.write_text(BOOT_CPU.format(repo=REPO, script=str(script)))
        cmd = [sys.executable, str(boot)]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def _check(out):
    assert out["venv"] == "UR3eVecEnv"
    assert "VecEnv" in out["vec_env_base"]  # subclasses SB3's VecEnv when SB3 is importable
    assert out["num_envs"] == 5 and out["obs_shape"] == [24] and out["act_shape"] == [4]
    assert out["obs"] == [5, 24] and out["rew"] == [5]
    assert out["VecNormalize"] == "_DispatchVecNormalize"
    assert out["other_id"] == ["sb3-make_vec_env", "CartPole-v1", 2]  # other ids reach SB3 unchanged


def test_train_rl_script_drops_in_cpu(tmp_path):
    out = _run(tmp_path, gpu=False)
    _check(out)
    assert out["ends"] >= 5  # the test stepper's 3-step horizon auto-resets every env


@pytest.mark.gpu
def test_train_rl_script_drops_in_gpu(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _run(tmp_path, gpu=True)
    _check(out)
    assert out["vecnormalize"] == "ur3e_amd.envs.vec_normalize" and out["vn_obs_dtype"] == "float32"
    # train_rl.py:90 saves to exactly the .pkl name, and the resume branch (:46-49) loads it back
    assert out["saved_files"] == ["rl_vecnormalize_l.pkl"]
    out2 = _run(tmp_path, gpu=True, resume=True)
    _check(out2)
    assert out2["rms_loaded"] == out["rms_saved"]
    assert out2["rms_saved"][0] > out["rms_saved"][0]  # the resumed run kept counting


def test_vecnormalize_stats_file_exact_path(tmp_path):
    """save() writes exactly the path it is given (np.savez would append .npz to '...pkl'); load reads it,
    a file left at path + '.npz' by an older build is still found, anything else is refused."""
    import numpy as np
    from ur3e_amd.envs.vec_normalize import STATS_KEYS, read_stats, write_stats
    arrays = {k: np.arange(3, dtype=np.float64) + i for i, k in enumerate(STATS_KEYS)}
    p = tmp_path / "rl_vecnormalize_l.pkl"
    write_stats(str(p), **arrays)
    assert sorted(os.listdir(tmp_path)) == ["rl_vecnormalize_l.pkl"]
    back = read_stats(str(p))
    assert all(np.array_equal(back[k], arrays[k]) for k in STATS_KEYS)
    old = tmp_path / "old.pkl"
    np.savez(str(old), **arrays)  # the old save(): lands at old.pkl.npz
    assert np.array_equal(read_stats(str(old))["cfg"], arrays["cfg"])
    bad = tmp_path / "sb3.pkl"
    bad.write_bytes(b"\x80\x04not a zip")
    with pytest.raises(ValueError):
        read_stats(str(bad))
    with pytest.raises(FileNotFoundError):
        read_stats(str(tmp_path / "missing.pkl"))


def test_install_drop_in_namespace():
    from ur3e_amd import register_envs as re_

    def sb3_make(env_id, n_envs=1, **kw):
        return ("sb3", env_id)

    class SB3VN:
        pass

    ns = {"make_vec_env": sb3_make, "VecNormalize": SB3VN}
    assert re_.install_drop_in(ns) == {"make_vec_env": True, "VecNormalize": True}
    assert ns["make_vec_env"]("Pendulum-v1") == ("sb3", "Pendulum-v1")
    assert re_.install_drop_in(ns) == {}  # idempotent
    with pytest.raises(NotImplementedError):
        ns["make_vec_env"]("gymnasium_env/ur3e-v2", n_envs=2, wrapper_class=object)
