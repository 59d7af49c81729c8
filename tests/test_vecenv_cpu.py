"""SB3 VecEnv semantics of UR3eVecEnv (auto-reset, terminal_observation,
TimeLimit.truncated, Monitor-style episode info), exercised on CPU with an
oracle-backed stepper (the GPU stepper is covered by tests/test_gpu_parity.py)."""
import numpy as np

from tests.helpers import OracleStepper
from ur3e_amd.envs.vec_env import UR3eVecEnv


def test_vecenv_autoreset_and_infos():
    n = 6
    env = UR3eVecEnv(num_envs=n, stepper=OracleStepper(n, seed=3, max_episode_steps=5))
    obs = env.reset()
    assert obs.shape == (n, 24)
    assert env.observation_space.shape == (24,)
    np.testing.assert_allclose(env.action_space.low, [0.04799994, -0.11650084, 0, 0])
    rng = np.random.default_rng(0)
    ends = 0
    for t in range(7):
        a = rng.uniform(env.action_space.low, env.action_space.high, size=(n, 4))
        obs, rew, dones, infos = env.step(a)
        assert obs.shape == (n, 24) and rew.shape == (n,) and dones.shape == (n,)
        for i in np.flatnonzero(dones):
            ends += 1
            assert infos[i]["terminal_observation"].shape == (24,)
            assert "TimeLimit.truncated" in infos[i]
            assert infos[i]["episode"]["l"] <= 5
    assert ends >= n  # every env hits the 5-step horizon at least once
    env.close()


def test_single_env_spaces_match_reference():
    from ur3e_amd.envs import UR3eEnv2
    e = UR3eEnv2()
    assert e.metadata["render_fps"] == 500
    assert e.observation_space.shape == (24,)
    np.testing.assert_allclose(e.action_space.high, [0.54799994, 0.38349916, 0.5, 1.0])


import pytest  # noqa: E402


@pytest.mark.parametrize("env_id,od,ad", [("gymnasium_env/ur3e-v0", 13, 4),
                                          ("gymnasium_env/imitation_indirect-v0", 24, 4),
                                          ("gymnasium_env/imitation_direct-v0", 13, 7)])
def test_vecenv_other_ids(env_id, od, ad):
    """The v0 / imitation ids: spaces from their reference classes, terminal observations of
    their own width, truncation tested before the increment (episodes of T+1 steps)."""
    n = 4
    T = 3
    env = UR3eVecEnv(num_envs=n, env_id=env_id,
                     stepper=OracleStepper(n, seed=1, max_episode_steps=T, env_id=env_id))
    assert env.observation_space.shape == (od,)
    assert env.action_space.shape == (ad,)
    obs = env.reset()
    assert obs.shape == (n, od)
    rng = np.random.default_rng(1)
    lens = []
    for _ in range(2 * (T + 1)):
        a = rng.uniform(env.action_space.low, env.action_space.high, size=(n, ad))
        obs, rew, dones, infos = env.step(a)
        assert obs.shape == (n, od)
        if env_id != "gymnasium_env/ur3e-v0":
            np.testing.assert_array_equal(rew, -1.0)
        for i in np.flatnonzero(dones):
            assert infos[i]["terminal_observation"].shape == (od,)
            lens.append(infos[i]["episode"]["l"])
    assert lens and max(lens) == T + 1
    env.close()


def test_register_ids_match_reference():
    from ur3e_amd import register_envs
    assert set(register_envs.IDS) == {"gymnasium_env/ur3e-v0", "gymnasium_env/imitation_indirect-v0",
                                      "gymnasium_env/imitation_direct-v0", "gymnasium_env/ur3e-v2"}
    for entry in register_envs.IDS.values():
        cls = register_envs._resolve(entry)
        assert cls.metadata["render_fps"] == 500


def test_vecenv_attr_methods():
    """SB3 VecEnv attribute API on the batched env: set_attr honours indices, get_attr returns
    per-env values, env_method answers render and refuses unknown methods."""
    n = 4
    env = UR3eVecEnv(num_envs=n, stepper=OracleStepper(n, seed=3, max_episode_steps=5))
    assert env.get_attr("render_mode") == [None] * n
    env.set_attr("tag", 7, indices=[1, 3])
    assert env.get_attr("tag") == [None, 7, None, 7]
    assert env.get_attr("tag", indices=1) == [7]
    assert env.env_method("render", indices=[0, 2]) == [None, None]
    with pytest.raises(AttributeError):
        env.env_method("no_such_method")
    with pytest.raises(AttributeError):
        env.get_attr("no_such_attr")
    env.close()
