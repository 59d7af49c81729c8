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
