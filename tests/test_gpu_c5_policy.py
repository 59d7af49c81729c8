"""GPU: config C5's env path under policy-generated actions.  The on-device PPO driver
(ur3e_amd/rl/ppo.py, train_rl.py:60-73 restated) drives UR3eVecEnv through the on-device VecNormalize
for 4 rollouts x 50 steps at 1,024 envs, with policy updates between rollouts (so the action
distribution moves as training does).  Every raw action the env received and every raw output it
returned (obs, reward, terminated, truncated, terminal obs) is recorded; replaying the actions through
the CPU oracle from the same reset must reproduce the outputs bit for bit, auto-resets included."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _Recorder:
    """runtime.Batch with the stepper interface, copying every step's actions and outputs to the host"""

    def __init__(self, batch):
        self.b = batch
        self.device = batch.device
        self.obs_dim, self.act_dim = batch.obs_dim, batch.act_dim
        self.log = []
        self.obs0 = None

    def __getattr__(self, k):
        return getattr(self.b, k)

    def reset(self):
        o = self.b.reset()
        self.obs0 = o.cpu().numpy().copy()
        return o

    def step(self, actions):
        out = self.b.step(actions)
        self.log.append([actions.detach().cpu().numpy().copy()] + [x.cpu().numpy().copy() for x in out])
        return out


def test_ppo_actions_replay_bit_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import pyoracle as po
    from ur3e_amd import runtime as rt
    from ur3e_amd.envs.specs import spec
    from ur3e_amd.envs.vec_env import UR3eVecEnv
    from ur3e_amd.envs.vec_normalize import VecNormalize
    from ur3e_amd.rl.ppo import PPO
    n, T, iters = 1024, 50, 4
    s = spec("gymnasium_env/ur3e-v2")
    md, mc = rt.load_model("main")
    # a short horizon puts truncations (and their auto-resets) inside the 200 recorded steps
    cfg = rt.make_config(task=s["task"], frame_skip=s["frame_skip"], max_episode_steps=120, model=md, seed=17,
                         task_gains=s["gains"])
    rec = _Recorder(rt.Batch(mc, cfg, n))
    venv = UR3eVecEnv(num_envs=n, stepper=rec)
    env = VecNormalize(venv, norm_obs=True, norm_reward=True, clip_obs=10.0)
    algo = PPO(env, n_steps=T, batch_size=256, n_epochs=1, device="cuda:0", seed=3)
    algo.learn(iters)
    torch.cuda.synchronize()
    assert len(rec.log) == T * iters
    # the Batch resets at creation and VecNormalize.reset resets again (a second episode): so does the oracle
    ob = po.OracleBatch(mc, po.config_from(cfg), n)
    ob.reset_all()
    np.testing.assert_array_equal(rec.obs0, ob.obs)
    ends = 0
    acts = np.stack([r[0] for r in rec.log])
    assert acts.std(axis=(0, 1)).min() > 0  # the policy's actions, not a constant
    for t, (a, obs, rew, term, trunc, tobs) in enumerate(rec.log):
        o_obs, o_rew, o_term, o_trunc, o_tobs = ob.step(a)
        np.testing.assert_array_equal(obs, o_obs, err_msg=f"obs step {t}")
        np.testing.assert_array_equal(rew, o_rew, err_msg=f"reward step {t}")
        np.testing.assert_array_equal(term, o_term, err_msg=f"terminated step {t}")
        np.testing.assert_array_equal(trunc, o_trunc, err_msg=f"truncated step {t}")
        done = (o_term | o_trunc).astype(bool)
        np.testing.assert_array_equal(tobs[done], o_tobs[done], err_msg=f"terminal obs step {t}")
        ends += int(done.sum())
    assert ends >= n, ends  # every env passed through at least one auto-reset on average
    venv.close()
