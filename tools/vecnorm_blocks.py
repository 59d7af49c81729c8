"""Diagnostic: the VecNormalize statistics kernel's two halves timed apart (HIP events over 64 calls at
4,096 envs x 24 obs): both blocks (norm_obs, training), the returns block alone (norm_obs off), neither
(training off: the apply kernel only)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd.envs.vec_env import UR3eVecEnv  # noqa: E402
from ur3e_amd.envs.vec_normalize import VecNormalize  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
venv = UR3eVecEnv(num_envs=n, device=0, seed=0)
env = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10.0)
env.reset_torch()
a = torch.as_tensor(env.action_space.low, dtype=torch.float64, device="cuda").expand(n, -1).contiguous()
obs, rew, term, trunc, tobs = venv.step_torch(a)
for label, no, tr in (("obs + returns", True, True), ("returns only", False, True), ("apply only", True, False)):
    env.norm_obs, env.training = no, tr
    for _ in range(4):
        env._kernel_step(n, obs, rew, term, trunc, tobs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(64):
        env._kernel_step(n, obs, rew, term, trunc, tobs)
    e1.record()
    torch.cuda.synchronize()
    print(f"{label}: {1e3 * e0.elapsed_time(e1) / 64:.1f} us per call", flush=True)
venv.close()
