"""Diagnostic: the C5 env path without the policy -- UR3eVecEnv (4,096 envs) -> on-device VecNormalize, 64 steps
with resident random actions -- for a kernel trace (rocprofv3 --kernel-trace --stats) of where the time
beyond the env step goes.  usage: vecnorm_trace.py [n_envs] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ur3e_amd.envs.vec_env import UR3eVecEnv  # noqa: E402
from ur3e_amd.envs.vec_normalize import VecNormalize  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
venv = UR3eVecEnv(num_envs=n, device=0, seed=0)
env = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10.0)
env.reset_torch()
lo = torch.as_tensor(env.action_space.low, dtype=torch.float64, device="cuda")
hi = torch.as_tensor(env.action_space.high, dtype=torch.float64, device="cuda")
acts = lo + (hi - lo) * torch.rand((steps + 8, n, lo.numel()), dtype=torch.float64, device="cuda")
for a in acts[:8]:
    env.step_torch(a)
for label, fn in (("env+vecnorm", env.step_torch), ("env only", venv.step_torch)):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in acts[8:]:
        fn(a)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{label}: {1e3 * dt / steps:.3f} ms per step, {n * steps / dt / 1e6:.2f} M env-steps/s", flush=True)
venv.close()
