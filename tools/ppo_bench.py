"""BASELINE config C5: PPO (config_rl.yml hyper-parameters, ur3e_amd/rl/ppo.py) driving the batched
ur3e-v2 env on MI355X, obs normalised on device (VecNormalize(norm_obs=True, norm_reward=False,
clip_obs=10), train_rl.py:57), policy on torch-ROCm, no host round trip in the rollout.
One process per GPU under torchrun: each rank steps its own env shard; gradients are averaged with
one flattened RCCL all-reduce per minibatch.  Prints one JSON line (rank 0) with
  rollout env-steps/s  (env + normalisation + policy inference, all ranks),
  iteration env-steps/s (rollout + the PPO update, all ranks).
usage: python tools/ppo_bench.py [--envs-per-gpu 4096] [--n-steps 16] [--batch-size 256] [--n-epochs 30]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--n-steps", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--n-epochs", type=int, default=30)
    ap.add_argument("--iterations", type=int, default=2)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from ur3e_amd.envs.vec_env import UR3eVecEnv
    from ur3e_amd.envs.vec_normalize import VecNormalize
    from ur3e_amd.rl.ppo import PPO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    group = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        group = dist.group.WORLD
    n = a.envs_per_gpu
    venv = UR3eVecEnv(num_envs=n, device=local, seed=0, env_id_offset=rank * n)
    env = VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=10.0, group=group)
    algo = PPO(env, n_steps=a.n_steps, batch_size=a.batch_size, n_epochs=a.n_epochs, device=f"cuda:{local}",
               seed=rank, group=group)
    algo.learn(1)  # warm-up: allocations, first kernels
    if group is not None:
        dist.barrier()
    times = algo.learn(a.iterations)
    roll = max(t["rollout_s"] for t in times)
    it = max(t["rollout_s"] + t["train_s"] for t in times)
    if group is not None:
        v = torch.tensor([roll, it], device=f"cuda:{local}")
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        roll, it = v.tolist()
    steps = a.n_steps * n * world
    if rank == 0:
        print(json.dumps({
            "metric": "PPO env-steps/sec incl. policy (config C5)", "n_gpus": world,
            "rollout_env_steps_per_s": steps / roll, "iteration_env_steps_per_s": steps / it,
            "rollout_ms_per_env_step": 1e3 * roll / a.n_steps, "train_s_per_iteration": it - roll,
            "config": {"envs_per_gpu": n, "n_steps": a.n_steps, "batch_size": a.batch_size, "n_epochs": a.n_epochs,
                       "net_arch": [256, 256], "obs_norm": "on-device VecNormalize", "dtype": "env f64, policy f32"},
            "losses": algo.stats}), flush=True)
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
