/* On-device observation / reward normalisation for the batched env: the SB3 VecNormalize wrapper
 * the reference puts around its vector env (gymnasium_src/scripts/regular_rl/rl/train_rl.py:57,
 * `VecNormalize(venv, norm_obs=True, norm_reward=False, clip_obs=clip_obs)`), so obs never leave HBM
 * between the step kernel and a torch-ROCm policy.
 *
 * Semantics are those of the third-party stable_baselines3==2.7.0 (requirements.txt:100), which is
 * not vendored in the reference:
 *   - RunningMeanStd (common/running_mean_std.py): count starts at epsilon 1e-4, mean 0, var 1;
 *     update(arr) = update_from_moments(np.mean(arr, 0), np.var(arr, 0), arr.shape[0]);
 *   - VecNormalize.step_wait (vec_env/vec_normalize.py): obs_rms.update(obs) if training and
 *     norm_obs; obs -> clip((obs - mean) / sqrt(var + eps), +-clip_obs) cast to float32;
 *     if training: returns = returns * gamma + reward, ret_rms.update(returns); reward ->
 *     clip(reward / sqrt(ret_rms.var + eps), +-clip_reward) if norm_reward; terminal observations of
 *     done envs normalised like obs; returns[done] = 0;
 *   - VecNormalize.reset: returns = 0, obs_rms.update(obs) if training and norm_obs, normalise.
 * Every reduction follows numpy's order (axis-0 mean/var of [N, dim]: row-sequential per column;
 * 1-D mean/var of the returns: numpy's pairwise summation), so the statistics are bit-identical to
 * SB3 running on the same inputs.
 *
 * All pointers are device pointers on the current HIP device; work is enqueued on `stream`.
 */
#ifndef UR3E_VECNORM_H
#define UR3E_VECNORM_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  double* obs_mean;  /* [dim] */
  double* obs_var;   /* [dim] */
  double* obs_count; /* [1]   */
  double* ret_mean;  /* [1]   */
  double* ret_var;   /* [1]   */
  double* ret_count; /* [1]   */
  double* returns;   /* [n]   discounted return per env */
} ur3e_vecnorm_stats_t;

typedef struct {
  int training, norm_obs, norm_reward;
  double clip_obs, clip_reward, gamma, epsilon;
} ur3e_vecnorm_cfg_t;

/* replaces VecNormalize.step_wait on the batched step outputs.  d_obs [n, dim] f64, d_rew [n] f64,
   d_term / d_trunc [n] u8, d_tobs [n, dim] f64 (read for done envs only).  Outputs: d_obs_out
   [n, dim] f32 (norm_obs), d_rew_out [n] f64, d_tobs_out [n, dim] f32 (rows of done envs only). */
int ur3e_vecnorm_step(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                      const double* d_obs, const double* d_rew, const unsigned char* d_term,
                      const unsigned char* d_trunc, const double* d_tobs, float* d_obs_out, double* d_rew_out,
                      float* d_tobs_out, void* stream);

/* replaces VecNormalize.reset after the env reset: returns = 0, obs statistics update, normalise */
int ur3e_vecnorm_reset(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                       const double* d_obs, float* d_obs_out, void* stream);

/* replaces VecNormalize.normalize_obs (no statistics update): d_obs [n, dim] -> d_obs_out f32 */
int ur3e_vecnorm_normalize_obs(const ur3e_vecnorm_stats_t* st, const ur3e_vecnorm_cfg_t* cfg, int n, int dim,
                               const double* d_obs, float* d_obs_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
