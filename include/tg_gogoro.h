/*
 * tg_gogoro.h -- fused Gogoro task kernels behind the C-ABI of libtgsim.so.
 *
 * These replace the per-step Python/TorchScript task code of the reference
 * task ``isaacgymenvs/tasks/gogoro_new.py`` (registered as "Gogoro",
 * ``tasks/__init__.py:49,74``):
 *
 *   tg_gogoro_pre_physics   <- Gogoro.pre_physics_step      gogoro_new.py:347-369
 *   tg_gogoro_post_physics  <- Gogoro.post_physics_step     gogoro_new.py:373-420
 *                              + compute_obs_rwd            gogoro_new.py:424-462
 *                              + reset_idx / randomize      gogoro_new.py:474-591
 *                              + VecTask.step timeout/clamp vec_task.py:345-353
 *
 * Resets are MASKED (every env whose reset_buf != 0 resets itself inside the
 * kernel) instead of the reference's ``reset_buf.nonzero()`` + host loop, so
 * no device->host synchronisation happens on the step path.
 *
 * Random draws: every ``*_draws`` pointer is either NULL (the kernel draws
 * from its counter-based Philox4x32-10 stream keyed by (seed, env, counter))
 * or points to caller-supplied raw draws in the reference's order mapped to
 * envs (replay mode, used by the parity tests):
 *   pre_draws   [N]      N(0,1)  steering action noise       (gogoro_new.py:362)
 *   reset_draws [N,11]   speed U, steer-offset N, speed-offset U, target U,
 *                        spawn U, 5x config N, damping U   (:479-482,486-487,554-559,577)
 *   obs_draws   [N,5]    N(0,1) x5 sensor noises            (:451-460)
 *   speed_draws [N]      U speed resample                   (:386)
 *   yaw_draws   [N]      U yaw resample                     (:387)
 * All pointers are device pointers for the HIP entry points and host
 * pointers for the oracle (oracle/gogoro_task.c) which shares this layout.
 */
#ifndef TG_GOGORO_H
#define TG_GOGORO_H
#include <stdint.h>
#include "tgsim.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TG_GOGORO_NUM_OBS 6
#define TG_GOGORO_HIST 5
#define TG_GOGORO_RESET_DRAWS 11

/* cfg["noises"] and task constants (cfg/task/Gogoro.yaml:34-57; gogoro_new.py:84-87). */
typedef struct tg_gogoro_params {
    float max_steering;            /* 0.5 */
    float max_steering_change;     /* 0.2 */
    float steering_action_noise[2];
    float imu_filter_noise[2];
    float imu_noise[2];
    float speed_sensor_noise[2];
    float speed_range[2];
    float steering_offset[2];
    float speed_sensor_offset[2];
    float seat_offset_x_range[2];
    float seat_offset_y_range[2];
    float seat_offset_z_range[2];
    float seat_offset_xr_range[2];
    float steering_damping_range[2];
    float spawn_z;                 /* 0.03 (gogoro_new.py:537) */
    float steer_stiffness;         /* 3000 (:578) */
    float steer_effort;            /* 100  (:599) */
    float steer_velocity;          /* 200  (:600) */
    float clip_obs;                /* cfg env.clipObservations (inf) */
    float clip_actions;            /* cfg env.clipActions (inf) */
    int64_t max_episode_length;    /* cfg env.max_steps */
    int32_t speed_freq_update;
    int32_t yaw_freq_update;
    int32_t num_envs;
    int32_t num_dof;
    int32_t dof_steer, dof_rear, dof_base_x, dof_base_y, dof_base_z;
    int32_t terrain_spawn;         /* USE_TERAIN: reset z = root_reset[:,2], the per-env terrain
                                      height - 0.03 clamped to [0, 100] (gogoro_new.py:523-534) */
    int32_t absolute_steer;        /* INCREMENTAL_STEER = False (gogoro_new.py:27,353-356): the
                                      command is action * max_steering, not the incremented one
                                      (0, the registered module's value: incremental) */
    int32_t debug_start_speed;     /* DEBUG_START_SPEED (gogoro_new.py:25,542-545): a reset env
                                      starts at 1.3 m/s along its spawn heading (0: at rest) */
    uint64_t seed;                 /* Philox key for device draws */
} tg_gogoro_params;

/* Every buffer the task path touches.  Layouts are the reference's:
 * root [N,13] (pos, quat xyzw, linvel, angvel), dof_state [N*D,2],
 * targets [N,D], dof props [N,D], obs [N,6], counters int64. */
typedef struct tg_gogoro_buffers {
    /* VecTask buffers (vec_task.py:263-276) */
    float   *obs_buf;        /* [N,6]  policy observation (noisy, clamped) */
    float   *rew_buf;        /* [N]    */
    int64_t *reset_buf;      /* [N]    */
    int64_t *progress_buf;   /* [N]    */
    uint8_t *timeout_buf;    /* [N]    bool */
    /* Gogoro task state (gogoro_new.py:70-105) */
    float   *action_history; /* [N,5]  */
    float   *curent_command; /* [N]    */
    float   *yaw_command;    /* [N]    */
    float   *curent_speed;   /* [N]    */
    float   *steer_offsets;  /* [N]    */
    float   *imu_offsets;    /* [N]    */
    float   *speed_offset;   /* [N]    curent_speed_offset */
    float   *config_vector;  /* [N,5]  */
    float   *buffer_obs;     /* [N,1,6] clean observation history */
    const float *thormang_pose; /* [D] reset DOF pose (gogoro_new.py:234,262) */
    const float *root_reset;    /* [N,13] reset template root state (:144-145) */
    /* sim-owned state / inputs (the IsaacGym tensor API targets) */
    float   *root;           /* [N,13] */
    float   *dof_state;      /* [N*D,2] */
    float   *pos_target;     /* [N,D]  set_dof_position_target_tensor */
    float   *vel_target;     /* [N,D]  set_dof_velocity_target_tensor */
    float   *dof_props;      /* [TG_NUM_PROPS,N,D] per-env DOF properties (tgsim.h TG_PROP_*) */
    uint8_t *env_dirty;      /* [N] set when per-env props changed (sim recomposes) */
} tg_gogoro_buffers;

/* Gogoro.pre_physics_step (gogoro_new.py:347-369) + VecTask action clamp
 * (vec_task.py:327).  actions [N] (the [N,1] action tensor), pre_draws [N] or NULL. */
int tg_gogoro_pre_physics(tg_sim *sim, const tg_gogoro_params *p, const tg_gogoro_buffers *b,
                          const float *actions, const float *pre_draws, uint64_t counter);

/* Gogoro.post_physics_step + compute_obs_rwd + reset_idx (masked) + the
 * VecTask.step tail (gogoro_new.py:373-601, vec_task.py:345-353).  Draw
 * arrays as documented above, each NULL for in-kernel Philox draws. */
int tg_gogoro_post_physics(tg_sim *sim, const tg_gogoro_params *p, const tg_gogoro_buffers *b,
                           const float *reset_draws, const float *obs_draws, const float *speed_draws,
                           const float *yaw_draws, uint64_t counter);

/* One VecTask.step (vec_task.py:313-359): pre_physics_step + n_simulate x
 * simulate + post_physics_step -- the same operations as
 * tg_gogoro_pre_physics(pre_draws, counter_pre) + n_simulate x tg_simulate +
 * tg_gogoro_post_physics(reset/obs/speed/yaw draws, counter_post).  With
 * n_simulate == 1 the whole step is ONE launch of the step kernel: the
 * pre-physics runs at its start on each env's lead lane, the post-physics
 * (resets with in-place seat composites, observations, reward, noise,
 * command resample) as its epilogue on the final state.  With n_simulate > 1
 * the pre-physics rides in the first simulate's compose launch.  The draw
 * arrays (layouts above, NULL = in-kernel Philox) let the parity tests drive
 * this timed path with the reference's recorded torch.rand/randn stream;
 * speed_draws and yaw_draws go together. */
int tg_gogoro_step(tg_sim *sim, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const float *actions,
                   int32_t n_simulate, const float *pre_draws, const float *reset_draws, const float *obs_draws,
                   const float *speed_draws, const float *yaw_draws, uint64_t counter_pre, uint64_t counter_post);

/* Gogoro.reset_idx(env_ids) outside post_physics_step (gogoro_new.py:150,505-591;
 * VecTask.reset_done, vec_task.py:391-406): ids [n] int32 device, reset_draws
 * [N,11] (rows of the listed envs used) or NULL. */
int tg_gogoro_reset_idx(tg_sim *sim, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const int32_t *ids,
                        int32_t n, const float *reset_draws, uint64_t counter);

#ifdef __cplusplus
}
#endif
#endif
