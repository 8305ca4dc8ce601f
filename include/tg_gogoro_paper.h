/*
 * tg_gogoro_paper.h -- fused task kernels for the Gogoro "paper" variant,
 * isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py (unregistered in the
 * reference's task map; cfg/task/Gogoro_paper.yaml).  SURVEY.md §8 f1.
 *
 * Replaces, per VecTask.step (vec_task.py:313-359):
 *   tg_paper_pre_physics   pre_physics_step          paper.py:349-393
 *                          (command clamp/scale, 5-slot command history and
 *                          the steering delay, wheel speed target)
 *   tg_paper_post_physics  post_physics_step         paper.py:397-482
 *                          + compute_obs_rwd         paper.py:491-547
 *                          + compute_gogoro_observations :771-808
 *                          + compute_gogoro_reward   paper.py:714-762
 *                          (20-step clean / noisy observation histories,
 *                          masked reset_idx :609-692, speed / yaw command
 *                          changes, head pushes :442-459), then VecTask's
 *                          time_outs (vec_task.py:345)
 *   tg_paper_reset_idx     reset_idx for explicit env ids
 *   tg_paper_step          the whole VecTask.step (GogoroPaper.step): the
 *                          pre-physics as the first simulate's compose
 *                          prologue, n_simulate simulates, the post-physics;
 *                          the same results as the three calls above
 *
 * The module's debug switches (paper.py:23-34) are parameters with the
 * committed values as defaults: DEBUGFIXBASE (a sim parameter, fix_base),
 * DEBUG_START_SPEED, RANDOM_DAMPING, PUSH_ROBOT, CENTER_ROBOT, USE_STEER_DELAY.
 *
 * Random draws.  NULL draw arrays -> in-kernel Philox4x32-10 keyed by (seed,
 * env, call counter, slot).  Replay arrays reproduce the reference's
 * torch.rand sequence (thormang_isaacgym_amd/tasks/paper_draws.py):
 *   reset_draws [N, 9]: speed, delay, steer_offset, speed_offset, imu_x_offset,
 *                       steering damping, seat x, seat y, seat z
 *   noise_draws [N, 6]: imu filter (roll, yaw), imu (droll, dyaw), speed noise,
 *                       delta-yaw filter
 *   speed_draws [N], yaw_draws [N], push_draws [N, 2] (x, z)
 * All are U[0,1) values; the kernels apply the reference's affine maps.
 */
#ifndef TG_GOGORO_PAPER_H
#define TG_GOGORO_PAPER_H

#include <stdint.h>

#include "tgsim.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TG_PAPER_HIST 20     /* buff_size, paper.py:103 */
#define TG_PAPER_OBS 8       /* num_obs, paper.py:100 */
#define TG_PAPER_CMD_HIST 5  /* command_history width = command_delay[1] (Gogoro_paper.yaml:49) */

typedef struct tg_paper_params {
    int32_t num_envs, num_dof, num_groups;
    int32_t dof_steer, dof_rear, dof_base_x, dof_base_y, dof_base_z;
    int64_t max_episode_length;                 /* env.max_steps */
    int32_t speed_freq_update, yaw_freq_update; /* noises.*_freq_update */
    float command_delay[2];                     /* noises.command_delay */
    float imu_filter_noise[2], imu_noise[2], speed_sensor_noise[2], speed_sensor_offset[2], imu_x_offset[2];
    float speed_range[2], steering_offset[2], steering_damping_range[2];
    float seat_offset_x_range[2], seat_offset_y_range[2], seat_offset_z_range[2];
    float max_steering;      /* 0.5  paper.py:81 */
    float max_tilt;          /* 0.38 paper.py:726 */
    float spawn_z;           /* 0.03 paper.py:629 */
    float start_speed;       /* 1.3  paper.py:652 */
    float push_force;        /* 30   paper.py:444 */
    int32_t push_interval;   /* 10   paper.py:443 */
    int32_t push_max_envs;   /* 2048 paper.py:443 (progress_buf[:2048]) */
    int32_t use_steer_delay, random_damping, center_robot, push_robot, debug_start_speed;
    float damping_stiffness; /* 13700, set_env_dof_prop call paper.py:668 */
    float damping_effort, damping_velocity;   /* 200, 1.0  paper.py:697-698 */
    float head_com[3];       /* head_p_link COM in the root-group frame */
    float group0_com[3];     /* root-group COM in its frame (wrench reference point) */
    int32_t perturbation_stride; /* floats between two envs' rows of b->perturbation (0: 3); the task
                                    points it at head_p_link's row of its [N, L, 3] perturbation tensor */
    uint64_t seed;
} tg_paper_params;

typedef struct tg_paper_buffers {
    float *obs_buf;            /* [N, 160] */
    float *buffer_obs;         /* [N, 20, 8] clean */
    float *buffer_obs_noisy;   /* [N, 20, 8] */
    float *rew_buf;            /* [N] */
    int64_t *reset_buf;        /* [N] */
    int64_t *progress_buf;     /* [N] */
    uint8_t *timeout_buf;      /* [N] */
    float *curent_command;     /* [N] */
    float *command_history;    /* [N, 5] */
    int64_t *steer_delay;      /* [N] */
    float *steer_offsets, *curent_speed, *curent_speed_offset, *curent_imu_x_offset, *curent_damping_cfg;
    float *yaw_command;        /* [N] */
    float *speed_no_noise;     /* [N] */
    float *perturbation;       /* [N, 3] world force on head_p_link (row stride p->perturbation_stride) */
    float *root_reset;         /* [N, 13] */
    const float *thormang_pose;/* [N, D] */
    float *root;               /* [N, 13] sim root state */
    float *dof_state;          /* [N*D, 2] */
    float *pos_target, *vel_target;  /* [N, D] */
    float *dof_props;          /* [TG_NUM_PROPS, N, D] */
    float *body_force;         /* [N, G, 6] or NULL (pushes off) */
    uint8_t *env_dirty;        /* [N] */
    float *scratch;            /* [N] per-env partial sums (reward term 7) */
    /* [N*L, 3] world-frame per-link forces or NULL: tg_paper_step applies them
     * to the next simulate exactly as tg_apply_rigid_body_force_tensors(sim,
     * rb_forces, NULL, TG_ENV_SPACE) right after the call would (the post_physics
     * pushes write head_p_link's rows first, paper.py:449-457), reduced to the
     * group wrenches inside the step's post-physics; the separate-call API
     * ignores it */
    const float *rb_forces;
} tg_paper_buffers;

typedef struct tg_sim tg_sim;

int tg_paper_pre_physics(tg_sim *sim, const tg_paper_params *p, const tg_paper_buffers *b, const float *actions,
                         uint64_t counter);
int tg_paper_post_physics(tg_sim *sim, const tg_paper_params *p, const tg_paper_buffers *b, const float *reset_draws,
                          const float *noise_draws, const float *speed_draws, const float *yaw_draws,
                          const float *push_draws, uint64_t counter);
int tg_paper_reset_idx(tg_sim *sim, const tg_paper_params *p, const tg_paper_buffers *b, const int32_t *ids,
                       int32_t n, const float *reset_draws, uint64_t counter);
/* pre_physics_step + n_simulate x simulate + post_physics_step with in-kernel
 * draws (counter: the post-physics call's).  With n_simulate == 1, a compiled
 * model with in-place seat composites, flat ground and a batch of at most one
 * step-kernel workgroup (16 envs) per CU, the whole step is ONE kernel launch:
 * the post-physics runs as the step kernel's epilogue and reward term 7's
 * batch sum is exchanged between the launch's workgroups (a workgroup that
 * never became resident makes tg_sync report TG_ERR_STATE).  Otherwise, or
 * with TG_PAPER_TWO_LAUNCH=1 in the environment at tg_sim creation: the step
 * kernel (pre-physics inside) and one post launch.  The one-launch form
 * passes each launch its own arrival target: do not capture it into a HIP
 * graph for replay (set TG_PAPER_TWO_LAUNCH=1 for that). */
int tg_paper_step(tg_sim *sim, const tg_paper_params *p, const tg_paper_buffers *b, const float *actions,
                  int32_t n_simulate, uint64_t counter);

#ifdef __cplusplus
}
#endif
#endif
