/*
 * tg_walk.h -- fused kernels of the Thormang3 flat-ground walk task
 * ("ThormangWalk"), behind the C-ABI of libtgsim.so.
 *
 * The reference has NO Thormang walking task: its
 * humanoid tasks are tasks/humanoid.py (MJCF humanoid) and a stub
 * tasks/MA_OP3.py.  This task is designed here on the reference's patterns
 * and is therefore PARITY UNPINNED against the reference; the GPU kernels
 * are checked against their own CPU restatement (oracle/walk_task.c).
 *   actions -> PD position targets   : cfg/task/MA_OP3.yaml:36-41 (control.*),
 *                                      tasks/humanoid.py:281-285 (action scaling)
 *   observation / reward layout      : tasks/humanoid.py:379-417 pattern,
 *                                      MA_OP3.yaml:72-99 (learn.* scales)
 *   domain randomisation             : MA_OP3.yaml:149-171 (mass, friction),
 *                                      gogoro_realistic_turning_sim_paper.py:443-454 (pushes)
 *
 * Observation [N,112]: 0 pelvis height; 1-3 base linear velocity (body frame)
 * * lin_vel_scale; 4-6 base angular velocity (body frame) * ang_vel_scale;
 * 7-9 projected gravity (body frame, unit); 10-12 commands (vx, vy, wz) *
 * (lin, lin, ang) scales; 13-45 dof_pos - default; 46-78 dof_vel * dof_vel_scale;
 * 79-111 previous actions.
 *
 * Draws (replay mode, NULL -> in-kernel Philox):
 *   reset_draws [N, 4 + 2*D]: command vx U, vy U, wz U, spawn yaw U, D joint
 *                             noise U, D joint velocity noise U
 *   push_draws  [N, 3]      : push force x U, y U, z U
 */
#ifndef TG_WALK_H
#define TG_WALK_H
#include <stdint.h>
#include "tgsim.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TG_WALK_MAX_DOF 40
#define TG_WALK_NUM_OBS_BASE 13

typedef struct tg_walk_params {
    int32_t num_envs;
    int32_t num_dof;
    int32_t num_obs;              /* 13 + 3*num_dof */
    int32_t num_groups;           /* body_force row stride */
    float action_scale;           /* control.actionScale */
    float clip_actions, clip_obs;
    float lin_vel_scale, ang_vel_scale, dof_pos_scale, dof_vel_scale;
    float cmd_vx[2], cmd_vy[2], cmd_wz[2];
    float rew_lin_vel_xy, rew_ang_vel_z, rew_upright, rew_alive, rew_action_rate, rew_dof_vel, rew_torque,
        rew_termination, rew_height;
    float target_height;          /* pelvis height reward reference */
    float termination_height;     /* pelvis z below -> fall */
    float termination_up;         /* up-vector z below -> fall */
    float spawn_height;           /* pelvis z at reset */
    float joint_noise;            /* +-U reset joint offset (rad) */
    float push_force;             /* max |F| of a push (N), 0 disables */
    int32_t push_interval;        /* steps between pushes */
    int64_t max_episode_length;
    float dt;                     /* control dt (reward integration) */
    float default_pos[TG_WALK_MAX_DOF];
    float stiffness[TG_WALK_MAX_DOF];
    uint64_t seed;
} tg_walk_params;

typedef struct tg_walk_buffers {
    float *obs_buf;               /* [N,num_obs] */
    float *rew_buf;               /* [N] */
    int64_t *reset_buf;           /* [N] */
    int64_t *progress_buf;        /* [N] */
    uint8_t *timeout_buf;         /* [N] */
    float *actions;               /* [N,D] current (clamped) actions */
    float *last_actions;          /* [N,D] */
    float *commands;              /* [N,3] vx, vy, wz */
    const float *root_reset;      /* [N,13] reset template (env origin) */
    float *root;                  /* [N,13] sim state */
    float *dof_state;             /* [N*D,2] */
    float *pos_target;            /* [N,D] */
    float *body_force;            /* [N,G,6] push wrench (group 0), or NULL */
    uint8_t *env_dirty;           /* [N] */
} tg_walk_buffers;

/* actions [N,D] -> clamp -> PD position targets default + scale*a */
int tg_walk_pre_physics(tg_sim *sim, const tg_walk_params *p, const tg_walk_buffers *b, const float *actions);
/* One VecTask.step of the task (tasks/base/vec_task.py:313-359 with
 * pre_physics_step, control_freq_inv = n_simulate simulate calls and
 * post_physics_step): the same results as tg_walk_pre_physics +
 * [tg_apply_body_forces(body_force) when b->body_force] + n_simulate x
 * tg_simulate + tg_walk_post_physics, with the pre-physics work fused into the
 * first simulate's compose launch (one launch fewer per step). */
int tg_walk_step(tg_sim *sim, const tg_walk_params *p, const tg_walk_buffers *b, const float *actions,
                 int32_t n_simulate, const float *reset_draws, const float *push_draws, uint64_t counter);
/* progress, masked resets, observation, reward, termination, timeouts, pushes */
int tg_walk_post_physics(tg_sim *sim, const tg_walk_params *p, const tg_walk_buffers *b, const float *reset_draws,
                         const float *push_draws, uint64_t counter);
/* reset_idx(env_ids) outside the step (initial reset, VecTask.reset_done) */
int tg_walk_reset_idx(tg_sim *sim, const tg_walk_params *p, const tg_walk_buffers *b, const int32_t *ids, int32_t n,
                      const float *reset_draws, uint64_t counter);

#ifdef __cplusplus
}
#endif
#endif
