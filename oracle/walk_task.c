/*
 * oracle/walk_task.c -- CPU restatement of the ThormangWalk task kernels
 * (thormang_isaacgym_amd/csrc/walk_task.hip).  TEST INFRASTRUCTURE ONLY.
 *
 * PARITY UNPINNED against the reference: the reference contains no Thormang
 * walking task.  The task is the build's own design
 * on the reference's patterns (include/tg_walk.h cites them); this file is
 * the independent checker of its GPU implementation, written as plain scalar
 * C over the same buffer layouts.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/tg_walk.h"

#define W_PI 3.14159265358979323846f

static float clampf_(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

void oracle_walk_pre_physics(const tg_walk_params *p, tg_walk_buffers *b, const float *actions) {
    const int D = p->num_dof;
    for (int e = 0; e < p->num_envs; ++e)
        for (int d = 0; d < D; ++d) {
            float a = clampf_(actions[e * D + d], -p->clip_actions, p->clip_actions);
            b->actions[e * D + d] = a;
            b->pos_target[e * D + d] = p->default_pos[d] + p->action_scale * a;
        }
}

void oracle_walk_reset_env(const tg_walk_params *p, tg_walk_buffers *b, int e, const float *r) {
    const int D = p->num_dof;
    b->commands[3 * e + 0] = p->cmd_vx[0] + r[0] * (p->cmd_vx[1] - p->cmd_vx[0]);
    b->commands[3 * e + 1] = p->cmd_vy[0] + r[1] * (p->cmd_vy[1] - p->cmd_vy[0]);
    b->commands[3 * e + 2] = p->cmd_wz[0] + r[2] * (p->cmd_wz[1] - p->cmd_wz[0]);
    float yaw = (r[3] * 2.0f - 1.0f) * W_PI;
    float *root = b->root + 13 * e;
    const float *tpl = b->root_reset + 13 * e;
    root[0] = tpl[0];
    root[1] = tpl[1];
    root[2] = p->spawn_height;
    root[3] = 0.0f;
    root[4] = 0.0f;
    root[5] = sinf(0.5f * yaw);
    root[6] = cosf(0.5f * yaw);
    for (int k = 7; k < 13; ++k) root[k] = 0.0f;
    for (int d = 0; d < D; ++d) {
        b->dof_state[2 * (e * D + d)] = p->default_pos[d] + (r[4 + d] * 2.0f - 1.0f) * p->joint_noise;
        b->dof_state[2 * (e * D + d) + 1] = 0.1f * (r[4 + D + d] * 2.0f - 1.0f);
        b->last_actions[e * D + d] = 0.0f;
        b->actions[e * D + d] = 0.0f;
    }
    b->progress_buf[e] = 0;
    b->reset_buf[e] = 0;
}

/* observation + reward + termination for one env (state already post-physics / post-reset) */
static void observe(const tg_walk_params *p, tg_walk_buffers *b, int e, int64_t prog) {
    const int D = p->num_dof;
    const float *r = b->root + 13 * e;
    float x = r[3], y = r[4], z = r[5], w = r[6];
    float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                  2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                  2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
    float vb[3], wb[3], gb[3];
    for (int i = 0; i < 3; ++i) {
        vb[i] = R[i] * r[7] + R[3 + i] * r[8] + R[6 + i] * r[9];
        wb[i] = R[i] * r[10] + R[3 + i] * r[11] + R[6 + i] * r[12];
        gb[i] = -R[6 + i];
    }
    float *o = b->obs_buf + (long)p->num_obs * e;
    const float *cmd = b->commands + 3 * e;
    o[0] = r[2];
    for (int i = 0; i < 3; ++i) {
        o[1 + i] = vb[i] * p->lin_vel_scale;
        o[4 + i] = wb[i] * p->ang_vel_scale;
        o[7 + i] = gb[i];
    }
    o[10] = cmd[0] * p->lin_vel_scale;
    o[11] = cmd[1] * p->lin_vel_scale;
    o[12] = cmd[2] * p->ang_vel_scale;
    float rate = 0.0f, vel2 = 0.0f, tq = 0.0f;
    for (int d = 0; d < D; ++d) {
        float q = b->dof_state[2 * (e * D + d)], qd = b->dof_state[2 * (e * D + d) + 1];
        float a = b->actions[e * D + d], la = b->last_actions[e * D + d];
        o[13 + d] = (q - p->default_pos[d]) * p->dof_pos_scale;
        o[13 + D + d] = qd * p->dof_vel_scale;
        o[13 + 2 * D + d] = a;
        rate += (a - la) * (a - la);
        vel2 += qd * qd;
        float t = p->stiffness[d] * (b->pos_target[e * D + d] - q);
        tq += t * t;
        b->last_actions[e * D + d] = a;
    }
    for (int k = 0; k < p->num_obs; ++k) o[k] = clampf_(o[k], -p->clip_obs, p->clip_obs);
    float lin_err = (cmd[0] - vb[0]) * (cmd[0] - vb[0]) + (cmd[1] - vb[1]) * (cmd[1] - vb[1]);
    float ang_err = (cmd[2] - wb[2]) * (cmd[2] - wb[2]);
    float dz = r[2] - p->target_height;
    float rew = p->rew_lin_vel_xy * expf(-lin_err / 0.25f) + p->rew_ang_vel_z * expf(-ang_err / 0.25f) +
                p->rew_upright * (-gb[2]) + p->rew_alive + p->rew_height * expf(-dz * dz / 0.01f) +
                p->rew_action_rate * rate + p->rew_dof_vel * vel2 + p->rew_torque * tq;
    int fall = (r[2] < p->termination_height) || (-gb[2] < p->termination_up);
    if (fall) rew += p->rew_termination;
    int64_t reset = (fall || prog >= p->max_episode_length - 1) ? 1 : 0;
    b->rew_buf[e] = rew;
    b->reset_buf[e] = reset;
    b->timeout_buf[e] = (prog >= p->max_episode_length - 1) && reset;
}

void oracle_walk_post_physics(const tg_walk_params *p, tg_walk_buffers *b, const float *reset_draws,
                              const float *push_draws) {
    const int D = p->num_dof;
    for (int e = 0; e < p->num_envs; ++e) {
        int64_t prog = b->progress_buf[e] + 1;
        b->progress_buf[e] = prog;
        if (b->reset_buf[e] != 0) {
            oracle_walk_reset_env(p, b, e, reset_draws + (long)(4 + 2 * D) * e);
            prog = 0;
        }
        observe(p, b, e, prog);
        if (b->body_force) {
            float *f = b->body_force + (long)6 * p->num_groups * e;
            int push = p->push_force > 0.0f && p->push_interval > 0 && prog > 0 && (prog % p->push_interval) == 0;
            const float *u = push_draws + 3 * e;
            f[0] = push ? p->push_force * (u[0] * 2.0f - 1.0f) : 0.0f;
            f[1] = push ? p->push_force * (u[1] * 2.0f - 1.0f) : 0.0f;
            f[2] = push ? 0.25f * p->push_force * (u[2] * 2.0f - 1.0f) : 0.0f;
            f[3] = f[4] = f[5] = 0.0f;
        }
    }
}
