/*
 * oracle/gogoro_task.c -- CPU restatement of the reference Gogoro task path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP task
 * kernels in thormang_isaacgym_amd/csrc/gogoro_task.hip; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is
 * pinned against the golden fixtures generated from the reference's own task
 * module (tests/golden/make_golden.py, tests/test_golden_oracle.py).
 *
 * Plain C, scalar, fp32 arithmetic in the reference's operation order
 * (torch CPU semantics: non-fused multiply/add, floor-style remainder, round
 * half to even).  Each function cites the reference lines it restates
 * (paths relative to /root/reference/isaacgymenvs/).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/tg_gogoro.h"

#define F_PI 3.14159265358979323846f
#define F_2PI 6.28318530717958647692f

/* torch.remainder for floating types: fmod, then shift into the divisor's sign. */
static float t_rem(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
    return m;
}
static float t_clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* isaacgym.torch_utils.get_euler_xyz (roll, yaw only) -- used at tasks/gogoro_new.py:696 */
static void euler_roll_yaw(const float *q, float *roll, float *yaw) {
    float x = q[0], y = q[1], z = q[2], w = q[3];
    float sinr = 2.0f * (w * x + y * z);
    float cosr = w * w - x * x - y * y + z * z;
    float siny = 2.0f * (w * z + x * y);
    float cosy = w * w + x * x - y * y - z * z;
    *roll = t_rem(atan2f(sinr, cosr), F_2PI);
    *yaw = t_rem(atan2f(siny, cosy), F_2PI);
}

/* isaacgym.torch_utils.quat_rotate_inverse -- tasks/gogoro_new.py:698-699 */
static void quat_rot_inv(const float *q, const float *v, float *o) {
    float x = q[0], y = q[1], z = q[2], w = q[3];
    float s = 2.0f * (w * w) - 1.0f;
    float cx = y * v[2] - z * v[1], cy = z * v[0] - x * v[2], cz = x * v[1] - y * v[0];
    float d = x * v[0] + y * v[1] + z * v[2];
    o[0] = v[0] * s - cx * w * 2.0f + x * d * 2.0f;
    o[1] = v[1] * s - cy * w * 2.0f + y * d * 2.0f;
    o[2] = v[2] * s - cz * w * 2.0f + z * d * 2.0f;
}

/* compute_gogoro_observations -- tasks/gogoro_new.py:692-723 (+ shortest_angle_distance :687-689) */
void oracle_gogoro_observation(const float *root, float desired_yaw, float last_command, float *obs) {
    float roll, yaw, lin[3], ang[3];
    euler_roll_yaw(root + 3, &roll, &yaw);
    quat_rot_inv(root + 3, root + 7, lin);
    quat_rot_inv(root + 3, root + 10, ang);
    if (roll > F_PI) roll = roll - F_2PI;
    if (roll < -F_PI) roll = roll + F_2PI;
    if (yaw > F_PI) yaw = yaw - F_2PI;
    if (yaw < -F_PI) yaw = yaw + F_2PI;
    float dyaw = t_rem(desired_yaw - yaw + F_PI, F_2PI) - F_PI;
    obs[0] = roll;
    obs[1] = ang[0];
    obs[2] = ang[2];
    obs[3] = lin[0];
    obs[4] = dyaw;
    obs[5] = last_command;
}

void oracle_gogoro_observations(int n, const float *root, const float *yaw_cmd, const float *cmd, float *obs) {
    for (int e = 0; e < n; ++e) oracle_gogoro_observation(root + 13 * e, yaw_cmd[e], cmd[e], obs + 6 * e);
}

/* compute_gogoro_reward -- tasks/gogoro_new.py:645-684 */
void oracle_gogoro_reward_one(const float *o, int64_t progress, const float *ah, int64_t max_len, float *rew,
                              int64_t *reset) {
    const float max_tilt = 0.30f;
    float tilt_err = t_clamp(o[0] / max_tilt, -1.0f, 1.0f);
    float yaw_err = t_clamp(o[4] / F_PI, -1.0f, 1.0f);
    float dtilt_err = t_clamp(o[1] / 0.3f, -1.0f, 1.0f);
    float y30 = yaw_err * 30.0f;
    float r1 = 1.0f / (1.0f + y30 * y30);
    float r2 = 1.0f - tilt_err * tilt_err;
    float r4 = 1.0f - dtilt_err * dtilt_err;
    float ce = 0.0f;
    for (int k = 0; k < 5; ++k) ce += 1.0f - ah[k] * ah[k];
    float r = r1 * 5.0f + r2 * 0.2f + r4 * 0.3f + ce * 0.5f;
    int felt = fabsf(o[0]) >= max_tilt;
    int finished = progress >= max_len - 1;
    *reset = (finished || felt) ? 1 : 0;
    *rew = felt ? -100.0f : r;
}

void oracle_gogoro_reward(int n, const float *buffer_obs, const int64_t *progress, const float *ah, int64_t max_len,
                          float *rew, int64_t *reset) {
    for (int e = 0; e < n; ++e)
        oracle_gogoro_reward_one(buffer_obs + 6 * e, progress[e], ah + 5 * e, max_len, rew + e, reset + e);
}

/* Gogoro.pre_physics_step -- tasks/gogoro_new.py:347-369 (INCREMENTAL_STEER, :27: the
 * incremented command :351-354, or with p->absolute_steer the absolute one :355-356)
 * plus VecTask.step's action clamp (vec_task.py:327). */
void oracle_gogoro_pre_physics(const tg_gogoro_params *p, tg_gogoro_buffers *b, const float *actions,
                               const float *pre_draws) {
    const int D = p->num_dof;
    for (int e = 0; e < p->num_envs; ++e) {
        float a = t_clamp(actions[e], -p->clip_actions, p->clip_actions);
        float *ah = b->action_history + 5 * e;
        for (int k = 0; k < 4; ++k) ah[k] = ah[k + 1];
        ah[4] = a;
        float c;
        if (p->absolute_steer) {
            c = a * p->max_steering;
        } else {
            float da = t_clamp(a * p->max_steering_change, -p->max_steering_change, p->max_steering_change);
            c = b->curent_command[e] + da;
        }
        c = t_clamp(c, -p->max_steering, p->max_steering);
        b->curent_command[e] = c;
        float noise = p->steering_action_noise[0] + pre_draws[e] * p->steering_action_noise[1];
        for (int d = 0; d < D; ++d) {
            b->pos_target[e * D + d] = 0.0f;
            b->vel_target[e * D + d] = 0.0f;
        }
        b->pos_target[e * D + p->dof_steer] = c + b->steer_offsets[e] + noise;
        b->vel_target[e * D + p->dof_rear] = b->curent_speed[e];
    }
}

static float u_aff(float lo, float hi, float u) { return lo + u * (float)((double)hi - (double)lo); }
static float n_aff(const float *mc, float r) { return mc[0] + r * mc[1]; }

/* Gogoro.reset_idx for ONE env -- tasks/gogoro_new.py:505-591 with randomize :474-482,
 * generate_spawn_r :485-492, euler_to_quaternion :496-502, set_env_dof_prop :595-601.
 * r[11] are this env's draws in the order documented in tg_gogoro.h.  The
 * gravity/mass part of apply_randomizations (:476) is not a per-env draw and is
 * handled by the sim's domain-randomisation state. */
void oracle_gogoro_reset_env(const tg_gogoro_params *p, tg_gogoro_buffers *b, int e, const float *r) {
    const int D = p->num_dof;
    b->curent_speed[e] = u_aff(p->speed_range[0], p->speed_range[1], r[0]);
    b->steer_offsets[e] = n_aff(p->steering_offset, r[1]);
    b->speed_offset[e] = u_aff(p->speed_sensor_offset[0], p->speed_sensor_offset[1], r[2]);
    float target = (r[3] * 2.0f - 1.0f) * F_PI;
    float rot = target + u_aff(-1.57f, 1.57f, r[4]);
    float h = rot / 2.0f;
    float *root = b->root + 13 * e;
    memcpy(root, b->root_reset + 13 * e, 13 * sizeof(float));
    if (!p->terrain_spawn) root[2] = p->spawn_z;
    root[3] = 0.0f;
    root[4] = 0.0f;
    root[5] = sinf(h);
    root[6] = cosf(h);
    for (int k = 7; k < 13; ++k) root[k] = 0.0f;
    if (p->debug_start_speed) {   /* DEBUG_START_SPEED, gogoro_new.py:542-545 */
        root[7] = 1.3f * cosf(rot);
        root[8] = 1.3f * sinf(rot);
    }
    for (int d = 0; d < D; ++d) {
        b->dof_state[2 * (e * D + d)] = b->thormang_pose[d];
        b->dof_state[2 * (e * D + d) + 1] = 0.0f;
    }
    float *cv = b->config_vector + 5 * e;
    cv[0] = n_aff(p->seat_offset_x_range, r[5]);
    cv[1] = n_aff(p->seat_offset_y_range, r[6]);
    cv[2] = n_aff(p->seat_offset_z_range, r[7]);
    cv[3] = n_aff(p->seat_offset_xr_range, r[8]);
    cv[4] = n_aff(p->steering_offset, r[9]);
    const long ND = (long)p->num_envs * D;
    float *prop = b->dof_props + (long)e * D;
    const int seat[3] = {p->dof_base_x, p->dof_base_y, p->dof_base_z};
    for (int k = 0; k < 3; ++k) {
        prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
        prop[TG_PROP_LOWER * ND + seat[k]] = cv[k];
        prop[TG_PROP_UPPER * ND + seat[k]] = cv[k] + 0.0001f;
    }
    b->imu_offsets[e] = cv[3];
    b->steer_offsets[e] = cv[4];
    const int st = p->dof_steer;
    prop[TG_PROP_DRIVE_MODE * ND + st] = 1.0f;
    prop[TG_PROP_STIFFNESS * ND + st] = p->steer_stiffness;
    prop[TG_PROP_DAMPING * ND + st] = u_aff(p->steering_damping_range[0], p->steering_damping_range[1], r[10]);
    prop[TG_PROP_EFFORT * ND + st] = p->steer_effort;
    prop[TG_PROP_VELOCITY * ND + st] = p->steer_velocity;
    b->env_dirty[e] = 1;
    b->progress_buf[e] = 0;
    b->reset_buf[e] = 0;
    for (int k = 0; k < 6; ++k) {
        b->obs_buf[6 * e + k] = 0.0f;
        b->buffer_obs[6 * e + k] = 0.0f;
    }
    b->curent_command[e] = 0.0f;
    b->yaw_command[e] = target;
    for (int k = 0; k < 5; ++k) b->action_history[5 * e + k] = 0.0f;
}

/* Gogoro.post_physics_step (tasks/gogoro_new.py:373-390) + compute_obs_rwd (:424-462)
 * + VecTask.step tail (vec_task.py:345-353), env by env.  Resets are masked on
 * the reset_buf value left by the previous step; the debug-line block
 * (:392-420) has no effect on any buffer and is not restated. */
void oracle_gogoro_post_physics(const tg_gogoro_params *p, tg_gogoro_buffers *b, const float *reset_draws,
                                const float *obs_draws, const float *speed_draws, const float *yaw_draws) {
    for (int e = 0; e < p->num_envs; ++e) {
        b->progress_buf[e] += 1;
        if (b->reset_buf[e] != 0) oracle_gogoro_reset_env(p, b, e, reset_draws + TG_GOGORO_RESET_DRAWS * e);
        float o[6];
        oracle_gogoro_observation(b->root + 13 * e, b->yaw_command[e], b->curent_command[e], o);
        for (int k = 0; k < 6; ++k) b->buffer_obs[6 * e + k] = o[k];
        oracle_gogoro_reward_one(o, b->progress_buf[e], b->action_history + 5 * e, p->max_episode_length,
                                 b->rew_buf + e, b->reset_buf + e);
        const float *nd = obs_draws + 5 * e;
        float r[6];
        memcpy(r, o, sizeof r);
        r[0] += n_aff(p->imu_filter_noise, nd[0]) + b->imu_offsets[e];
        r[1] += n_aff(p->imu_noise, nd[1]);
        r[2] += n_aff(p->imu_noise, nd[2]);
        r[3] += n_aff(p->speed_sensor_noise, nd[3]);
        r[3] += b->speed_offset[e];
        r[3] = nearbyintf(r[4]);                      /* quirk: :457-458 */
        r[4] += n_aff(p->imu_filter_noise, nd[4]);
        for (int k = 0; k < 6; ++k) b->obs_buf[6 * e + k] = t_clamp(r[k], -p->clip_obs, p->clip_obs);
        if (b->progress_buf[e] == p->speed_freq_update)
            b->curent_speed[e] = u_aff(p->speed_range[0], p->speed_range[1], speed_draws[e]);
        float yc = b->yaw_command[e];
        if (b->progress_buf[e] == p->yaw_freq_update) yc = u_aff(-F_PI, F_PI, yaw_draws[e]);
        if (yc > F_PI) yc = yc - F_2PI;
        if (yc < -F_PI) yc = yc + F_2PI;
        b->yaw_command[e] = yc;
        b->timeout_buf[e] = (b->progress_buf[e] >= p->max_episode_length - 1) && (b->reset_buf[e] != 0);
    }
}
