/*
 * oracle/gogoro_paper_task.c -- CPU restatement of the Gogoro "paper" variant
 * task path (isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP kernels in
 * thormang_isaacgym_amd/csrc/gogoro_paper_task.hip, pinned against the golden
 * fixtures recorded from the reference module itself
 * (tests/golden/make_golden_paper.py, tests/test_golden_paper.py).
 *
 * Scalar fp32 in the reference's operation order (torch CPU semantics).
 * Line numbers refer to gogoro_realistic_turning_sim_paper.py unless noted.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/tg_gogoro_paper.h"

#define F_PI 3.14159265358979323846f
#define F_2PI 6.28318530717958647692f
#define H TG_PAPER_HIST
#define O TG_PAPER_OBS
#define CH TG_PAPER_CMD_HIST

static float t_rem(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
    return m;
}
static float t_clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
/* get_randoms(shape, bounds) = bounds[0] + rand * (bounds[1] - bounds[0]) (:555-556) */
static float u_aff(const float *b, float u) { return b[0] + u * (float)((double)b[1] - (double)b[0]); }

static void quat_rot_inv(const float *q, const float *v, float *o) {
    float x = q[0], y = q[1], z = q[2], w = q[3];
    float s = 2.0f * (w * w) - 1.0f;
    float cx = y * v[2] - z * v[1], cy = z * v[0] - x * v[2], cz = x * v[1] - y * v[0];
    float d = x * v[0] + y * v[1] + z * v[2];
    o[0] = v[0] * s - cx * w * 2.0f + x * d * 2.0f;
    o[1] = v[1] * s - cy * w * 2.0f + y * d * 2.0f;
    o[2] = v[2] * s - cz * w * 2.0f + z * d * 2.0f;
}

/* compute_gogoro_observations (:771-808) with shortest_angle_distance (:766-767) */
void oracle_paper_observation(const float *root, float desired_yaw, float command, float delay_norm, float *obs) {
    const float *q = root + 3;
    float x = q[0], y = q[1], z = q[2], w = q[3];
    float roll = t_rem(atan2f(2.0f * (w * x + y * z), w * w - x * x - y * y + z * z), F_2PI);
    float yaw = t_rem(atan2f(2.0f * (w * z + x * y), w * w + x * x - y * y - z * z), F_2PI);
    float lin[3], ang[3];
    quat_rot_inv(q, root + 7, lin);
    quat_rot_inv(q, root + 10, ang);
    if (roll > F_PI) roll = roll - F_2PI;
    if (roll < -F_PI) roll = roll + F_2PI;
    if (yaw > F_PI) yaw = yaw - F_2PI;
    if (yaw < -F_PI) yaw = yaw + F_2PI;
    obs[0] = roll;
    obs[1] = yaw;
    obs[2] = ang[0];
    obs[3] = ang[2];
    obs[4] = lin[0];
    obs[5] = t_rem(desired_yaw - yaw + F_PI, F_2PI) - F_PI;
    obs[6] = command;
    obs[7] = delay_norm;
}

/* compute_gogoro_reward (:714-762) for one env; r7 = 1 - mean(diff(act/0.5)^2)
 * over the whole batch (torch.mean without dim, :740) is passed in. */
static void reward_one(const float *bo, int64_t progress, int64_t max_len, float max_tilt, float r7, float *rew,
                       int64_t *reset) {
    const float *last = bo + (H - 1) * O;
    float tilt = last[0], dtilt = last[2], yaw_err = last[5];
    float act = last[6] / 0.5f;
    float tilt_err = t_clamp(tilt / max_tilt, -1.0f, 1.0f);
    yaw_err = t_clamp(yaw_err / F_PI, -1.0f, 1.0f);
    float dtilt_err = t_clamp(dtilt / 0.3f, -1.0f, 1.0f);
    float r1 = 1.0f - yaw_err * yaw_err;
    float r2 = 1.0f - tilt_err * tilt_err;
    float r4 = 1.0f - dtilt_err * dtilt_err;
    float tilt_w = 1.0f - tanhf(50.0f * (tilt_err * tilt_err));
    float dtilt_w = 1.0f - tanhf(50.0f * (dtilt_err * dtilt_err));
    float r5 = 1.0f - (act * act) * (tilt_w * dtilt_w);
    float r = r1 * 0.45f + r2 * 0.1f + r4 * 0.35f + r5 * 2.0f + r7 * 0.2f;
    int finished = progress >= max_len - 1;
    int felt = fabsf(tilt) >= max_tilt;
    r = r < 0.0f ? 0.0f : r;
    *rew = felt ? -1.0f : r;
    *reset = (finished || felt) ? 1 : 0;
}

/* sum over envs of sum_t (a[t+1]-a[t])^2 with a = act/0.5 (double accumulation:
 * the product kernels and torch only agree to rounding here) */
static double act_diff_sq(const float *bo) {
    double s = 0.0;
    for (int t = 0; t + 1 < H; ++t) {
        float d = bo[(t + 1) * O + 6] / 0.5f - bo[t * O + 6] / 0.5f;
        s += (double)(d * d);
    }
    return s;
}

/* pre_physics_step (:349-393) */
void oracle_paper_pre_physics(const tg_paper_params *p, tg_paper_buffers *b, const float *actions) {
    int D = p->num_dof;
    for (int e = 0; e < p->num_envs; ++e) {
        float a = t_clamp(actions[e], -1.0f, 1.0f);
        float cmd = a * p->max_steering;
        b->curent_command[e] = cmd;
        float *h = b->command_history + CH * e;
        for (int k = 0; k < CH - 1; ++k) h[k] = h[k + 1];
        h[CH - 1] = cmd;
        int idx;
        if (p->use_steer_delay) {
            int64_t d = b->steer_delay[e];   /* command_history[:, -steer_delay]; -0 selects slot 0 */
            idx = d == 0 ? 0 : (int)(CH - d);
        } else {
            idx = CH - 3;
        }
        float *pt = b->pos_target + (size_t)D * e, *vt = b->vel_target + (size_t)D * e;
        for (int d = 0; d < D; ++d) { pt[d] = 0.0f; vt[d] = 0.0f; }
        pt[p->dof_steer] = h[idx];
        vt[p->dof_rear] = b->curent_speed[e];
    }
}

/* reset_idx for one env (:609-692) with its draws r[9] (randomize :565-575 then the per-id loop) */
void oracle_paper_reset_env(const tg_paper_params *p, tg_paper_buffers *b, int e, const float *r) {
    int D = p->num_dof;
    size_t ND = (size_t)p->num_envs * D;
    b->curent_speed[e] = u_aff(p->speed_range, r[0]);
    b->steer_delay[e] = (int64_t)u_aff(p->command_delay, r[1]);
    b->steer_offsets[e] = u_aff(p->steering_offset, r[2]);
    float *pz = b->perturbation + (size_t)(p->perturbation_stride ? p->perturbation_stride : 3) * e;
    pz[0] = pz[1] = pz[2] = 0.0f;
    b->curent_speed_offset[e] = u_aff(p->speed_sensor_offset, r[3]);
    float *root = b->root + 13 * (size_t)e;
    const float *tpl = b->root_reset + 13 * (size_t)e;
    memcpy(root, tpl, 13 * sizeof(float));
    root[2] = p->spawn_z;
    root[3] = 0.0f; root[4] = 0.0f; root[5] = 0.0f; root[6] = 1.0f;   /* euler_to_quaternion(0, 0, 0) */
    for (int k = 7; k < 13; ++k) root[k] = 0.0f;
    if (p->debug_start_speed) {
        root[7] = p->start_speed * cosf(0.0f);
        root[8] = p->start_speed * sinf(0.0f);
    }
    float *dof = b->dof_state + 2 * (size_t)e * D;
    for (int d = 0; d < D; ++d) {
        dof[2 * d] = b->thormang_pose[(size_t)e * D + d];
        dof[2 * d + 1] = 0.0f;
    }
    b->curent_imu_x_offset[e] = u_aff(p->imu_x_offset, r[4]);
    float *prop = b->dof_props + (size_t)e * D;
    if (p->random_damping) {   /* set_env_dof_prop(id, damping, 13700, "steering_joint") :694-699 */
        float damp = u_aff(p->steering_damping_range, r[5]);
        b->curent_damping_cfg[e] = damp;
        int st = p->dof_steer;
        prop[TG_PROP_DRIVE_MODE * ND + st] = (float)TG_DOF_MODE_POS;
        prop[TG_PROP_STIFFNESS * ND + st] = p->damping_stiffness;
        prop[TG_PROP_DAMPING * ND + st] = damp;
        prop[TG_PROP_EFFORT * ND + st] = p->damping_effort;
        prop[TG_PROP_VELOCITY * ND + st] = p->damping_velocity;
        b->env_dirty[e] = 1;
    }
    if (!p->center_robot) {    /* seat offsets :673-682 */
        const int seat[3] = {p->dof_base_x, p->dof_base_y, p->dof_base_z};
        const float *rg[3] = {p->seat_offset_x_range, p->seat_offset_y_range, p->seat_offset_z_range};
        for (int k = 0; k < 3; ++k) {
            float lo = u_aff(rg[k], r[6 + k]);
            prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
            prop[TG_PROP_LOWER * ND + seat[k]] = lo;
            prop[TG_PROP_UPPER * ND + seat[k]] = (float)((double)lo + 0.0001);
        }
        b->env_dirty[e] = 1;
    }
    b->progress_buf[e] = 0;
    b->reset_buf[e] = 0;
    memset(b->obs_buf + (size_t)H * O * e, 0, H * O * sizeof(float));
    memset(b->buffer_obs + (size_t)H * O * e, 0, H * O * sizeof(float));
    memset(b->buffer_obs_noisy + (size_t)H * O * e, 0, H * O * sizeof(float));
    b->curent_command[e] = 0.0f;
    b->yaw_command[e] = 0.0f;   /* spawn_yaw_tgt (generate_spawn_r :580) */
    memset(b->command_history + CH * e, 0, CH * sizeof(float));
    b->speed_no_noise[e] = 0.0f;
}

/* post_physics_step (:397-482) + compute_obs_rwd (:491-547), then VecTask's
 * time_outs (vec_task.py:345). */
void oracle_paper_post_physics(const tg_paper_params *p, tg_paper_buffers *b, const float *reset_draws,
                               const float *noise, const float *speed_draws, const float *yaw_draws,
                               const float *push_draws) {
    int n = p->num_envs;
    for (int e = 0; e < n; ++e) {
        b->progress_buf[e] += 1;
        if (b->reset_buf[e] != 0) oracle_paper_reset_env(p, b, e, reset_draws + 9 * (size_t)e);
    }
    const float dn = (float)((double)p->command_delay[1] - (double)p->command_delay[0]);
    double dsum = 0.0;
    for (int e = 0; e < n; ++e) {
        float ob[O];
        float dl = (float)(b->steer_delay[e] - (int64_t)p->command_delay[0]) / dn;
        oracle_paper_observation(b->root + 13 * (size_t)e, b->yaw_command[e], b->curent_command[e], dl, ob);
        float *bo = b->buffer_obs + (size_t)H * O * e, *bn = b->buffer_obs_noisy + (size_t)H * O * e;
        memmove(bo, bo + O, (H - 1) * O * sizeof(float));
        memmove(bn, bn + O, (H - 1) * O * sizeof(float));
        memcpy(bo + (H - 1) * O, ob, sizeof ob);
        memcpy(bn + (H - 1) * O, ob, sizeof ob);
        dsum += act_diff_sq(bo);
    }
    float r7 = 1.0f - (float)(dsum / ((double)n * (H - 1)));
    for (int e = 0; e < n; ++e) {
        float *bo = b->buffer_obs + (size_t)H * O * e, *bn = b->buffer_obs_noisy + (size_t)H * O * e;
        reward_one(bo, b->progress_buf[e], p->max_episode_length, p->max_tilt, r7, b->rew_buf + e, b->reset_buf + e);
        b->speed_no_noise[e] = bo[(H - 1) * O + 4];
        const float *u = noise + 6 * (size_t)e;
        float *l = bn + (H - 1) * O;
        l[0] += u_aff(p->imu_filter_noise, u[0]);
        l[1] += u_aff(p->imu_filter_noise, u[1]);
        l[0] += b->curent_imu_x_offset[e];
        l[2] += u_aff(p->imu_noise, u[2]);
        l[3] += u_aff(p->imu_noise, u[3]);
        l[4] += u_aff(p->speed_sensor_noise, u[4]);
        l[4] += b->curent_speed_offset[e];
        l[4] = l[4] < 0.0f ? 0.0f : l[4];
        l[5] += u_aff(p->imu_filter_noise, u[5]);
        l[0] /= F_PI;
        l[1] /= F_PI;
        l[2] /= 3.0f;
        l[3] /= 3.0f;
        l[4] /= 5.0f;
        l[5] /= F_PI;
        l[6] /= p->max_steering;
        float dcmd = bo[(H - 2) * O + 6] - bo[(H - 1) * O + 6];
        l[2] += dcmd;
        l[0] += dcmd * 0.3f;
        for (int t = 0; t < H; ++t) bn[t * O + 1] = 0.0f;
        memcpy(b->obs_buf + (size_t)H * O * e, bn, H * O * sizeof(float));
    }
    /* command changes (:402-417); speed_command_change[speed_command_change] is
     * the identity on every input the reference accepts */
    for (int e = 0; e < n; ++e) {
        if (b->progress_buf[e] == p->speed_freq_update) b->curent_speed[e] = u_aff(p->speed_range, speed_draws[e]);
        if (b->progress_buf[e] == p->yaw_freq_update)   /* get_randoms(n, [-pi, pi]) */
            b->yaw_command[e] = -F_PI + yaw_draws[e] * (float)(2.0 * 3.14159265358979323846);
        float y = b->yaw_command[e];
        y = y > F_PI ? y - (float)(3.14159265358979323846 * 2) : y;
        y = y < -F_PI ? y + (float)(3.14159265358979323846 * 2) : y;
        b->yaw_command[e] = y;
    }
    /* pushes (:442-459) on head_p_link, first push_max_envs envs */
    if (p->push_robot) {
        for (int e = 0; e < n && e < p->push_max_envs; ++e) {
            if ((b->progress_buf[e] + 1) % p->push_interval != 0) continue;
            float yaw = b->buffer_obs[(size_t)H * O * e + (H - 1) * O + 1];
            float xf = (push_draws[2 * e] * 2.0f - 1.0f) * p->push_force;
            float zf = -(push_draws[2 * e + 1] * p->push_force);
            float *pe = b->perturbation + (size_t)(p->perturbation_stride ? p->perturbation_stride : 3) * e;
            pe[0] = xf * cosf(yaw + F_PI / 2.0f);
            pe[1] = xf * sinf(yaw + F_PI / 2.0f);
            pe[2] = zf;
        }
    }
    for (int e = 0; e < n; ++e) {
        int64_t prog = b->progress_buf[e];
        b->timeout_buf[e] = (prog >= p->max_episode_length - 1) && (b->reset_buf[e] != 0);
    }
}

/* apply_rigid_body_force_tensors of the head perturbation (:457) as the root
 * group's wrench: world force at head_p_link's COM -> force at the group COM
 * plus the moment (p_head - p_com) x f (tg_apply_body_forces convention). */
void oracle_paper_head_wrench(const tg_paper_params *p, const tg_paper_buffers *b) {
    int G = p->num_groups;
    for (int e = 0; e < p->num_envs; ++e) {
        const float *q = b->root + 13 * (size_t)e + 3;
        float x = q[0], y = q[1], z = q[2], w = q[3];
        float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                      2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                      2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
        float dl[3] = {p->head_com[0] - p->group0_com[0], p->head_com[1] - p->group0_com[1],
                       p->head_com[2] - p->group0_com[2]};
        float r[3];
        for (int i = 0; i < 3; ++i) r[i] = R[3 * i] * dl[0] + R[3 * i + 1] * dl[1] + R[3 * i + 2] * dl[2];
        const float *f = b->perturbation + 3 * (size_t)e;
        float *wr = b->body_force + (size_t)6 * G * e;
        memset(wr, 0, (size_t)6 * G * sizeof(float));
        wr[0] = f[0]; wr[1] = f[1]; wr[2] = f[2];
        wr[3] = r[1] * f[2] - r[2] * f[1];
        wr[4] = r[2] * f[0] - r[0] * f[2];
        wr[5] = r[0] * f[1] - r[1] * f[0];
    }
}
