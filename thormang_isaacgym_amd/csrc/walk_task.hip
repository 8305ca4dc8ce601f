// walk_task.hip -- fused ThormangWalk task kernels (include/tg_walk.h): the
// action kernel runs one lane per (env, dof); post-physics and reset run one
// wavefront per env (lane = dof).  The reference has no walking task; the
// semantics are this build's design and are checked against oracle/walk_task.c.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/tg_walk.h"
#include "tg_kernels.h"

namespace tg {

#define W_PI 3.14159265358979323846f

__device__ __forceinline__ float clampw(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

__global__ __launch_bounds__(256) void walk_pre_kernel(tg_walk_params p, tg_walk_buffers b, const float *actions) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;   // num_envs * num_dof < 2^32
    const unsigned D = (unsigned)p.num_dof;
    if (t >= (unsigned)p.num_envs * D) return;
    const int d = (int)(t % D);
    float a = clampw(actions[t], -p.clip_actions, p.clip_actions);
    b.actions[t] = a;
    b.pos_target[t] = p.default_pos[d] + p.action_scale * a;
}

// sum over the wavefront, returned to every lane: DPP within each 16-lane row
// (half-mirror, quad swaps, row rotate by 8), then the four row totals
template <int CTRL> __device__ __forceinline__ float dppw(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_total(float v) {
    v += dppw<0x141>(v);
    v += dppw<0x4E>(v);
    v += dppw<0xB1>(v);
    v += dppw<0x128>(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

// One wavefront per env: lane d handles dof d (reset, dof observations, the
// per-dof reward sums); lane 0 the root, commands, reward and termination.
// Every input of the env (the lane's dof, the root, the commands) is read in
// one batch with the progress / reset flags, so the wave pays one memory
// latency; a reset env then replaces them with the freshly drawn values.
__device__ void walk_env(const tg_walk_params &p, const tg_walk_buffers &b, int e, bool reset, int64_t prog,
                         const float *reset_draws, uint32_t c_lo, uint32_t c_hi) {
    const int lane = threadIdx.x % 64;   // one wavefront per env, 64 >= num_dof (TG_WALK_MAX_DOF)
    const int D = p.num_dof;
    float *root = b.root + 13 * (size_t)e;
    float *o = b.obs_buf + (size_t)p.num_obs * e;
    const float co = p.clip_obs;
    const bool dl = lane < D;
    const size_t i = (size_t)e * D + lane;
    float q = 0.0f, qd = 0.0f, a = 0.0f, la = 0.0f, pt = 0.0f;
    float rt[13], cmd[3];
    if (dl) {   // issued before the reset flag is known (a reset env overwrites them)
        pt = b.pos_target[i];
        q = b.dof_state[2 * i];
        qd = b.dof_state[2 * i + 1];
        a = b.actions[i];
        la = b.last_actions[i];
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 13; ++k) rt[k] = root[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) cmd[k] = b.commands[3 * (size_t)e + k];
    }
    if (reset) {
        if (dl) {
            q = p.default_pos[lane] + (walk_draw(p, reset_draws, e, 4 + lane, c_lo, c_hi) * 2.0f - 1.0f) * p.joint_noise;
            qd = 0.1f * (walk_draw(p, reset_draws, e, 4 + D + lane, c_lo, c_hi) * 2.0f - 1.0f);
            b.dof_state[2 * i] = q;
            b.dof_state[2 * i + 1] = qd;
            b.actions[i] = 0.0f;
            a = la = 0.0f;
        }
        if (lane == 0) {
            float r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = walk_draw(p, reset_draws, e, k, c_lo, c_hi);
            cmd[0] = p.cmd_vx[0] + r[0] * (p.cmd_vx[1] - p.cmd_vx[0]);
            cmd[1] = p.cmd_vy[0] + r[1] * (p.cmd_vy[1] - p.cmd_vy[0]);
            cmd[2] = p.cmd_wz[0] + r[2] * (p.cmd_wz[1] - p.cmd_wz[0]);
            const float yaw = (r[3] * 2.0f - 1.0f) * W_PI;
            const float *tpl = b.root_reset + 13 * (size_t)e;
            rt[0] = tpl[0];
            rt[1] = tpl[1];
            rt[2] = p.spawn_height;
            rt[3] = 0.0f;
            rt[4] = 0.0f;
            rt[5] = sinf(0.5f * yaw);
            rt[6] = cosf(0.5f * yaw);
#pragma unroll
            for (int k = 7; k < 13; ++k) rt[k] = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k) b.commands[3 * (size_t)e + k] = cmd[k];
#pragma unroll
            for (int k = 0; k < 13; ++k) root[k] = rt[k];
            b.progress_buf[e] = 0;
        }
    }
    // dof observations and the per-dof reward terms
    float rate = 0.0f, vel2 = 0.0f, tq = 0.0f;
    if (dl) {
        o[13 + lane] = clampw((q - p.default_pos[lane]) * p.dof_pos_scale, -co, co);
        o[13 + D + lane] = clampw(qd * p.dof_vel_scale, -co, co);
        o[13 + 2 * D + lane] = clampw(a, -co, co);
        rate = (a - la) * (a - la);
        vel2 = qd * qd;
        const float tt = p.stiffness[lane] * (pt - q);
        tq = tt * tt;
        b.last_actions[i] = a;
    }
    rate = wave_total(rate);
    vel2 = wave_total(vel2);
    tq = wave_total(tq);
    if (lane != 0) return;
    const float x = rt[3], y = rt[4], z = rt[5], w = rt[6];
    const float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                        2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                        2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
    float vb[3], wb[3], gb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        vb[k] = R[k] * rt[7] + R[3 + k] * rt[8] + R[6 + k] * rt[9];
        wb[k] = R[k] * rt[10] + R[3 + k] * rt[11] + R[6 + k] * rt[12];
        gb[k] = -R[6 + k];
    }
    o[0] = clampw(rt[2], -co, co);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        o[1 + k] = clampw(vb[k] * p.lin_vel_scale, -co, co);
        o[4 + k] = clampw(wb[k] * p.ang_vel_scale, -co, co);
        o[7 + k] = clampw(gb[k], -co, co);
    }
    o[10] = clampw(cmd[0] * p.lin_vel_scale, -co, co);
    o[11] = clampw(cmd[1] * p.lin_vel_scale, -co, co);
    o[12] = clampw(cmd[2] * p.ang_vel_scale, -co, co);
    const float lin_err = (cmd[0] - vb[0]) * (cmd[0] - vb[0]) + (cmd[1] - vb[1]) * (cmd[1] - vb[1]);
    const float ang_err = (cmd[2] - wb[2]) * (cmd[2] - wb[2]);
    const float dz = rt[2] - p.target_height;
    float rew = p.rew_lin_vel_xy * expf(-lin_err / 0.25f) + p.rew_ang_vel_z * expf(-ang_err / 0.25f) +
                p.rew_upright * (-gb[2]) + p.rew_alive + p.rew_height * expf(-dz * dz / 0.01f) +
                p.rew_action_rate * rate + p.rew_dof_vel * vel2 + p.rew_torque * tq;
    const bool fall = (rt[2] < p.termination_height) || (-gb[2] < p.termination_up);
    if (fall) rew += p.rew_termination;
    const bool rs = fall || prog >= p.max_episode_length - 1;
    b.rew_buf[e] = rew;
    b.reset_buf[e] = rs ? 1 : 0;
    b.timeout_buf[e] = (prog >= p.max_episode_length - 1) && rs;
}

#ifndef TG_WALK_POST_WPB
#define TG_WALK_POST_WPB 16
#endif
// WALK_POST_WPB wavefronts (envs) per workgroup
constexpr int WALK_POST_WPB = TG_WALK_POST_WPB;
__global__ __launch_bounds__(64 * WALK_POST_WPB) void walk_post_kernel(tg_walk_params p, tg_walk_buffers b,
                                                                       const float *reset_draws, const float *push_draws,
                                                                       uint32_t c_lo, uint32_t c_hi) {
    const int e = blockIdx.x * WALK_POST_WPB + threadIdx.x / 64;
    if (e >= p.num_envs) return;
    const int lane = threadIdx.x % 64;
    int64_t prog = b.progress_buf[e] + 1;
    const bool reset = b.reset_buf[e] != 0;
    if (lane == 0) b.progress_buf[e] = prog;
    if (reset) prog = 0;
    walk_env(p, b, e, reset, prog, reset_draws, c_lo, c_hi);
    if (lane != 0 || !b.body_force) return;
    float *f = b.body_force + (size_t)6 * p.num_groups * e;
    const bool push = p.push_force > 0.0f && p.push_interval > 0 && prog > 0 && (prog % p.push_interval) == 0;
    float u[3];
    if (push_draws) {
        u[0] = push_draws[3 * (size_t)e]; u[1] = push_draws[3 * (size_t)e + 1]; u[2] = push_draws[3 * (size_t)e + 2];
    } else {
        U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, 0x50555348u}, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        u[0] = u01(x.x); u[1] = u01(x.y); u[2] = u01(x.z);
    }
    f[0] = push ? p.push_force * (u[0] * 2.0f - 1.0f) : 0.0f;
    f[1] = push ? p.push_force * (u[1] * 2.0f - 1.0f) : 0.0f;
    f[2] = push ? 0.25f * p.push_force * (u[2] * 2.0f - 1.0f) : 0.0f;
    f[3] = 0.0f; f[4] = 0.0f; f[5] = 0.0f;
}

__global__ __launch_bounds__(64) void walk_reset_idx_kernel(tg_walk_params p, tg_walk_buffers b, const int32_t *ids,
                                                            int n, const float *reset_draws, uint32_t c_lo,
                                                            uint32_t c_hi) {
    const int e = ids[blockIdx.x];
    if (e < 0 || e >= p.num_envs) return;
    walk_env(p, b, e, true, 0, reset_draws, c_lo, c_hi);
}

int launch_walk_pre(const tg_walk_params &p, const tg_walk_buffers &b, const float *actions, hipStream_t s) {
    const size_t tot = (size_t)p.num_envs * p.num_dof;
    hipLaunchKernelGGL(walk_pre_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, p, b, actions);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_walk_post(const tg_walk_params &p, const tg_walk_buffers &b, const float *rd, const float *pd,
                     uint64_t counter, hipStream_t s) {
    if (p.num_dof > TG_WALK_MAX_DOF) return TG_ERR_ARG;
    hipLaunchKernelGGL(walk_post_kernel, dim3((p.num_envs + WALK_POST_WPB - 1) / WALK_POST_WPB),
                       dim3(64 * WALK_POST_WPB), 0, s, p, b, rd, pd,
                       (uint32_t)counter, (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_walk_reset_idx(const tg_walk_params &p, const tg_walk_buffers &b, const int32_t *ids, int n,
                          const float *rd, uint64_t counter, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(walk_reset_idx_kernel, dim3(n), dim3(64), 0, s, p, b, ids, n, rd,
                       (uint32_t)counter, (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

}  // namespace tg
