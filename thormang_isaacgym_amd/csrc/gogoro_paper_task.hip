// gogoro_paper_task.hip -- fused task kernels of the Gogoro "paper" variant
// (include/tg_gogoro_paper.h; reference
// isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py, line numbers below).
//
// One wavefront per env (lane = history slot / dof):
//   paper_pre_kernel    pre_physics_step (:349-393)
//   paper_post_kernel   post_physics_step (:397-482): masked reset_idx
//                       (:609-692), observation (:771-808), 20-step clean /
//                       noisy histories (:503-547), reward terms 1-5, command
//                       changes, head pushes and the root-group wrench
//   paper_finish_kernel one workgroup: batch mean of the squared command
//                       differences (torch.mean without dim, :740, reward term
//                       7), rewards, resets, VecTask time_outs
// fp32 in the reference's operation order (compiled -ffp-contract=off).
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/tg_gogoro_paper.h"
#include "tg_kernels.h"

namespace tg {

#define P_PI 3.14159265358979323846f
#define P_2PI 6.28318530717958647692f
constexpr int PH = TG_PAPER_HIST, PO = TG_PAPER_OBS, PC = TG_PAPER_CMD_HIST, PHO = PH * PO;

__device__ __forceinline__ float p_rem(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
    return m;
}
__device__ __forceinline__ float p_clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ float p_aff(const float *b, float u) {
    return b[0] + u * (float)((double)b[1] - (double)b[0]);
}
__device__ __forceinline__ float p_wsum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// reset draw k (0..8) of env e: replay array or Philox (4 per counter)
__device__ __forceinline__ float p_draw(const tg_paper_params &p, const float *arr, int stride, int e, int k,
                                        uint32_t c_lo, uint32_t c_hi, uint32_t tag) {
    if (arr) return arr[(size_t)stride * e + k];
    const U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, tag + (uint32_t)(k >> 2)}, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
    const uint32_t c = (k & 3) == 0 ? x.x : (k & 3) == 1 ? x.y : (k & 3) == 2 ? x.z : x.w;
    return u01(c);
}

__global__ __launch_bounds__(64) void paper_pre_kernel(tg_paper_params p, tg_paper_buffers b, const float *actions) {
    const int e = blockIdx.x, lane = threadIdx.x;
    const int D = p.num_dof;
    float *h = b.command_history + PC * (size_t)e;
    float hv = 0.f, cmd = 0.f;
    {
        const float a = p_clamp(actions[e], -1.0f, 1.0f);
        cmd = a * p.max_steering;
        if (lane < PC) hv = lane < PC - 1 ? h[lane + 1] : cmd;
    }
    __syncthreads();
    if (lane < PC) h[lane] = hv;
    __syncthreads();
    float *pt = b.pos_target + (size_t)D * e, *vt = b.vel_target + (size_t)D * e;
    for (int d = lane; d < D; d += 64) {
        pt[d] = 0.0f;
        vt[d] = 0.0f;
    }
    __syncthreads();
    if (lane == 0) {
        b.curent_command[e] = cmd;
        int idx = PC - 3;
        if (p.use_steer_delay) {   // command_history[:, -steer_delay]; -0 selects slot 0
            const int64_t d = b.steer_delay[e];
            idx = d == 0 ? 0 : (int)(PC - d);
        }
        pt[p.dof_steer] = h[idx];
        vt[p.dof_rear] = b.curent_speed[e];
    }
}

// reset_idx for env e (:609-692) by one wavefront
__device__ void paper_reset_env(const tg_paper_params &p, const tg_paper_buffers &b, int e, const float *rd,
                                uint32_t c_lo, uint32_t c_hi) {
    const int lane = threadIdx.x;
    const int D = p.num_dof;
    const size_t ND = (size_t)p.num_envs * D;
    for (int i = lane; i < PHO; i += 64) {
        b.obs_buf[(size_t)PHO * e + i] = 0.0f;
        b.buffer_obs[(size_t)PHO * e + i] = 0.0f;
        b.buffer_obs_noisy[(size_t)PHO * e + i] = 0.0f;
    }
    if (lane < PC) b.command_history[PC * (size_t)e + lane] = 0.0f;
    for (int d = lane; d < D; d += 64) {
        b.dof_state[2 * ((size_t)e * D + d)] = b.thormang_pose[(size_t)e * D + d];
        b.dof_state[2 * ((size_t)e * D + d) + 1] = 0.0f;
    }
    if (lane != 0) return;
    const uint32_t tag = 0x50415052u;
    float r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) r[k] = p_draw(p, rd, 9, e, k, c_lo, c_hi, tag);
    b.curent_speed[e] = p_aff(p.speed_range, r[0]);
    b.steer_delay[e] = (int64_t)p_aff(p.command_delay, r[1]);
    b.steer_offsets[e] = p_aff(p.steering_offset, r[2]);
    float *pz = b.perturbation + (size_t)(p.perturbation_stride ? p.perturbation_stride : 3) * e;
    pz[0] = 0.0f;
    pz[1] = 0.0f;
    pz[2] = 0.0f;
    b.curent_speed_offset[e] = p_aff(p.speed_sensor_offset, r[3]);
    float *root = b.root + 13 * (size_t)e;
    const float *tpl = b.root_reset + 13 * (size_t)e;
#pragma unroll
    for (int k = 0; k < 13; ++k) root[k] = tpl[k];
    root[2] = p.spawn_z;
    root[3] = 0.0f; root[4] = 0.0f; root[5] = 0.0f; root[6] = 1.0f;
#pragma unroll
    for (int k = 7; k < 13; ++k) root[k] = 0.0f;
    if (p.debug_start_speed) {
        root[7] = p.start_speed * cosf(0.0f);
        root[8] = p.start_speed * sinf(0.0f);
    }
    b.curent_imu_x_offset[e] = p_aff(p.imu_x_offset, r[4]);
    float *prop = b.dof_props + (size_t)e * D;
    if (p.random_damping) {
        const float damp = p_aff(p.steering_damping_range, r[5]);
        b.curent_damping_cfg[e] = damp;
        const int st = p.dof_steer;
        prop[TG_PROP_DRIVE_MODE * ND + st] = (float)TG_DOF_MODE_POS;
        prop[TG_PROP_STIFFNESS * ND + st] = p.damping_stiffness;
        prop[TG_PROP_DAMPING * ND + st] = damp;
        prop[TG_PROP_EFFORT * ND + st] = p.damping_effort;
        prop[TG_PROP_VELOCITY * ND + st] = p.damping_velocity;
        b.env_dirty[e] = 1;
    }
    if (!p.center_robot) {
        const int seat[3] = {p.dof_base_x, p.dof_base_y, p.dof_base_z};
        const float *rg[3] = {p.seat_offset_x_range, p.seat_offset_y_range, p.seat_offset_z_range};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float lo = p_aff(rg[k], r[6 + k]);
            prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
            prop[TG_PROP_LOWER * ND + seat[k]] = lo;
            prop[TG_PROP_UPPER * ND + seat[k]] = (float)((double)lo + 0.0001);
        }
        b.env_dirty[e] = 1;
    }
    b.progress_buf[e] = 0;
    b.reset_buf[e] = 0;
    b.curent_command[e] = 0.0f;
    b.yaw_command[e] = 0.0f;
    b.speed_no_noise[e] = 0.0f;
}

// compute_gogoro_observations (:771-808)
__device__ void paper_observe(const float *root, float desired_yaw, float command, float delay_norm, float *obs) {
    const float x = root[3], y = root[4], z = root[5], w = root[6];
    float roll = p_rem(atan2f(2.0f * (w * x + y * z), w * w - x * x - y * y + z * z), P_2PI);
    float yaw = p_rem(atan2f(2.0f * (w * z + x * y), w * w + x * x - y * y - z * z), P_2PI);
    float lin[3], ang[3];
    const float s = 2.0f * (w * w) - 1.0f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float *v = root + (k == 0 ? 7 : 10);
        float *o = k == 0 ? lin : ang;
        const float cx = y * v[2] - z * v[1], cy = z * v[0] - x * v[2], cz = x * v[1] - y * v[0];
        const float d = x * v[0] + y * v[1] + z * v[2];
        o[0] = v[0] * s - cx * w * 2.0f + x * d * 2.0f;
        o[1] = v[1] * s - cy * w * 2.0f + y * d * 2.0f;
        o[2] = v[2] * s - cz * w * 2.0f + z * d * 2.0f;
    }
    if (roll > P_PI) roll = roll - P_2PI;
    if (roll < -P_PI) roll = roll + P_2PI;
    if (yaw > P_PI) yaw = yaw - P_2PI;
    if (yaw < -P_PI) yaw = yaw + P_2PI;
    obs[0] = roll;
    obs[1] = yaw;
    obs[2] = ang[0];
    obs[3] = ang[2];
    obs[4] = lin[0];
    obs[5] = p_rem(desired_yaw - yaw + P_PI, P_2PI) - P_PI;
    obs[6] = command;
    obs[7] = delay_norm;
}

__global__ __launch_bounds__(64) void paper_post_kernel(tg_paper_params p, tg_paper_buffers b, const float *rd,
                                                        const float *nd, const float *sd, const float *yd,
                                                        const float *pd, uint32_t c_lo, uint32_t c_hi) {
    __shared__ float ob[PO], nz[PO];
    const int e = blockIdx.x, lane = threadIdx.x;
    const bool reset = b.reset_buf[e] != 0;
    const int64_t prog0 = b.progress_buf[e] + 1;
    __syncthreads();
    if (lane == 0) b.progress_buf[e] = prog0;
    if (reset) paper_reset_env(p, b, e, rd, c_lo, c_hi);
    __syncthreads();
    const int64_t prog = reset ? 0 : prog0;
    float *bo = b.buffer_obs + (size_t)PHO * e, *bn = b.buffer_obs_noisy + (size_t)PHO * e;
    if (lane == 0) {
        const float dn = (float)((double)p.command_delay[1] - (double)p.command_delay[0]);
        const float dl = (float)(b.steer_delay[e] - (int64_t)p.command_delay[0]) / dn;
        float o[PO];
        paper_observe(b.root + 13 * (size_t)e, b.yaw_command[e], b.curent_command[e], dl, o);
        const float dcmd = bo[(PH - 1) * PO + 6] - o[6];   // clean[-2][6] - clean[-1][6] after the shift
        // noisy newest entry (:521-542)
        const uint32_t tag = 0x50414e5au;
        float u[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) u[k] = p_draw(p, nd, 6, e, k, c_lo, c_hi, tag);
        float l[PO];
#pragma unroll
        for (int k = 0; k < PO; ++k) l[k] = o[k];
        l[0] += p_aff(p.imu_filter_noise, u[0]);
        l[1] += p_aff(p.imu_filter_noise, u[1]);
        l[0] += b.curent_imu_x_offset[e];
        l[2] += p_aff(p.imu_noise, u[2]);
        l[3] += p_aff(p.imu_noise, u[3]);
        l[4] += p_aff(p.speed_sensor_noise, u[4]);
        l[4] += b.curent_speed_offset[e];
        l[4] = l[4] < 0.0f ? 0.0f : l[4];
        l[5] += p_aff(p.imu_filter_noise, u[5]);
        l[0] /= P_PI;
        l[1] /= P_PI;
        l[2] /= 3.0f;
        l[3] /= 3.0f;
        l[4] /= 5.0f;
        l[5] /= P_PI;
        l[6] /= p.max_steering;
        l[2] += dcmd;
        l[0] += dcmd * 0.3f;
        l[1] = 0.0f;
#pragma unroll
        for (int k = 0; k < PO; ++k) { ob[k] = o[k]; nz[k] = l[k]; }
        b.speed_no_noise[e] = o[4];
    }
    __syncthreads();
    // shift both histories by one entry and append
    float vc[3], vn[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int i = lane + 64 * j;
        if (i < PHO) {
            vc[j] = i < PHO - PO ? bo[i + PO] : ob[i - (PHO - PO)];
            vn[j] = i < PHO - PO ? bn[i + PO] : nz[i - (PHO - PO)];
            if ((i % PO) == 1) vn[j] = 0.0f;   // noisy[:, :, 1] = 0
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int i = lane + 64 * j;
        if (i < PHO) {
            bo[i] = vc[j];
            bn[i] = vn[j];
            b.obs_buf[(size_t)PHO * e + i] = vn[j];
        }
    }
    __syncthreads();
    // reward term 7 partial: sum_t (a[t+1] - a[t])^2, a = act / 0.5
    float dsq = 0.0f;
    if (lane < PH - 1) {
        const float dd = bo[(lane + 1) * PO + 6] / 0.5f - bo[lane * PO + 6] / 0.5f;
        dsq = dd * dd;
    }
    dsq = p_wsum(dsq);
    if (lane == 0) {
        b.scratch[e] = dsq;
        // reward terms 1-5 (:722-746)
        const float *last = bo + (PH - 1) * PO;
        const float tilt_err = p_clamp(last[0] / p.max_tilt, -1.0f, 1.0f);
        const float yaw_err = p_clamp(last[5] / P_PI, -1.0f, 1.0f);
        const float dtilt_err = p_clamp(last[2] / 0.3f, -1.0f, 1.0f);
        const float act = last[6] / 0.5f;
        const float r1 = 1.0f - yaw_err * yaw_err;
        const float r2 = 1.0f - tilt_err * tilt_err;
        const float r4 = 1.0f - dtilt_err * dtilt_err;
        const float tilt_w = 1.0f - tanhf(50.0f * (tilt_err * tilt_err));
        const float dtilt_w = 1.0f - tanhf(50.0f * (dtilt_err * dtilt_err));
        const float r5 = 1.0f - (act * act) * (tilt_w * dtilt_w);
        b.rew_buf[e] = r1 * 0.45f + r2 * 0.1f + r4 * 0.35f + r5 * 2.0f;
        // command changes (:402-417)
        if (prog == p.speed_freq_update) b.curent_speed[e] = p_aff(p.speed_range, p_draw(p, sd, 1, e, 0, c_lo, c_hi, 0x50415344u));
        float yc = b.yaw_command[e];
        if (prog == p.yaw_freq_update) yc = -P_PI + p_draw(p, yd, 1, e, 0, c_lo, c_hi, 0x50415957u) * (float)(2.0 * 3.14159265358979323846);
        yc = yc > P_PI ? yc - (float)(3.14159265358979323846 * 2) : yc;
        yc = yc < -P_PI ? yc + (float)(3.14159265358979323846 * 2) : yc;
        b.yaw_command[e] = yc;
        // pushes on head_p_link (:442-459)
        float *pert = b.perturbation + (size_t)(p.perturbation_stride ? p.perturbation_stride : 3) * e;
        if (p.push_robot && e < p.push_max_envs && (prog + 1) % p.push_interval == 0) {
            const float yaw = last[1];
            const float xf = (p_draw(p, pd, 2, e, 0, c_lo, c_hi, 0x50415055u) * 2.0f - 1.0f) * p.push_force;
            const float zf = -(p_draw(p, pd, 2, e, 1, c_lo, c_hi, 0x50415055u) * p.push_force);
            pert[0] = xf * cosf(yaw + P_PI / 2.0f);
            pert[1] = xf * sinf(yaw + P_PI / 2.0f);
            pert[2] = zf;
        }
        if (b.body_force) {   // root-group wrench: force at the head COM
            const float *q = b.root + 13 * (size_t)e + 3;
            const float x = q[0], y = q[1], z = q[2], w = q[3];
            const float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                                2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                                2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
            const float dl[3] = {p.head_com[0] - p.group0_com[0], p.head_com[1] - p.group0_com[1],
                                 p.head_com[2] - p.group0_com[2]};
            float r[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) r[i] = R[3 * i] * dl[0] + R[3 * i + 1] * dl[1] + R[3 * i + 2] * dl[2];
            float *wr = b.body_force + (size_t)6 * p.num_groups * e;
            wr[0] = pert[0]; wr[1] = pert[1]; wr[2] = pert[2];
            wr[3] = r[1] * pert[2] - r[2] * pert[1];
            wr[4] = r[2] * pert[0] - r[0] * pert[2];
            wr[5] = r[0] * pert[1] - r[1] * pert[0];
        }
    }
    if (b.body_force) {
        float *wr = b.body_force + (size_t)6 * p.num_groups * e;
        for (int i = 6 + lane; i < 6 * p.num_groups; i += 64) wr[i] = 0.0f;
    }
}

// one workgroup: batch mean for reward term 7, rewards, resets, time_outs
__global__ __launch_bounds__(1024) void paper_finish_kernel(tg_paper_params p, tg_paper_buffers b) {
    __shared__ double part[1024];
    const int t = threadIdx.x, n = p.num_envs;
    double s = 0.0;
    for (int e = t; e < n; e += 1024) s += (double)b.scratch[e];
    part[t] = s;
    __syncthreads();
    for (int w = 512; w >= 1; w >>= 1) {
        if (t < w) part[t] += part[t + w];
        __syncthreads();
    }
    const float r7 = 1.0f - (float)(part[0] / ((double)n * (PH - 1)));
    for (int e = t; e < n; e += 1024) {
        const float tilt = b.buffer_obs[(size_t)PHO * e + (PH - 1) * PO];
        const int64_t prog = b.progress_buf[e];
        const bool finished = prog >= p.max_episode_length - 1;
        const bool felt = fabsf(tilt) >= p.max_tilt;
        float r = b.rew_buf[e] + r7 * 0.2f;
        r = r < 0.0f ? 0.0f : r;
        b.rew_buf[e] = felt ? -1.0f : r;
        const bool rs = finished || felt;
        b.reset_buf[e] = rs ? 1 : 0;
        b.timeout_buf[e] = finished && rs;
    }
}

__global__ __launch_bounds__(64) void paper_reset_idx_kernel(tg_paper_params p, tg_paper_buffers b, const int32_t *ids,
                                                             const float *rd, uint32_t c_lo, uint32_t c_hi) {
    const int e = ids[blockIdx.x];
    if (e < 0 || e >= p.num_envs) return;
    paper_reset_env(p, b, e, rd, c_lo, c_hi);
}

int launch_paper_pre(const tg_paper_params &p, const tg_paper_buffers &b, const float *actions, hipStream_t s) {
    hipLaunchKernelGGL(paper_pre_kernel, dim3(p.num_envs), dim3(64), 0, s, p, b, actions);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_paper_post(const tg_paper_params &p, const tg_paper_buffers &b, const float *rd, const float *nd,
                      const float *sd, const float *yd, const float *pd, uint64_t counter, hipStream_t s) {
    hipLaunchKernelGGL(paper_post_kernel, dim3(p.num_envs), dim3(64), 0, s, p, b, rd, nd, sd, yd, pd,
                       (uint32_t)counter, (uint32_t)(counter >> 32));
    hipLaunchKernelGGL(paper_finish_kernel, dim3(1), dim3(1024), 0, s, p, b);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_paper_reset_idx(const tg_paper_params &p, const tg_paper_buffers &b, const int32_t *ids, int n,
                           const float *rd, uint64_t counter, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(paper_reset_idx_kernel, dim3(n), dim3(64), 0, s, p, b, ids, rd, (uint32_t)counter,
                       (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

}  // namespace tg
