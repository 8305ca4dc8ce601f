// gogoro_task.hip -- fused Gogoro task kernels (one env per lane).
//
// Replaces the reference's per-step TorchScript / Python task code
// (isaacgymenvs/tasks/gogoro_new.py):
//   pre_kernel  : pre_physics_step :347-369 (+ VecTask action clamp, vec_task.py:327)
//   post_kernel : post_physics_step :373-390, compute_obs_rwd :424-462,
//                 compute_gogoro_observations :692-723, compute_gogoro_reward :645-684,
//                 reset_idx/randomize/generate_spawn_r/set_env_dof_prop :474-601
//                 (masked: no nonzero(), no host sync), VecTask timeout/obs clamp
//                 (vec_task.py:345-353).
// Arithmetic follows the reference's fp32 operation order (this TU is built
// with -ffp-contract=off) so results match oracle/gogoro_task.c and the
// golden fixtures to fp32 rounding of the transcendental functions.
#include <atomic>
#include <hip/hip_runtime.h>
#include <math.h>

#include "gogoro_math.h"
#include "tg_kernels.h"

namespace tg {

__global__ __launch_bounds__(256) void pre_kernel(tg_gogoro_params p, tg_gogoro_buffers b, const float *actions,
                                                  const float *pre_draws, uint32_t c_lo, uint32_t c_hi) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= p.num_envs) return;
    const int D = p.num_dof;
    float a = t_clamp(actions[e], -p.clip_actions, p.clip_actions);
    float *ah = b.action_history + 5 * e;
    float h0 = ah[1], h1 = ah[2], h2 = ah[3], h3 = ah[4];
    ah[0] = h0; ah[1] = h1; ah[2] = h2; ah[3] = h3; ah[4] = a;
    float c;
    if (p.absolute_steer) {   // INCREMENTAL_STEER = False (gogoro_new.py:355-356)
        c = t_clamp(a * p.max_steering, -p.max_steering, p.max_steering);
    } else {
        float da = t_clamp(a * p.max_steering_change, -p.max_steering_change, p.max_steering_change);
        c = t_clamp(b.curent_command[e] + da, -p.max_steering, p.max_steering);
    }
    b.curent_command[e] = c;
    float r;
    if (pre_draws) r = pre_draws[e];
    else {
        U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, 0x50524531u}, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        r = gauss(x.x, x.y);
    }
    float noise = p.steering_action_noise[0] + r * p.steering_action_noise[1];
    b.pos_target[(size_t)e * D + p.dof_steer] = c + b.steer_offsets[e] + noise;
    b.vel_target[(size_t)e * D + p.dof_rear] = b.curent_speed[e];
}

__device__ void philox_reset_draws(int e, uint32_t c_lo, uint32_t c_hi, uint32_t k0, uint32_t k1, float *r);

__device__ void reset_env(const tg_gogoro_params &p, const tg_gogoro_buffers &b, int e, const float *r) {
    const int D = p.num_dof;
    b.curent_speed[e] = u_aff(p.speed_range[0], p.speed_range[1], r[0]);
    b.speed_offset[e] = u_aff(p.speed_sensor_offset[0], p.speed_sensor_offset[1], r[2]);
    const float target = (r[3] * 2.0f - 1.0f) * F_PI;
    const float rot = target + u_aff(-1.57f, 1.57f, r[4]);
    const float hh = rot / 2.0f;
    float *root = b.root + 13 * (size_t)e;
    const float *tpl = b.root_reset + 13 * (size_t)e;
    root[0] = tpl[0];
    root[1] = tpl[1];
    root[2] = p.terrain_spawn ? tpl[2] : p.spawn_z;
    root[3] = 0.0f;
    root[4] = 0.0f;
    root[5] = sinf(hh);
    root[6] = cosf(hh);
#pragma unroll
    for (int k = 7; k < 13; ++k) root[k] = 0.0f;
    if (p.debug_start_speed) {   // DEBUG_START_SPEED (gogoro_new.py:542-545)
        root[7] = 1.3f * cosf(rot);
        root[8] = 1.3f * sinf(rot);
    }
    float *dof = b.dof_state + 2 * (size_t)e * D;
#pragma unroll 8
    for (int d = 0; d < D; ++d) {   // unrolled: 8 pose loads in flight instead of one per store
        dof[2 * d] = b.thormang_pose[d];
        dof[2 * d + 1] = 0.0f;
    }
    float *cv = b.config_vector + 5 * (size_t)e;
    cv[0] = n_aff(p.seat_offset_x_range, r[5]);
    cv[1] = n_aff(p.seat_offset_y_range, r[6]);
    cv[2] = n_aff(p.seat_offset_z_range, r[7]);
    cv[3] = n_aff(p.seat_offset_xr_range, r[8]);
    cv[4] = n_aff(p.steering_offset, r[9]);
    const size_t ND = (size_t)p.num_envs * D;
    float *prop = b.dof_props + (size_t)e * D;
    const int seat[3] = {p.dof_base_x, p.dof_base_y, p.dof_base_z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
        prop[TG_PROP_LOWER * ND + seat[k]] = cv[k];
        prop[TG_PROP_UPPER * ND + seat[k]] = cv[k] + 0.0001f;
    }
    b.imu_offsets[e] = cv[3];
    b.steer_offsets[e] = cv[4];
    const int st = p.dof_steer;
    prop[TG_PROP_DRIVE_MODE * ND + st] = 1.0f;
    prop[TG_PROP_STIFFNESS * ND + st] = p.steer_stiffness;
    prop[TG_PROP_DAMPING * ND + st] = u_aff(p.steering_damping_range[0], p.steering_damping_range[1], r[10]);
    prop[TG_PROP_EFFORT * ND + st] = p.steer_effort;
    prop[TG_PROP_VELOCITY * ND + st] = p.steer_velocity;
    b.env_dirty[e] = 1;
    b.progress_buf[e] = 0;
    b.reset_buf[e] = 0;
    b.curent_command[e] = 0.0f;
    b.yaw_command[e] = target;
#pragma unroll
    for (int k = 0; k < 5; ++k) b.action_history[5 * (size_t)e + k] = 0.0f;
}

// post_physics_step with POST_LPE lanes per env (4 envs per wavefront): the
// env's 9 Philox blocks (5 reset, 3 sensor noise, 1 command resample) run at
// once on lanes 0-8 and reach the lead lane through LDS, every input is read
// in one batch before the reset flag is known, a reset's dof writes are spread
// over the env's lanes, and the lead lane does the scalar task math on
// register copies.  Same counters and the same fp32 operations as the
// lane-per-env formulation (reset_env / philox_reset_draws), so the same values.
constexpr int POST_LPE = 16;
constexpr int POST_EPB = 64 / POST_LPE;
__global__ __launch_bounds__(64) void post_kernel(tg_gogoro_params p, tg_gogoro_buffers b, const float *reset_draws,
                                                  const float *obs_draws, const float *speed_draws,
                                                  const float *yaw_draws, uint32_t c_lo, uint32_t c_hi) {
    __shared__ float xch[POST_EPB][POST_LPE * 3];
    const int le = threadIdx.x / POST_LPE, l = threadIdx.x % POST_LPE;
    const int e0 = blockIdx.x * POST_EPB + le;
    const bool owner = e0 < p.num_envs;
    const int e = owner ? e0 : p.num_envs - 1;   // tail lanes redo the last env, never store
    const bool lead = l == 0;
    const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
    const int D = p.num_dof;
    // ---- inputs (lead lane), one batch
    int64_t prog = b.progress_buf[e] + 1;
    const bool rflag = b.reset_buf[e] != 0;
    float rt[13], ah[5], yawc = 0.0f, cmdc = 0.0f, imu = 0.0f;
    if (lead) {
        const float *root = b.root + 13 * (size_t)e;
#pragma unroll
        for (int k = 0; k < 13; ++k) rt[k] = root[k];
#pragma unroll
        for (int k = 0; k < 5; ++k) ah[k] = b.action_history[5 * (size_t)e + k];
        yawc = b.yaw_command[e];
        cmdc = b.curent_command[e];
        imu = b.imu_offsets[e];
    }
    // ---- draws: lane k < 9 runs Philox block k and leaves its (up to 3) floats in xch
    if (l < 9) {
        float v[3];
        gogoro_post_block(l, e, c_lo, c_hi, k0, k1, v);
#pragma unroll
        for (int j = 0; j < 3; ++j) xch[le][3 * l + j] = v[j];
    }
    __syncthreads();
    float r[TG_GOGORO_RESET_DRAWS];
    if (rflag) {
        if (reset_draws) {
#pragma unroll
            for (int k = 0; k < TG_GOGORO_RESET_DRAWS; ++k) r[k] = reset_draws[(size_t)e * TG_GOGORO_RESET_DRAWS + k];
        } else {
#pragma unroll
            for (int k = 0; k < TG_GOGORO_RESET_DRAWS; ++k) r[k] = xch[le][GOGORO_RSLOT[k]];
        }
        // reset_env: dof writes over the env's lanes, the rest on the lead lane
        if (owner) {
            float *dof = b.dof_state + 2 * (size_t)e * D;
            for (int d = l; d < D; d += POST_LPE) {
                dof[2 * d] = b.thormang_pose[d];
                dof[2 * d + 1] = 0.0f;
            }
        }
        if (lead) {
            const float target = (r[3] * 2.0f - 1.0f) * F_PI;
            const float rot = target + u_aff(-1.57f, 1.57f, r[4]);
            const float hh = rot / 2.0f;
            const float *tpl = b.root_reset + 13 * (size_t)e;
            rt[0] = tpl[0];
            rt[1] = tpl[1];
            rt[2] = p.terrain_spawn ? tpl[2] : p.spawn_z;
            rt[3] = 0.0f;
            rt[4] = 0.0f;
            rt[5] = sinf(hh);
            rt[6] = cosf(hh);
#pragma unroll
            for (int k = 7; k < 13; ++k) rt[k] = 0.0f;
            if (p.debug_start_speed) {   // DEBUG_START_SPEED (gogoro_new.py:542-545)
                rt[7] = 1.3f * cosf(rot);
                rt[8] = 1.3f * sinf(rot);
            }
            float cv[5];
            cv[0] = n_aff(p.seat_offset_x_range, r[5]);
            cv[1] = n_aff(p.seat_offset_y_range, r[6]);
            cv[2] = n_aff(p.seat_offset_z_range, r[7]);
            cv[3] = n_aff(p.seat_offset_xr_range, r[8]);
            cv[4] = n_aff(p.steering_offset, r[9]);
            imu = cv[3];
            yawc = target;
            cmdc = 0.0f;
#pragma unroll
            for (int k = 0; k < 5; ++k) ah[k] = 0.0f;
            if (owner) {
                b.curent_speed[e] = u_aff(p.speed_range[0], p.speed_range[1], r[0]);
                b.speed_offset[e] = u_aff(p.speed_sensor_offset[0], p.speed_sensor_offset[1], r[2]);
                float *root = b.root + 13 * (size_t)e;
#pragma unroll
                for (int k = 0; k < 13; ++k) root[k] = rt[k];
#pragma unroll
                for (int k = 0; k < 5; ++k) b.config_vector[5 * (size_t)e + k] = cv[k];
                const size_t ND = (size_t)p.num_envs * D;
                float *prop = b.dof_props + (size_t)e * D;
                const int seat[3] = {p.dof_base_x, p.dof_base_y, p.dof_base_z};
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
                    prop[TG_PROP_LOWER * ND + seat[k]] = cv[k];
                    prop[TG_PROP_UPPER * ND + seat[k]] = cv[k] + 0.0001f;
                }
                b.imu_offsets[e] = cv[3];
                b.steer_offsets[e] = cv[4];
                const int st = p.dof_steer;
                prop[TG_PROP_DRIVE_MODE * ND + st] = 1.0f;
                prop[TG_PROP_STIFFNESS * ND + st] = p.steer_stiffness;
                prop[TG_PROP_DAMPING * ND + st] = u_aff(p.steering_damping_range[0], p.steering_damping_range[1], r[10]);
                prop[TG_PROP_EFFORT * ND + st] = p.steer_effort;
                prop[TG_PROP_VELOCITY * ND + st] = p.steer_velocity;
                b.env_dirty[e] = 1;
                b.curent_command[e] = 0.0f;
#pragma unroll
                for (int k = 0; k < 5; ++k) b.action_history[5 * (size_t)e + k] = 0.0f;
            }
        }
        prog = 0;
    }
    if (!lead) return;
    float o[6];
    observation(rt, yawc, cmdc, o);
    // compute_gogoro_reward
    bool felt;
    const float rew = gogoro_reward(o, ah, felt);
    const bool finished = prog >= p.max_episode_length - 1;
    const int64_t reset = (finished || felt) ? 1 : 0;
    // sensor noise (compute_obs_rwd :449-462)
    float nd[5];
    if (obs_draws) {
#pragma unroll
        for (int k = 0; k < 5; ++k) nd[k] = obs_draws[(size_t)e * 5 + k];
    } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) nd[k] = xch[le][GOGORO_NSLOT[k]];
    }
    float rr[6];
    noisy_observation(p, o, nd, imu, rr);
    // command resampling (:384-389)
    float su, yu;
    if (speed_draws) { su = speed_draws[e]; yu = yaw_draws[e]; }
    else { su = xch[le][24]; yu = xch[le][25]; }
    float yc = yawc;
    if (prog == p.yaw_freq_update) yc = u_aff(-F_PI, F_PI, yu);
    if (yc > F_PI) yc = yc - F_2PI;
    if (yc < -F_PI) yc = yc + F_2PI;
    if (!owner) return;
    b.progress_buf[e] = prog;
    float *bo = b.buffer_obs + 6 * (size_t)e;
    float *ob = b.obs_buf + 6 * (size_t)e;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        bo[k] = o[k];
        ob[k] = t_clamp(rr[k], -p.clip_obs, p.clip_obs);
    }
    b.rew_buf[e] = felt ? -100.0f : rew;
    b.reset_buf[e] = reset;
    if (prog == p.speed_freq_update) b.curent_speed[e] = u_aff(p.speed_range[0], p.speed_range[1], su);
    b.yaw_command[e] = yc;
    b.timeout_buf[e] = (prog >= p.max_episode_length - 1) && (reset != 0);
}

__device__ void philox_reset_draws(int e, uint32_t c_lo, uint32_t c_hi, uint32_t k0, uint32_t k1, float *r);

__global__ __launch_bounds__(256) void reset_idx_kernel(tg_gogoro_params p, tg_gogoro_buffers b, const int32_t *ids,
                                                        int n, const float *reset_draws, uint32_t c_lo, uint32_t c_hi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int e = ids[i];
    if (e < 0 || e >= p.num_envs) return;
    float r[TG_GOGORO_RESET_DRAWS];
    if (reset_draws) {
#pragma unroll
        for (int k = 0; k < TG_GOGORO_RESET_DRAWS; ++k) r[k] = reset_draws[(size_t)e * TG_GOGORO_RESET_DRAWS + k];
    } else {
        philox_reset_draws(e, c_lo, c_hi, (uint32_t)p.seed, (uint32_t)(p.seed >> 32), r);
    }
    reset_env(p, b, e, r);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        b.obs_buf[6 * (size_t)e + k] = 0.0f;
        b.buffer_obs[6 * (size_t)e + k] = 0.0f;
    }
}

__device__ void philox_reset_draws(int e, uint32_t c_lo, uint32_t c_hi, uint32_t k0, uint32_t k1, float *r) {
    U4 x0 = philox(U4{(uint32_t)e, c_lo, c_hi, 0x52535430u}, k0, k1);
    U4 x1 = philox(U4{(uint32_t)e, c_lo, c_hi, 0x52535431u}, k0, k1);
    U4 x2 = philox(U4{(uint32_t)e, c_lo, c_hi, 0x52535432u}, k0, k1);
    U4 x3 = philox(U4{(uint32_t)e, c_lo, c_hi, 0x52535433u}, k0, k1);
    U4 x4 = philox(U4{(uint32_t)e, c_lo, c_hi, 0x52535434u}, k0, k1);
    r[0] = u01(x0.x); r[1] = gauss(x0.y, x0.z); r[2] = u01(x0.w);
    r[3] = u01(x1.x); r[4] = u01(x1.y); r[5] = gauss(x1.z, x1.w);
    r[6] = gauss(x2.x, x2.y); r[7] = gauss(x2.z, x2.w);
    r[8] = gauss(x3.x, x3.y); r[9] = gauss(x3.z, x3.w);
    r[10] = u01(x4.x);
}

// one env per lane with a long dependent chain per lane: spread the envs over
// as many CUs as possible (16-lane workgroups up to 1024 workgroups)
static int env_threads(int n) {
    int t = 16;
    while (t < 256 && (n + t - 1) / t > 1024) t *= 2;
    return t;
}

int launch_gogoro_reset_idx(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const int32_t *ids, int n,
                            const float *reset_draws, uint64_t counter, hipStream_t stream) {
    if (n <= 0) return 0;
    const int t = env_threads(n);
    hipLaunchKernelGGL(reset_idx_kernel, dim3((n + t - 1) / t), dim3(t), 0, stream, p, b, ids, n, reset_draws,
                       (uint32_t)counter, (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

int launch_gogoro_pre(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const float *actions,
                      const float *pre_draws, uint64_t counter, hipStream_t stream) {
    const int t = env_threads(p.num_envs);
    dim3 grid((p.num_envs + t - 1) / t), block(t);
    hipLaunchKernelGGL(pre_kernel, grid, block, 0, stream, p, b, actions, pre_draws, (uint32_t)counter,
                       (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

int launch_gogoro_post(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const float *reset_draws,
                       const float *obs_draws, const float *speed_draws, const float *yaw_draws, uint64_t counter,
                       hipStream_t stream) {
    dim3 grid((p.num_envs + POST_EPB - 1) / POST_EPB), block(64);
    hipLaunchKernelGGL(post_kernel, grid, block, 0, stream, p, b, reset_draws, obs_draws, speed_draws, yaw_draws,
                       (uint32_t)counter, (uint32_t)(counter >> 32));
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

// ---------------------------------------------------------------- indexed setters
__global__ void scatter_rows_kernel(float *dst, const float *src, const int32_t *ids, int n, int row) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n * row) return;
    const int i = (int)(t / row), k = (int)(t % row);
    const size_t o = (size_t)ids[i] * row + k;
    dst[o] = src[o];
}
__global__ void mark_dirty_kernel(uint8_t *dirty, const int32_t *ids, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dirty[ids[i]] = 1;
}

int launch_scatter_rows(float *dst, const float *src, const int32_t *ids, int n, int row, hipStream_t stream) {
    if (n <= 0) return 0;
    size_t tot = (size_t)n * row;
    hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, dst, src, ids,
                       n, row);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_scatter_field(float *dst, const float *src, const int32_t *ids, int n, int row, hipStream_t stream) {
    return launch_scatter_rows(dst, src, ids, n, row, stream);
}
int launch_mark_dirty(uint8_t *dirty, const int32_t *ids, int n, hipStream_t stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(mark_dirty_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, dirty, ids, n);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

// ---------------------------------------------------------------- RNG test hook (tg_rng_fill)
// Block i = philox({i, counter lo, counter hi, 0}, seed): kind 0 the 4 raw
// words (bit patterns in the float slots), kind 1 u01 of each word, kind 2
// gauss(x, y), gauss(z, w) -- the very functions the task kernels draw with.
__global__ void rng_fill_kernel(int kind, uint32_t k0, uint32_t k1, uint32_t c_lo, uint32_t c_hi, float *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const U4 x = philox(U4{(uint32_t)i, c_lo, c_hi, 0u}, k0, k1);
    if (kind == 0) {
        uint32_t *o = reinterpret_cast<uint32_t *>(out) + 4 * (size_t)i;
        o[0] = x.x; o[1] = x.y; o[2] = x.z; o[3] = x.w;
    } else if (kind == 1) {
        float *o = out + 4 * (size_t)i;
        o[0] = u01(x.x); o[1] = u01(x.y); o[2] = u01(x.z); o[3] = u01(x.w);
    } else {
        float *o = out + 2 * (size_t)i;
        o[0] = gauss(x.x, x.y); o[1] = gauss(x.z, x.w);
    }
}

// ---------------------------------------------------------------- stale-LDS test hook (tg_debug_fill_lds)
// Every workgroup takes the whole 160 KB LDS of its CU and writes the pattern
// into every dword; with several workgroups per CU launched, every CU's LDS
// leaves the launch holding the pattern (LDS is not cleared between kernels)
constexpr int FILL_LDS_BYTES = 160 * 1024;
__global__ __launch_bounds__(256) void fill_lds_kernel(uint32_t pattern, uint32_t *sink) {
    extern __shared__ uint32_t lds_fill[];
    for (int i = threadIdx.x; i < FILL_LDS_BYTES / 4; i += blockDim.x) lds_fill[i] = pattern;
    __syncthreads();
    // one read back so the stores are not dead (the sink is never written in practice)
    if (lds_fill[(threadIdx.x * 37) % (FILL_LDS_BYTES / 4)] != pattern && sink) sink[0] = 1u;
}

int launch_fill_lds(uint32_t pattern, hipStream_t stream) {
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return TG_ERR_HIP;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        return TG_ERR_HIP;
    const uint64_t bit = 1ull << dev;
    if (!(attr_set.load(std::memory_order_acquire) & bit)) {
        if (hipFuncSetAttribute((const void *)fill_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                FILL_LDS_BYTES) != hipSuccess)
            return TG_ERR_HIP;
        attr_set.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(fill_lds_kernel, dim3(4 * ncu), dim3(256), FILL_LDS_BYTES, stream, pattern, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

int launch_rng_fill(int kind, uint64_t seed, uint64_t counter, float *out, int n, hipStream_t stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(rng_fill_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, kind, (uint32_t)seed,
                       (uint32_t)(seed >> 32), (uint32_t)counter, (uint32_t)(counter >> 32), out, n);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

}  // namespace tg
