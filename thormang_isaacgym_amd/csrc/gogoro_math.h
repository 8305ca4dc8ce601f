// gogoro_math.h -- the Gogoro task's per-env arithmetic shared by the
// separate post-physics kernel (gogoro_task.hip post_kernel) and the step
// kernel's fused epilogue (articulation.hip GogoroPost), so both evaluate the
// same fp32 operations in the reference's order
// (isaacgymenvs/tasks/gogoro_new.py:645-723: compute_gogoro_observations,
// compute_gogoro_reward; :474-601 reset_idx draws).
#pragma once
#include <hip/hip_runtime.h>
#ifndef __HIPCC_RTC__   // hipRTC (jit.cpp) provides the device math itself
#include <math.h>
#endif

#include "tg_kernels.h"

namespace tg {

#define F_PI 3.14159265358979323846f
#define F_2PI 6.28318530717958647692f

__device__ __forceinline__ float t_rem(float a, float b) {
#pragma clang fp contract(off) reassociate(off)
    float m = fmodf(a, b);
    if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
    return m;
}
__device__ __forceinline__ float t_clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ float u_aff(float lo, float hi, float u) {
#pragma clang fp contract(off) reassociate(off)
    return lo + u * (hi - lo);
}
__device__ __forceinline__ float n_aff(const float *mc, float r) {
#pragma clang fp contract(off) reassociate(off)
    return mc[0] + r * mc[1];
}

// compute_gogoro_observations (:692-723) on one root row [13]
__device__ __forceinline__ void observation(const float *root, float desired_yaw, float cmd, float *obs) {
#pragma clang fp contract(off) reassociate(off)
    const float x = root[3], y = root[4], z = root[5], w = root[6];
    float roll = t_rem(atan2f(2.0f * (w * x + y * z), w * w - x * x - y * y + z * z), F_2PI);
    float yaw = t_rem(atan2f(2.0f * (w * z + x * y), w * w + x * x - y * y - z * z), F_2PI);
    const float s = 2.0f * (w * w) - 1.0f;
    // quat_rotate_inverse(q, v) = v*s - cross(q,v)*w*2 + q*dot(q,v)*2
    const float *v = root + 7;
    float d = x * v[0] + y * v[1] + z * v[2];
    float lin_x = v[0] * s - (y * v[2] - z * v[1]) * w * 2.0f + x * d * 2.0f;
    const float *o = root + 10;
    float da = x * o[0] + y * o[1] + z * o[2];
    float ang_x = o[0] * s - (y * o[2] - z * o[1]) * w * 2.0f + x * da * 2.0f;
    float ang_z = o[2] * s - (x * o[1] - y * o[0]) * w * 2.0f + z * da * 2.0f;
    if (roll > F_PI) roll = roll - F_2PI;
    if (roll < -F_PI) roll = roll + F_2PI;
    if (yaw > F_PI) yaw = yaw - F_2PI;
    if (yaw < -F_PI) yaw = yaw + F_2PI;
    obs[0] = roll;
    obs[1] = ang_x;
    obs[2] = ang_z;
    obs[3] = lin_x;
    obs[4] = t_rem(desired_yaw - yaw + F_PI, F_2PI) - F_PI;
    obs[5] = cmd;
}

// compute_gogoro_reward (:645-684): the reward; felt = |roll| >= 0.30
__device__ __forceinline__ float gogoro_reward(const float *o, const float *ah, bool &felt) {
#pragma clang fp contract(off) reassociate(off)
    const float max_tilt = 0.30f;
    float tilt_err = t_clamp(o[0] / max_tilt, -1.0f, 1.0f);
    float yaw_err = t_clamp(o[4] / F_PI, -1.0f, 1.0f);
    float dtilt_err = t_clamp(o[1] / 0.3f, -1.0f, 1.0f);
    float y30 = yaw_err * 30.0f;
    float r1 = 1.0f / (1.0f + y30 * y30);
    float r2 = 1.0f - tilt_err * tilt_err;
    float r4 = 1.0f - dtilt_err * dtilt_err;
    float ce = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) ce += 1.0f - ah[k] * ah[k];
    felt = fabsf(o[0]) >= max_tilt;
    return r1 * 5.0f + r2 * 0.2f + r4 * 0.3f + ce * 0.5f;
}

// compute_obs_rwd's sensor noise (:449-462) on the clean observation o:
// nd = the 5 normal draws (imu filter, imu, imu, speed sensor, imu filter)
__device__ __forceinline__ void noisy_observation(const tg_gogoro_params &p, const float *o, const float *nd,
                                                  float imu_offset, float *rr) {
#pragma clang fp contract(off) reassociate(off)
#pragma unroll
    for (int k = 0; k < 6; ++k) rr[k] = o[k];
    rr[0] += n_aff(p.imu_filter_noise, nd[0]) + imu_offset;
    rr[1] += n_aff(p.imu_noise, nd[1]);
    rr[2] += n_aff(p.imu_noise, nd[2]);
    rr[3] = rintf(rr[4]);                     // quirk :457-458 (speed-sensor value discarded)
    rr[4] += n_aff(p.imu_filter_noise, nd[4]);
}

// The 9 Philox blocks of one env's post-physics step (5 reset, 3 sensor
// noise, 1 command resample; counter (e, c_lo, c_hi, key)).  Block l leaves
// three floats v[0..2] in exchange slots 3 l .. 3 l + 2; the reset draws are
// slots GOGORO_RSLOT, the noise draws GOGORO_NSLOT, the speed / yaw resample
// draws slots 24 / 25.
__device__ __forceinline__ void gogoro_post_block(int l, int e, uint32_t c_lo, uint32_t c_hi, uint32_t k0,
                                                  uint32_t k1, float *v) {
    const uint32_t key = l < 5 ? 0x52535430u + (uint32_t)l : (l < 8 ? 0x4F425330u + (uint32_t)(l - 5) : 0x434D4430u);
    const U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, key}, k0, k1);
    const float A = u01(x.x), B = gauss(x.x, x.y), C = gauss(x.y, x.z), Dd = u01(x.w), E = u01(x.y),
                F = gauss(x.z, x.w);
    v[0] = (l == 0 || l == 1 || l == 4 || l == 8) ? A : B;
    v[1] = l == 0 ? C : ((l == 1 || l == 8) ? E : F);
    v[2] = l == 0 ? Dd : F;
}
constexpr int GOGORO_RSLOT[TG_GOGORO_RESET_DRAWS] = {0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 12};
constexpr int GOGORO_NSLOT[5] = {15, 16, 18, 19, 21};

}  // namespace tg
