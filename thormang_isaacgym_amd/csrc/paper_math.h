// paper_math.h -- the GogoroPaper task's per-env arithmetic shared by the
// separate post-physics kernel (gogoro_paper_task.hip paper_post_kernel) and
// the step kernel's fused epilogue (articulation_kernels.h PaperPost), so both
// evaluate the same fp32 operations in the reference's order
// (isaacgymenvs/tasks/gogoro_realistic_turning_sim_paper.py: reset_idx
// :609-692, observation histories :503-547, compute_gogoro_observations
// :771-808, compute_gogoro_reward :714-762, command changes :402-417, head
// pushes :442-459).  Every function turns fp contraction and reassociation
// off itself: the epilogue's unit is compiled -ffast-math for the physics.
#pragma once
#include <hip/hip_runtime.h>
#ifndef __HIPCC_RTC__   // hipRTC (jit.cpp) provides the device math itself
#include <math.h>
#endif

#include "tg_kernels.h"

namespace tg {
namespace paper {

// std::is_void without <type_traits> (hipRTC units, jit.cpp)
template <class T> struct IsVoid { static constexpr bool value = false; };
template <> struct IsVoid<void> { static constexpr bool value = true; };

#define P_PI 3.14159265358979323846f
#define P_2PI 6.28318530717958647692f
constexpr int PH = TG_PAPER_HIST, PO = TG_PAPER_OBS, PC = TG_PAPER_CMD_HIST, PHO = PH * PO;

// Philox stream tags of the draw kinds (4 draws per counter block)
constexpr uint32_t P_TAG_RESET = 0x50415052u, P_TAG_NOISE = 0x50414e5au, P_TAG_SPEED = 0x50415344u,
                   P_TAG_YAW = 0x50415957u, P_TAG_PUSH = 0x50415055u;
// the post-physics' 8 Philox blocks (reset 3, noise 2, speed, yaw, push):
// the tag of block k
__device__ __forceinline__ uint32_t post_block_tag(int k) {
    return k < 3 ? P_TAG_RESET + k : k < 5 ? P_TAG_NOISE + (k - 3) : k == 5 ? P_TAG_SPEED : k == 6 ? P_TAG_YAW : P_TAG_PUSH;
}

__device__ __forceinline__ float p_rem(float a, float b) {
#pragma clang fp contract(off) reassociate(off)
    float m = fmodf(a, b);
    if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
    return m;
}
__device__ __forceinline__ float p_clamp(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ float p_aff(const float *b, float u) {
#pragma clang fp contract(off) reassociate(off)
    return b[0] + u * (float)((double)b[1] - (double)b[0]);
}

// the per-env values the post-physics reads, held by the env's lead lane
struct PaperLead {
    float root[13];
    float speed, speed_off, imu_off, yaw_cmd, cmd;
    int64_t delay;
};

// reset_idx for env e, lead-lane part: the draws and the scalar state, written
// to HBM and returned in L (tpl: the env's root reset template)
// (M: a model whose seat chain is a set of translating locks and comp its
// composite cache: the new seat windows update the composite in place
// (tl_update) instead of marking the env for a compose; M = void: mark it.
// ext: the composite's translating-lock extension already in LDS, or null:
// read from comp)
template <class M = void>
__device__ __forceinline__ void reset_lead(const tg_paper_params &p, const tg_paper_buffers &b, int e, const float *r,
                                           const float *tpl, PaperLead &L, float *comp = nullptr,
                                           const float *ext = nullptr) {
#pragma clang fp contract(off) reassociate(off)
    const int D = p.num_dof;
    const size_t ND = (size_t)p.num_envs * D;
    L.speed = p_aff(p.speed_range, r[0]);
    L.delay = (int64_t)p_aff(p.command_delay, r[1]);
    b.curent_speed[e] = L.speed;
    b.steer_delay[e] = L.delay;
    b.steer_offsets[e] = p_aff(p.steering_offset, r[2]);
    float *pz = b.perturbation + (size_t)(p.perturbation_stride ? p.perturbation_stride : 3) * e;
    pz[0] = 0.0f;
    pz[1] = 0.0f;
    pz[2] = 0.0f;
    L.speed_off = p_aff(p.speed_sensor_offset, r[3]);
    b.curent_speed_offset[e] = L.speed_off;
    float *root = b.root + 13 * (size_t)e;
#pragma unroll
    for (int k = 0; k < 13; ++k) L.root[k] = tpl[k];
    L.root[2] = p.spawn_z;
    L.root[3] = 0.0f; L.root[4] = 0.0f; L.root[5] = 0.0f; L.root[6] = 1.0f;
#pragma unroll
    for (int k = 7; k < 13; ++k) L.root[k] = 0.0f;
    if (p.debug_start_speed) {
        L.root[7] = p.start_speed * cosf(0.0f);
        L.root[8] = p.start_speed * sinf(0.0f);
    }
#pragma unroll
    for (int k = 0; k < 13; ++k) root[k] = L.root[k];
    L.imu_off = p_aff(p.imu_x_offset, r[4]);
    b.curent_imu_x_offset[e] = L.imu_off;
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
        // (a drive gain: read by the step kernel directly, no compose needed --
        // but the generic path keeps marking the env)
        if (!comp) b.env_dirty[e] = 1;
    }
    if (!p.center_robot) {
        const int seat[3] = {p.dof_base_x, p.dof_base_y, p.dof_base_z};
        const float *rg[3] = {p.seat_offset_x_range, p.seat_offset_y_range, p.seat_offset_z_range};
        float lo[3], hi[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = p_aff(rg[k], r[6 + k]);
            hi[k] = (float)((double)lo[k] + 0.0001);
            prop[TG_PROP_DRIVE_MODE * ND + seat[k]] = 0.0f;
            prop[TG_PROP_LOWER * ND + seat[k]] = lo[k];
            prop[TG_PROP_UPPER * ND + seat[k]] = hi[k];
        }
        bool inplace = false;
        if constexpr (!IsVoid<M>::value) {
            if constexpr (M::NTL > 0) {
                if (comp) {
                    // the seat windows only translate the rider: its composite
                    // from the moments the last compose stored (tl_update) at
                    // the new window centres, as compose_env pins them
                    float qn[M::NTL];
#pragma unroll
                    for (int k = 0; k < M::NTL; ++k) {
                        qn[k] = 0.f;
#pragma unroll
                        for (int j = 0; j < 3; ++j)
                            if (seat[j] == M::tl_dof[k]) qn[k] = 0.5f * (lo[j] + hi[j]);
                    }
                    float *c = comp + (size_t)e * M::KC;
                    tl_update<M>(c, ext ? ext : c + CompLayout<M>::ext(), qn);
                    inplace = true;
                }
            }
        }
        if (!inplace) b.env_dirty[e] = 1;
    }
    b.progress_buf[e] = 0;
    b.reset_buf[e] = 0;
    b.curent_command[e] = 0.0f;
    b.yaw_command[e] = 0.0f;
    b.speed_no_noise[e] = 0.0f;
    L.cmd = 0.0f;
    L.yaw_cmd = 0.0f;
}

// compute_gogoro_observations (:771-808)
__device__ __forceinline__ void observe(const float *root, float desired_yaw, float command, float delay_norm,
                                        float *obs) {
#pragma clang fp contract(off) reassociate(off)
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

// the newest clean (o) and noisy (l) history entries of the lead lane's env
// (:503-547), from its post-reset values L, the previous newest command entry
// old6 and the 6 noise draws u
__device__ __forceinline__ void entries(const tg_paper_params &p, const PaperLead &L, float old6, const float *u,
                                        float *o, float *l) {
#pragma clang fp contract(off) reassociate(off)
    const float dn = (float)((double)p.command_delay[1] - (double)p.command_delay[0]);
    const float dl = (float)(L.delay - (int64_t)p.command_delay[0]) / dn;
    observe(L.root, L.yaw_cmd, L.cmd, dl, o);
    const float dcmd = old6 - o[6];   // clean[-2][6] - clean[-1][6] after the shift
#pragma unroll
    for (int k = 0; k < PO; ++k) l[k] = o[k];
    l[0] += p_aff(p.imu_filter_noise, u[0]);
    l[1] += p_aff(p.imu_filter_noise, u[1]);
    l[0] += L.imu_off;
    l[2] += p_aff(p.imu_noise, u[2]);
    l[3] += p_aff(p.imu_noise, u[3]);
    l[4] += p_aff(p.speed_sensor_noise, u[4]);
    l[4] += L.speed_off;
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
}

// reward terms 1-5 (:722-746) on the newest clean entry
__device__ __forceinline__ float reward15(const tg_paper_params &p, const float *last) {
#pragma clang fp contract(off) reassociate(off)
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
    return r1 * 0.45f + r2 * 0.1f + r4 * 0.35f + r5 * 2.0f;
}

// rewards, resets, time_outs of env e from its reward terms 1-5 and the batch
// sum of reward term 7's partials (tot)
__device__ __forceinline__ void finish_env(const tg_paper_params &p, const tg_paper_buffers &b, int e, double tot,
                                           float tilt, int64_t prog, float rew) {
#pragma clang fp contract(off) reassociate(off)
    const float r7 = 1.0f - (float)(tot / ((double)p.num_envs * (PH - 1)));
    const bool finished = prog >= p.max_episode_length - 1;
    const bool felt = fabsf(tilt) >= p.max_tilt;
    float r = rew + r7 * 0.2f;
    r = r < 0.0f ? 0.0f : r;
    b.rew_buf[e] = felt ? -1.0f : r;
    const bool rs = finished || felt;
    b.reset_buf[e] = rs ? 1 : 0;
    b.timeout_buf[e] = finished && rs;
}

// command changes (:402-417) and head pushes (:442-459) of the lead lane's env,
// the root-group wrench when the task asks for one; su, yu: the speed and yaw
// draws, px, pz: the push draws
__device__ __forceinline__ void commands(const tg_paper_params &p, const tg_paper_buffers &b, int e, int64_t prog,
                                         const PaperLead &L, const float *last, float su, float yu, float px,
                                         float pz) {
#pragma clang fp contract(off) reassociate(off)
    if (prog == p.speed_freq_update) b.curent_speed[e] = p_aff(p.speed_range, su);
    float yc = L.yaw_cmd;
    if (prog == p.yaw_freq_update) yc = -P_PI + yu * (float)(2.0 * 3.14159265358979323846);
    yc = yc > P_PI ? yc - (float)(3.14159265358979323846 * 2) : yc;
    yc = yc < -P_PI ? yc + (float)(3.14159265358979323846 * 2) : yc;
    b.yaw_command[e] = yc;
    float *pert = b.perturbation + (size_t)(p.perturbation_stride ? p.perturbation_stride : 3) * e;
    if (p.push_robot && e < p.push_max_envs && (prog + 1) % p.push_interval == 0) {
        const float yaw = last[1];
        const float xf = (px * 2.0f - 1.0f) * p.push_force;
        const float zf = -(pz * p.push_force);
        pert[0] = xf * cosf(yaw + P_PI / 2.0f);
        pert[1] = xf * sinf(yaw + P_PI / 2.0f);
        pert[2] = zf;
    }
    if (b.body_force) {   // root-group wrench: force at the head COM
        const float x = L.root[3], y = L.root[4], z = L.root[5], w = L.root[6];
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

}  // namespace paper
}  // namespace tg
