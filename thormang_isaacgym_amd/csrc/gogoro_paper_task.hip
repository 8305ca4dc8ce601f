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
//   paper_finish_kernel batch mean of the squared command differences
//                       (torch.mean without dim, :740, reward term 7; every
//                       workgroup sums the whole batch), rewards, resets,
//                       VecTask time_outs
// fp32 in the reference's operation order (compiled -ffp-contract=off).
#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

#include "../../include/tg_gogoro_paper.h"
#include "tg_kernels.h"
#include "generated/models.inc"
#include "articulation_kernels.h"   // CompLayout, tl_update: in-place seat composites

namespace tg {

using namespace paper;

// envs (one wavefront each) per workgroup of the pre / post kernels: N / 8
// workgroups rather than N, which the dispatcher would issue one by one
constexpr int PAPER_EPW = 8;
// an env's lanes are one wavefront: its LDS / memory hand-offs need only a
// wavefront-scope fence
__device__ __forceinline__ void p_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

__global__ __launch_bounds__(64 * PAPER_EPW) void paper_pre_kernel(tg_paper_params p, tg_paper_buffers b,
                                                                   const float *actions) {
    // every input in one batch; the shifted history stays in registers (lane =
    // slot) and the delayed command is taken from its lane
    static_assert(PC <= 64, "one history slot per lane");
    const int e = blockIdx.x * PAPER_EPW + threadIdx.x / 64, lane = threadIdx.x % 64;
    if (e >= p.num_envs) return;
    const int D = p.num_dof;
    float *h = b.command_history + PC * (size_t)e;
    const float a = p_clamp(actions[e], -1.0f, 1.0f);
    const float cmd = a * p.max_steering;
    const float hn = lane < PC - 1 ? h[lane + 1] : 0.0f;
    const int64_t delay = p.use_steer_delay ? b.steer_delay[e] : 0;
    const float speed = b.curent_speed[e];
    const float hv = lane < PC - 1 ? hn : cmd;
    int idx = PC - 3;
    if (p.use_steer_delay) idx = delay == 0 ? 0 : (int)(PC - delay);   // command_history[:, -steer_delay]; -0 selects slot 0
    const float steer = __shfl(hv, idx, 64);
    p_wave_sync();   // every lane's history read is done before the shifted history is stored
    if (lane < PC) h[lane] = hv;
    float *pt = b.pos_target + (size_t)D * e, *vt = b.vel_target + (size_t)D * e;
    for (int d = lane; d < D; d += 64) {
        pt[d] = d == p.dof_steer ? steer : 0.0f;
        vt[d] = d == p.dof_rear ? speed : 0.0f;
    }
    if (lane == 0) b.curent_command[e] = cmd;
}

// reset_idx for env e (:609-692), lane-parallel part: histories (zero_hist;
// the fused post kernel rewrites them in full anyway) and dof state
__device__ void paper_reset_lanes(const tg_paper_params &p, const tg_paper_buffers &b, int e, bool zero_hist) {
    const int lane = threadIdx.x % 64;
    const int D = p.num_dof;
    if (zero_hist) {
        for (int i = lane; i < PHO; i += 64) {
            b.obs_buf[(size_t)PHO * e + i] = 0.0f;
            b.buffer_obs[(size_t)PHO * e + i] = 0.0f;
            b.buffer_obs_noisy[(size_t)PHO * e + i] = 0.0f;
        }
    }
    if (lane < PC) b.command_history[PC * (size_t)e + lane] = 0.0f;
    for (int d = lane; d < D; d += 64) {
        b.dof_state[2 * ((size_t)e * D + d)] = b.thormang_pose[(size_t)e * D + d];
        b.dof_state[2 * ((size_t)e * D + d) + 1] = 0.0f;
    }
}

// reset_idx for env e (:609-692) by one wavefront
__device__ void paper_reset_env(const tg_paper_params &p, const tg_paper_buffers &b, int e, const float *rd,
                                uint32_t c_lo, uint32_t c_hi) {
    paper_reset_lanes(p, b, e, true);
    if (threadIdx.x % 64 != 0) return;
    float r[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) r[k] = p_draw(p, rd, 9, e, k, c_lo, c_hi, P_TAG_RESET);
    PaperLead L;
    reset_lead(p, b, e, r, b.root_reset + 13 * (size_t)e, L);
}

// M (comp non-null): the sim's model with in-place seat composites (codegen
// FUSED bit 4), void: resets mark their envs for a compose
// the batch sum of reward term 7 in the canonical order (TG_PAPER_T7_*; a
// block's sum from blk(c)), by threads 0 .. TG_PAPER_T7_THREADS - 1 of the
// workgroup; every thread of the workgroup calls it (one barrier)
constexpr int FIN_WG = 1024, T7T = TG_PAPER_T7_THREADS;
template <class BLK> __device__ __forceinline__ double t7_batch_sum(int nblk, BLK blk) {
    __shared__ double wsum[T7T / 64];
    const int t = threadIdx.x;
    if (t < T7T) {
        double s = 0.0;
        for (int c = t; c < nblk; c += T7T) s += blk(c);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
        if ((t & 63) == 0) wsum[t >> 6] = s;
    }
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < T7T / 64; ++w) tot += wsum[w];
    return tot;
}
// rb_out (M with the link-com block): the post-physics' rb_forces reduced to
// the next simulate's group wrenches by the env's wavefront after its own
// writes (rb_force_env, as rb_force_kernel would at the next simulate)
template <class M> constexpr bool paper_rb_fusable() {
    if constexpr (std::is_void<M>::value) return false;
    else return M::LCOM != 0 && M::NL <= 64 && M::NG <= 64;
}
template <class M, bool ON = paper_rb_fusable<M>()> struct PaperRb {
    __device__ static void run(const tg_paper_params &, const tg_paper_buffers &, int, float *, float *) {}
};
template <class M> struct PaperRb<M, true> {
    __device__ static void run(const tg_paper_params &p, const tg_paper_buffers &b, int e, float *comp, float *out) {
        __shared__ float T[PAPER_EPW][M::NL][12], F[PAPER_EPW][M::NL][10];
        const int wv = threadIdx.x / 64;
        // this wave's global writes (reset root / dofs / seat windows /
        // composite, pushes) before its lanes read them back
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        rb_force_env<M>(b.root, b.dof_state, comp, e, nullptr, b.rb_forces, nullptr, TG_ENV_SPACE, out,
                        threadIdx.x % 64, T[wv], F[wv], b.dof_props, p.num_envs);
    }
};

// fin: the step kernel formed the term-7 block sums already (PaperPre.t7, in
// b.scratch, tg_paper_step), so each workgroup sums the batch first, in the
// canonical order, and its envs end with their final rewards / resets: no
// finish launch (the host asks for it only when N is a multiple of
// PAPER_EPW: no thread returns before the barrier)
template <class M>
__global__ __launch_bounds__(64 * PAPER_EPW) void paper_post_kernel(tg_paper_params p, tg_paper_buffers b, const float *rd,
                                                        const float *nd, const float *sd, const float *yd,
                                                        const float *pd, uint32_t c_lo, uint32_t c_hi, float *comp,
                                                        int fin, float *rb_out) {
    static_assert(64 * PAPER_EPW >= T7T, "the canonical sum's threads");
    double tot = 0.0;
    if (fin) {
        const double *bs = reinterpret_cast<const double *>(b.scratch);
        tot = t7_batch_sum((p.num_envs + TG_PAPER_T7_BLK - 1) / TG_PAPER_T7_BLK, [&](int c) { return bs[c]; });
    }
    // Every HBM input of the env is issued in one batch at the start (the
    // lead lane's scalars and root-reset template, every lane's history
    // entries), so the kernel waits on memory once; a reset replaces them by
    // the reset values in registers.  The histories' command column and the
    // newest entry go through LDS rather than back through HBM.
    __shared__ float ob_[PAPER_EPW][PO], nz_[PAPER_EPW][PO], ch_[PAPER_EPW][PH];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int e = blockIdx.x * PAPER_EPW + wv;
    if (e >= p.num_envs) return;
    float *ob = ob_[wv], *nz = nz_[wv], *ch = ch_[wv];
    // the step's 8 Philox blocks, one per lane (reset 3, noise 2, speed, yaw,
    // push), so the lead lane only looks its draws up
    __shared__ float dr_[PAPER_EPW][8][4];
    float(*dr)[4] = dr_[wv];
    if (lane < 8) {
        const uint32_t tag = post_block_tag(lane);
        const U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, tag}, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
        dr[lane][0] = u01(x.x);
        dr[lane][1] = u01(x.y);
        dr[lane][2] = u01(x.z);
        dr[lane][3] = u01(x.w);
    }
    // draw k of a kind whose Philox blocks start at blk: replay array or the block
    auto draw = [&](const float *arr, int stride, int k, int blk) {
        return arr ? arr[(size_t)stride * e + k] : dr[blk + (k >> 2)][k & 3];
    };
    const bool lead = lane == 0;
    float *bo = b.buffer_obs + (size_t)PHO * e, *bn = b.buffer_obs_noisy + (size_t)PHO * e;
    const bool reset = b.reset_buf[e] != 0;
    const int64_t prog0 = b.progress_buf[e] + 1;
    float vc[3], vn[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int i = lane + 64 * j;
        vc[j] = vn[j] = 0.0f;
        if (i < PHO - PO) {
            vc[j] = bo[i + PO];
            vn[j] = bn[i + PO];
        }
    }
    PaperLead L;
    float tpl[13], old6 = 0.0f;
    if (lead) {
        const float *rt = b.root + 13 * (size_t)e, *tp = b.root_reset + 13 * (size_t)e;
#pragma unroll
        for (int k = 0; k < 13; ++k) {
            L.root[k] = rt[k];
            tpl[k] = tp[k];
        }
        L.speed = b.curent_speed[e];
        L.speed_off = b.curent_speed_offset[e];
        L.imu_off = b.curent_imu_x_offset[e];
        L.yaw_cmd = b.yaw_command[e];
        L.cmd = b.curent_command[e];
        L.delay = b.steer_delay[e];
        old6 = bo[(PH - 1) * PO + 6];
    }
    const int64_t prog = reset ? 0 : prog0;
    p_wave_sync();   // the Philox blocks
    if (reset) {
        paper_reset_lanes(p, b, e, false);
#pragma unroll
        for (int j = 0; j < 3; ++j) vc[j] = vn[j] = 0.0f;
        if (lead) {
            float r[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) r[k] = draw(rd, 9, k, 0);
            reset_lead<M>(p, b, e, r, tpl, L, comp);
            old6 = 0.0f;
        }
    } else if (lead) {
        b.progress_buf[e] = prog0;
    }
    if (lead) {
        float u[6], o[PO], l[PO];
#pragma unroll
        for (int k = 0; k < 6; ++k) u[k] = draw(nd, 6, k, 3);
        entries(p, L, old6, u, o, l);   // newest clean / noisy entries (:503-547)
#pragma unroll
        for (int k = 0; k < PO; ++k) { ob[k] = o[k]; nz[k] = l[k]; }
        b.speed_no_noise[e] = o[4];
    }
    p_wave_sync();
    // both histories shifted by one entry, the new one appended
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int i = lane + 64 * j;
        if (i < PHO) {
            if (i >= PHO - PO) {
                vc[j] = ob[i - (PHO - PO)];
                vn[j] = nz[i - (PHO - PO)];
            }
            if ((i % PO) == 1) vn[j] = 0.0f;   // noisy[:, :, 1] = 0
            if ((i % PO) == 6) ch[i / PO] = vc[j];
            bo[i] = vc[j];
            bn[i] = vn[j];
            b.obs_buf[(size_t)PHO * e + i] = vn[j];
        }
    }
    p_wave_sync();
    // reward term 7 partial: sum_t (a[t+1] - a[t])^2, a = act / 0.5
    float dsq = 0.0f;
    if (lane < PH - 1) {
        const float dd = ch[lane + 1] / 0.5f - ch[lane] / 0.5f;
        dsq = dd * dd;
    }
    dsq = p_wsum(dsq);
    if (lead) {
        if (!fin) b.scratch[e] = dsq;
        const float *last = ob;
        const float rew = reward15(p, last);
        if (fin) finish_env(p, b, e, tot, last[0], prog, rew);
        else b.rew_buf[e] = rew;
        commands(p, b, e, prog, L, last, draw(sd, 1, 0, 5), draw(yd, 1, 0, 6), draw(pd, 2, 0, 7), draw(pd, 2, 1, 7));
    }
    if (b.body_force) {
        float *wr = b.body_force + (size_t)6 * p.num_groups * e;
        for (int i = 6 + lane; i < 6 * p.num_groups; i += 64) wr[i] = 0.0f;
    }
    if (rb_out) PaperRb<M>::run(p, b, e, comp, rb_out);
}

// batch mean for reward term 7, then rewards, resets, time_outs of the
// workgroup's FIN_WG envs.  Every workgroup forms the whole batch sum itself
// (the per-env partials are 4 B/env and L2-resident, and every workgroup adds
// them in the same order, so all agree bit for bit): no second launch and no
// single-workgroup tail whose dependent loads run one after another.
__global__ __launch_bounds__(FIN_WG) void paper_finish_kernel(tg_paper_params p, tg_paper_buffers b) {
    const int t = threadIdx.x, n = p.num_envs;
    const int e = blockIdx.x * FIN_WG + t;
    // the env's own inputs first, so their latency overlaps the sum
    float tilt = 0.f, rew = 0.f;
    int64_t prog = 0;
    if (e < n) {
        tilt = b.buffer_obs[(size_t)PHO * e + (PH - 1) * PO];
        prog = b.progress_buf[e];
        rew = b.rew_buf[e];
    }
    // the per-env partials of the post kernel, block sums formed here
    const double tot = t7_batch_sum((n + TG_PAPER_T7_BLK - 1) / TG_PAPER_T7_BLK, [&](int c) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < TG_PAPER_T7_BLK; ++i) {
            const int k = c * TG_PAPER_T7_BLK + i;
            s += (double)(k < n ? b.scratch[k] : 0.0f);
        }
        return s;
    });
    if (e >= n) return;
    finish_env(p, b, e, tot, tilt, prog, rew);
}

__global__ __launch_bounds__(64) void paper_reset_idx_kernel(tg_paper_params p, tg_paper_buffers b, const int32_t *ids,
                                                             const float *rd, uint32_t c_lo, uint32_t c_hi) {
    const int e = ids[blockIdx.x];
    if (e < 0 || e >= p.num_envs) return;
    paper_reset_env(p, b, e, rd, c_lo, c_hi);
}

int launch_paper_pre(const tg_paper_params &p, const tg_paper_buffers &b, const float *actions, hipStream_t s) {
    hipLaunchKernelGGL(paper_pre_kernel, dim3((p.num_envs + PAPER_EPW - 1) / PAPER_EPW), dim3(64 * PAPER_EPW), 0, s, p,
                       b, actions);
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}
int launch_paper_post(const tg_paper_params &p, const tg_paper_buffers &b, const float *rd, const float *nd,
                      const float *sd, const float *yd, const float *pd, uint64_t counter, hipStream_t s,
                      uint64_t model_hash, float *comp, bool *inplace, bool fin, float *rb_out, bool *rb_done) {
    const dim3 grid((p.num_envs + PAPER_EPW - 1) / PAPER_EPW), block(64 * PAPER_EPW);
    const uint32_t lo = (uint32_t)counter, hi = (uint32_t)(counter >> 32);
    bool done = false;
#define TG_PAPER_POST(MODEL)                                                                                  \
    if constexpr ((MODEL::FUSED & 4) != 0 && MODEL::NTL > 0) {                                              \
        if (!done && comp && model_hash == MODEL::hash) {                                                    \
            const bool rb = rb_out && b.rb_forces && paper_rb_fusable<MODEL>();                                \
            hipLaunchKernelGGL(paper_post_kernel<MODEL>, grid, block, 0, s, p, b, rd, nd, sd, yd, pd, lo, hi, comp, \
                               (int)fin, rb ? rb_out : nullptr);                                     \
            if (rb_done) *rb_done = rb;                                                                      \
            done = true;                                                                                     \
        }                                                                                                    \
    }
    TG_FOR_EACH_MODEL(TG_PAPER_POST)
#undef TG_PAPER_POST
    if (inplace) *inplace = done;
    if (!done) {
        if (rb_done) *rb_done = false;
        hipLaunchKernelGGL(paper_post_kernel<void>, grid, block, 0, s, p, b, rd, nd, sd, yd, pd, lo, hi, nullptr, (int)fin,
                           nullptr);
    }
    if (!fin) hipLaunchKernelGGL(paper_finish_kernel, dim3((p.num_envs + FIN_WG - 1) / FIN_WG), dim3(FIN_WG), 0, s, p, b);
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
