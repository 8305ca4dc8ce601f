// Internal kernel argument blocks and launchers shared by the C-ABI host code
// (tgsim_api.cpp) and the kernel translation units.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#ifndef __HIPCC_RTC__
#include <string>
#endif

#include "../../include/tg_gogoro.h"
#include "../../include/tg_gogoro_paper.h"
#include "../../include/tg_walk.h"
#include "../../include/tgsim.h"

namespace tg {

constexpr int TG_PM_MAX_DOF = 64;   // prologue lanes: one wavefront per env, lane = dof

// optional Gogoro pre-physics prologue of the compose launch (tg_gogoro_step)
struct GogoroPre {
    const float *actions;     // [N] (null: none)
    float *action_history, *curent_command, *pos_target, *vel_target;
    const float *steer_offsets, *curent_speed;
    const float *pre_draws;   // [N] replayed steering-noise N(0,1) draws, or null (Philox)
    float clip_actions, max_steering_change, max_steering, noise_mean, noise_std;
    int dof_steer, dof_rear;
    int absolute_steer;       // INCREMENTAL_STEER = False (tg_gogoro_params.absolute_steer)
    uint32_t k0, k1, c_lo, c_hi;
};

// the GogoroPaper pre-physics (paper_pre_kernel) as a compose prologue:
// one wavefront per env, lane = command-history slot / dof
struct PaperPre {
    const float *actions;     // [N] (null: none)
    float *command_history;   // [N, TG_PAPER_CMD_HIST]
    const int64_t *steer_delay;
    const float *curent_speed;
    float *curent_command, *pos_target, *vel_target;
    float max_steering;
    int use_steer_delay, dof_steer, dof_rear;
    // reward term 7's partials, formed here for a post launch that finishes
    // the batch itself (t7 null: the post kernel forms them): the sum over
    // each block of TG_PAPER_T7_BLK envs (one step-kernel workgroup)
    const float *buffer_obs;   // [N, TG_PAPER_HIST * TG_PAPER_OBS] clean history
    const int64_t *reset_buf;  // [N]
    double *t7;                // [ceil(N / TG_PAPER_T7_BLK)] block sums
};
// the canonical order of the term-7 batch sum (paper_post_kernel with the
// finish inline, paper_finish_kernel): per block of TG_PAPER_T7_BLK envs the
// partials added in env order (double); thread t of TG_PAPER_T7_THREADS adds
// blocks t, t + TG_PAPER_T7_THREADS, ...; xor-butterfly per wavefront; the
// wavefront sums in order
#define TG_PAPER_T7_BLK 16
#define TG_PAPER_T7_THREADS 512

struct StepArgs {
    int N, D;
    float h;
    int substeps;
    float gx, gy, gz;
    float lin_damp, ang_damp, max_depen, rest, margin, ground_mu, baumgarte, lim_k, lim_c;
    float coff;                    // physx.contact_offset (contact_row_phi); <= 0: every point speculative
    int iters, viters, fix_base;   // biased (position) and bias-free (velocity) PGS sweeps
    int tgs;                       // solver_type 1: position iterations as sub-steps (step_par.h PGS)
    float *root;              // [N,13]
    float *dof;               // [N*D,2]
    const float *pos_tgt;     // [N,D]
    const float *vel_tgt;     // [N,D]
    const float *act;         // [N,D] or null
    const float *props;       // [TG_NUM_PROPS,N,D]
    const float *force;       // [N,G,6] or null
    const float *shape_mu;    // [N,S]
    const float *mass_scale;  // [N,L] or null
    float *comp;              // [KC,N]
    uint8_t *dirty;           // [N]
    int *err;                 // [1] sticky state-error flag (compose: a locked dof's window widened), read by tg_sync
    const float *hf;          // terrain heights [rows, cols] or null (z = 0 plane)
    int hf_rows, hf_cols;
    float hf_hs, hf_vs, hf_ox, hf_oy, hf_mu;
    // optional prologue of the compose launch (tg_walk_step): the task's
    // actions -> clamp(+-pm_clip) -> PD position targets pm_default + pm_scale*a
    // (null pm_actions: none)
    const float *pm_actions;  // [N,D]
    float *pm_act_out;        // [N,D] clamped actions
    float *pm_tgt_out;        // [N,D] position targets
    float pm_scale, pm_clip;
    float pm_default[TG_PM_MAX_DOF];
    GogoroPre gp;
    PaperPre pp;
    // pm_in_step: the walk prologue runs inside the step kernel instead (the
    // drive targets are formed from pm_actions where pass 2a loads them, the
    // fused WalkPost epilogue writes pm_act_out / pm_tgt_out); skip_compose:
    // no env can be dirty and no compose prologue is requested, so the
    // compose launch is left out (tgsim_api.cpp dirty_possible)
    int pm_in_step, skip_compose;
    // compose_list: compose only the envs in clist[0, *ccount) (ccount null: none)
    // -- a fused epilogue's resets -- with compose_list_kernel; cnext (or null):
    // the reset count the coming epilogue appends to, zeroed by the compose launch
    int compose_list;
    const int *clist, *ccount;
    int *cnext;
    // gp_in_step: the Gogoro pre-physics (gp) runs at the start of the step
    // kernel (lead lane; values through the env's LDS) instead of in compose
    int gp_in_step;
    // cuni (or null): a device flag, 1 while every env's composite block
    // equals env 0's (uniform_check_kernel after each full compose); the step
    // kernel then reads env 0's block for every env, so the per-env cache
    // costs L2 hits, not HBM reads (models whose task kernels edit composites
    // in place never get the flag).  DOF property rows are always per env.
    int *cuni;
    // pp_in_step: the GogoroPaper pre-physics (pp) likewise (models with the
    // pre-physics slots, codegen FUSED bits 2 | 4)
    int pp_in_step;
    // a pending apply_rigid_body_force_tensors reduced by the (full) compose
    // launch of this simulate (rbf_forces null: none)
    const float *rbf_forces, *rbf_torques;
    int rbf_space;
    float *rbf_out;
};

// tg_walk_step's fused post-physics epilogue (articulation.hip WalkPost)
struct WalkPostArgs {
    tg_walk_params p;
    tg_walk_buffers b;
    const float *reset_draws, *push_draws;
    uint32_t c_lo, c_hi;
};
// tg_gogoro_step's fused post-physics epilogue (articulation.hip GogoroPost)
struct GogoroPostArgs {
    tg_gogoro_params p;
    tg_gogoro_buffers b;
    uint32_t c_lo, c_hi;
    int *reset_list, *reset_count;   // [N] ids of the envs reset (and made dirty) / their count, or null
    int tl_inplace;                  // the epilogue updates a reset env's composite itself (M::NTL > 0)
    // replayed draws (include/tg_gogoro.h layouts), each null for Philox
    const float *reset_draws, *obs_draws, *speed_draws, *yaw_draws;
};
// tg_paper_step's fused post-physics epilogue (articulation_kernels.h
// PaperPost): the whole GogoroPaper step in one launch.  Reward term 7's
// batch sum needs every workgroup's block sum: each workgroup publishes its
// own in the prologue (PaperPre.t7) and adds one to *t7_count; the epilogue
// waits until the count reaches t7_target (the host's running total, one
// launch's worth of blocks more than before it), so every workgroup of the
// launch must be resident at once (the host checks the grid against the CUs)
struct PaperPostArgs {
    tg_paper_params p;
    tg_paper_buffers b;
    uint32_t c_lo, c_hi;   // the post-physics call's Philox counter
    float *rb_out;         // b.rb_forces reduced to the next simulate's group wrenches [N,G,6], or null
    unsigned *t7_count;    // arrivals of the term-7 block sums (monotonic over launches)
    unsigned t7_target;
    int nblk;              // term-7 blocks (workgroups) of this launch
};
#ifndef __HIPCC_RTC__   // host launchers (not part of a hipRTC unit, jit.cpp)
// compose + step kernel with the GogoroPaper post-physics fused in; returns 1
// when the model has no such instantiation
int launch_step_paper(uint64_t hash, const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream,
                      hipEvent_t ev_begin = nullptr, hipEvent_t ev_end = nullptr);
// compose + step kernel with the Gogoro post-physics fused in; returns 1 when
// the model has no such instantiation
int launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                       hipEvent_t ev_begin = nullptr, hipEvent_t ev_end = nullptr);
// compose + step kernel with the walk post-physics fused in; returns 1 (nothing
// launched) when the model / ground has no fused instantiation
int launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                     hipEvent_t ev_begin = nullptr, hipEvent_t ev_end = nullptr);

// ev_begin / ev_end (optional) are recorded around the step kernel itself
int launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin = nullptr,
                hipEvent_t ev_end = nullptr);
int compiled_hashes(uint64_t *out, int cap);
int launch_body_states(uint64_t hash, const float *root, const float *dof, int n, float *out, hipStream_t stream);
// per-link forces / torques [N*L,3] -> group wrenches [N,G,6] (rb_force_kernel)
int launch_rb_forces(uint64_t hash, const float *root, const float *dof, const float *comp, int n,
                     const float *mass_scale, const float *forces, const float *torques, int space, float *out,
                     const float *props, hipStream_t stream);
int model_kc(uint64_t hash);
int model_tl(uint64_t hash);
int model_epb(uint64_t hash);   // envs per step-kernel workgroup of a compiled model (0: not compiled in)
int model_fused(uint64_t hash);   // codegen FUSED bits of a compiled model (0: none / not compiled in)
int launch_compose_only(uint64_t hash, const StepArgs &a, hipStream_t stream);   // every dirty env, no step   // translating locks of a compiled model (codegen translating_locks), 0 otherwise

// run-time compiled models (jit.cpp, tg_model_jit): the launchers above fall
// through to these when no compiled-in specialisation matches the hash
int jit_compile(uint64_t hash, const char *struct_name, const char *model_source, const char *include_dir,
                const char *cache_dir, std::string &err);
bool jit_has(uint64_t hash);
int jit_kc(uint64_t hash);
int jit_launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end);
int jit_launch_body_states(uint64_t hash, const float *root, const float *dof, int n, float *out, hipStream_t stream);
int jit_launch_rb_forces(uint64_t hash, const float *root, const float *dof, const float *comp, int n,
                         const float *mass_scale, const float *forces, const float *torques, int space, float *out,
                         const float *props, hipStream_t stream);

int launch_gogoro_pre(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const float *actions,
                      const float *pre_draws, uint64_t counter, hipStream_t stream);
int launch_gogoro_post(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const float *reset_draws,
                       const float *obs_draws, const float *speed_draws, const float *yaw_draws, uint64_t counter,
                       hipStream_t stream);

int launch_gogoro_reset_idx(const tg_gogoro_params &p, const tg_gogoro_buffers &b, const int32_t *ids, int n,
                            const float *reset_draws, uint64_t counter, hipStream_t stream);

int launch_paper_pre(const tg_paper_params &p, const tg_paper_buffers &b, const float *actions, hipStream_t s);
// model_hash / comp: the sim's model and composite cache -- a model with
// in-place seat composites (codegen FUSED bit 4) gets them and *inplace is set
int launch_paper_post(const tg_paper_params &p, const tg_paper_buffers &b, const float *rd, const float *nd,
                      const float *sd, const float *yd, const float *pd, uint64_t counter, hipStream_t s,
                      uint64_t model_hash = 0, float *comp = nullptr, bool *inplace = nullptr,
                      bool fin = false, float *rb_out = nullptr, bool *rb_done = nullptr);
int launch_paper_reset_idx(const tg_paper_params &p, const tg_paper_buffers &b, const int32_t *ids, int n,
                           const float *rd, uint64_t counter, hipStream_t s);
int launch_walk_pre(const tg_walk_params &p, const tg_walk_buffers &b, const float *actions, hipStream_t s);
int launch_walk_post(const tg_walk_params &p, const tg_walk_buffers &b, const float *rd, const float *pd,
                     uint64_t counter, hipStream_t s);
int launch_walk_reset_idx(const tg_walk_params &p, const tg_walk_buffers &b, const int32_t *ids, int n,
                          const float *rd, uint64_t counter, hipStream_t s);

// indexed scatter: dst[ids[i]*row + k] = src[ids[i]*row + k]
int launch_scatter_rows(float *dst, const float *src, const int32_t *ids, int n, int row, hipStream_t stream);
// dst[f][ids[i]][k] (field f of a [F,N,row] array) = src[ids[i]*row + k]
int launch_scatter_field(float *dst, const float *src, const int32_t *ids, int n, int row, hipStream_t stream);
int launch_mark_dirty(uint8_t *dirty, const int32_t *ids, int n, hipStream_t stream);
// tg_rng_fill test hook (gogoro_task.hip): n Philox blocks, counter (i, c_lo, c_hi, 0)
int launch_rng_fill(int kind, uint64_t seed, uint64_t counter, float *out, int n, hipStream_t stream);
int launch_fill_lds(uint32_t pattern, hipStream_t stream);

#endif   // __HIPCC_RTC__

// ---------------------------------------------------------------- Philox4x32-10
struct U4 {
    uint32_t x, y, z, w;
};
// Random123's philox4x32 with 10 rounds (Salmon et al., SC'11): round
// (hi0,lo0) = M0 * c0, (hi1,lo1) = M1 * c2, c' = (hi1^c1^k0, lo1, hi0^c3^k1, lo0),
// then the Weyl key bump.  Host + device: the host copy backs tg_philox4x32_10
// (the known-answer test against Random123's kat_vectors, tests/test_rng.py).
__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}
__host__ __device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0 = mulhi32(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        uint32_t hi1 = mulhi32(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
// Box-Muller from two 32-bit draws
__device__ __forceinline__ float gauss(uint32_t a, uint32_t b) {
    float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777217.0f);
    float u2 = u01(b);
    return sqrtf(-2.0f * __logf(u1)) * __cosf(6.28318530718f * u2);
}

// ThormangWalk reset draw k of env e (replay array or in-kernel Philox, 4 draws per counter)
__device__ __forceinline__ float walk_draw(const tg_walk_params &p, const float *reset_draws, int e, int k,
                                           uint32_t c_lo, uint32_t c_hi) {
    const int n = 4 + 2 * p.num_dof;
    if (reset_draws) return reset_draws[(size_t)n * e + k];
    const U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, 0x57524530u + (uint32_t)(k >> 2)}, (uint32_t)p.seed,
                        (uint32_t)(p.seed >> 32));
    const uint32_t c = (k & 3) == 0 ? x.x : (k & 3) == 1 ? x.y : (k & 3) == 2 ? x.z : x.w;
    return u01(c);
}

}  // namespace tg
