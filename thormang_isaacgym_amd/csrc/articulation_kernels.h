// articulation_kernels.h -- the model-generic kernel templates of the
// articulation step (compose, step_par_kernel with its task epilogues, link
// states, rigid-body force reduction).  Included by articulation.hip, which
// instantiates them for the models compiled into libtgsim.so, and compiled at
// run time by hipRTC (jit.cpp) for a model loaded from a URDF that is not
// compiled in.  See articulation.hip for the algorithm overview.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "../../include/tgsim.h"
#include "gogoro_math.h"
#include "tg_math.h"
#include "tg_kernels.h"

namespace tg {

// per-env composite cache layout (SoA, [KC][N])
// Per-env composite cache, env-major ([N][KC] floats): group g's block of 24
// floats (joint placement R (9) + t (3), then mass, com (3), inertia about the
// com (6), 2 pad) at 24 g, then 12 floats (R, t) per contact shape.  A lane
// takes a group's 22 inputs with 6 16-byte loads from one base address.
// Models with translating locks (codegen translating_locks: the Gogoro seat
// chain) append an extension at ext(): the lock group's mass moments at the
// composed lock positions -- mass, first moment S (3), second moment about the
// group origin Io (6: xx yy zz xy xz yz, rotated link inertias included) --
// then per lock k (xk): its composed position q0, the mass m_k and first
// moment S_k of the links below it, its axis w_k in the group frame; then the
// placement translation t0 (3) of every group hanging below a lock (xag) and of
// every shape of the lock group below one (xash), as composed.
template <class M> struct CompLayout {
    static constexpr int GB = 24;
    static constexpr int xtree(int g) { return GB * g; }
    static constexpr int inertia(int g) { return GB * g + 12; }
    static constexpr int shape(int s) { return GB * M::NG + 12 * s; }
    static constexpr int ext() { return GB * M::NG + 12 * M::NS; }
    static constexpr int xk(int k) { return ext() + 10 + 8 * k; }
    static constexpr int xag(int j) { return ext() + 10 + 8 * M::NTL + 3 * j; }
    static constexpr int xash(int j) { return ext() + 10 + 8 * M::NTL + 3 * M::NAG + 3 * j; }
    // link com block (M::LCOM): com of link l in its group's joint-aligned frame at lcom(l)
    static constexpr int lcom(int l) { return ext() + M::KX + 3 * l; }
    static_assert(M::KC == GB * M::NG + 12 * M::NS + M::KX + (M::LCOM ? ((3 * M::NL + 3) & ~3) : 0), "codegen KC");
    static_assert(M::NTL == 0 || 10 + 8 * M::NTL + 3 * (M::NAG + M::NASH) <= M::KX, "codegen KX");
};

__device__ __forceinline__ float prop(const StepArgs &a, int f, int e, int d) {
    return a.props[((size_t)f * a.N + e) * a.D + d];
}

// ---------------------------------------------------------------- compose
// Per-env group composites from the locked joint positions (centre of each
// lock window) and the per-link mass scale (domain randomisation).  One
// wavefront per env (envs that are not dirty exit at once): link poses in
// their group-root frame level by level (lane = link), per-link mass terms in
// parallel, then lane g sums group g's links in link order (deterministic, the
// order of oracle/physics_ref.c) and writes the group's cache rows.
#ifdef TG_SECTION_PROF
static __device__ unsigned long long tg_cprof_acc[8];   // compose sections, lane 0 of every composed env
#define TG_CPROF_INIT unsigned long long tg_c0 = clock64();
#define TG_CPROF(k)                                                              \
    {                                                                            \
        const unsigned long long t1 = clock64();                                \
        if (threadIdx.x % 64 == 0) atomicAdd(&tg_cprof_acc[k], t1 - tg_c0);      \
        tg_c0 = t1;                                                              \
    }
#else
#define TG_CPROF_INIT
#define TG_CPROF(k)
#endif

// groups with more links than this are summed by wave reductions (lane = link)
constexpr int COMPOSE_SERIAL_MAX = 8;
template <class M> constexpr int max_small_group() {
    int m = 0;
    for (int g = 0; g < M::NG; ++g)
        if (M::group_nlinks[g] <= COMPOSE_SERIAL_MAX && M::group_nlinks[g] > m) m = M::group_nlinks[g];
    return m;
}
template <int NV> __device__ __forceinline__ void wave_sum_n(float *v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], m, 64);
}

// COMPOSE_WPB wavefronts per workgroup, one env each: a launch over all envs
// is N / COMPOSE_WPB workgroups (most waves exit at once), not N
constexpr int COMPOSE_WPB = 8;

// Prologue (tg_walk_step): the walk task's pre_physics_step fused into the
// compose launch that precedes every step kernel -- the same fp32 operations
// as walk_task.hip walk_pre_kernel (no contraction: default + scale * a).
__device__ __forceinline__ float pm_clamp(const StepArgs &a, float x) {
    return x < -a.pm_clip ? -a.pm_clip : (x > a.pm_clip ? a.pm_clip : x);
}
__device__ __forceinline__ float pm_target(const StepArgs &a, int d, float c) {
#pragma clang fp contract(off)
    return a.pm_default[d] + a.pm_scale * c;
}
__device__ __forceinline__ void target_prologue(const StepArgs &a, int e, int lane) {
    if (lane >= a.D) return;
    const unsigned i = (unsigned)e * (unsigned)a.D + (unsigned)lane;
    const float c = pm_clamp(a, a.pm_actions[i]);
    a.pm_act_out[i] = c;
    a.pm_tgt_out[i] = pm_target(a, lane, c);
}

// Prologue (tg_gogoro_step): gogoro_task.hip pre_kernel for env e on one lane
// -- the same fp32 operations (no contraction / reassociation here either)
// and the same Philox draw.
// the pre-physics values of env e: new action history ah[5], command, steering
// position target, rear-wheel velocity target (nothing stored)
__device__ __forceinline__ void gogoro_pre_values(const GogoroPre &g, int e, float *ah, float &cmd, float &tsteer,
                                                  float &vrear) {
#pragma clang fp contract(off) reassociate(off)
    const float x = g.actions[e];
    const float a = x < -g.clip_actions ? -g.clip_actions : (x > g.clip_actions ? g.clip_actions : x);
    const float *ah0 = g.action_history + 5 * (size_t)e;
    ah[0] = ah0[1]; ah[1] = ah0[2]; ah[2] = ah0[3]; ah[3] = ah0[4]; ah[4] = a;
    const float m = g.max_steering_change, ms = g.max_steering;
    float c;
    if (g.absolute_steer) {   // INCREMENTAL_STEER = False (gogoro_new.py:355-356)
        c = a * ms;
    } else {
        float da = a * m;
        da = da < -m ? -m : (da > m ? m : da);
        c = g.curent_command[e] + da;
    }
    c = c < -ms ? -ms : (c > ms ? ms : c);
    cmd = c;
    float r;
    if (g.pre_draws) {
        r = g.pre_draws[e];
    } else {
        const U4 u = philox(U4{(uint32_t)e, g.c_lo, g.c_hi, 0x50524531u}, g.k0, g.k1);
        r = gauss(u.x, u.y);
    }
    const float noise = g.noise_mean + r * g.noise_std;
    tsteer = c + g.steer_offsets[e] + noise;
    vrear = g.curent_speed[e];
}
__device__ __forceinline__ void gogoro_pre_store(const GogoroPre &g, int e, int D, const float *ah, float cmd,
                                                 float tsteer, float vrear) {
    float *h = g.action_history + 5 * (size_t)e;
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = ah[k];
    g.curent_command[e] = cmd;
    g.pos_target[(size_t)e * D + g.dof_steer] = tsteer;
    g.vel_target[(size_t)e * D + g.dof_rear] = vrear;
}
__device__ __forceinline__ void gogoro_pre_prologue(const GogoroPre &g, int e, int D) {
    float ah[5], cmd, ts, vr;
    gogoro_pre_values(g, e, ah, cmd, ts, vr);
    gogoro_pre_store(g, e, D, ah, cmd, ts, vr);
}

// the GogoroPaper pre_physics_step (paper_pre_kernel in gogoro_paper_task.hip,
// the same operations) for env e by its compose wavefront: the command history
// shifted in registers (lane = slot), the delayed command taken from its lane,
// the drive target rows written lane-strided
__device__ __forceinline__ void paper_pre_prologue(const PaperPre &pp, int e, int D, int lane) {
    constexpr int PC = TG_PAPER_CMD_HIST;
    static_assert(PC <= 64, "one history slot per lane");
    float *h = pp.command_history + PC * (size_t)e;
    const float act = pp.actions[e];
    const float ac = act < -1.0f ? -1.0f : (act > 1.0f ? 1.0f : act);
    const float cmd = ac * pp.max_steering;
    const float hn = lane < PC - 1 ? h[lane + 1] : 0.0f;
    const int64_t delay = pp.use_steer_delay ? pp.steer_delay[e] : 0;
    const float speed = pp.curent_speed[e];
    const float hv = lane < PC - 1 ? hn : cmd;
    int idx = PC - 3;
    if (pp.use_steer_delay) idx = delay == 0 ? 0 : (int)(PC - delay);   // command_history[:, -steer_delay]
    const float steer = __shfl(hv, idx, 64);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // every lane's history read before the stores
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < PC) h[lane] = hv;
    float *pt = pp.pos_target + (size_t)D * e, *vt = pp.vel_target + (size_t)D * e;
    for (int d = lane; d < D; d += 64) {
        pt[d] = d == pp.dof_steer ? steer : 0.0f;
        vt[d] = d == pp.dof_rear ? speed : 0.0f;
    }
    if (lane == 0) pp.curent_command[e] = cmd;
}

// Reward term 7's per-env partial sum_t (a[t+1] - a[t])^2, a = command / 0.5,
// over the clean history's command column as the post-physics will leave it
// (the 19 newest entries shifted down, the step's command appended; zero for
// an env that resets) -- the values paper_post_kernel would form, added in its
// 64-lane xor-butterfly order with no reassociation or contraction (this unit
// is compiled -ffast-math), so the post launch can finish the batch mean
// itself bit for bit (gogoro_realistic_turning_sim_paper.py:740).
__device__ __forceinline__ float paper_t7_partial(const PaperPre &pp, int e, float cmd) {
    constexpr int PH = TG_PAPER_HIST, PO = TG_PAPER_OBS;
    static_assert(PH - 1 <= 32, "partials on the butterfly's lower 32 lanes");
    const float *bo = pp.buffer_obs + (size_t)PH * PO * e;
    const bool rs = pp.reset_buf[e] != 0;
    float ch[PH];
#pragma unroll
    for (int t = 0; t < PH - 1; ++t) ch[t] = bo[(t + 1) * PO + 6];
    ch[PH - 1] = cmd;
    float v[32];
    {
#pragma clang fp reassociate(off) contract(off)
#pragma unroll
        for (int l = 0; l < 32; ++l) {
            if (l < PH - 1) {
                const float dd = ch[l + 1] / 0.5f - ch[l] / 0.5f;
                v[l] = dd * dd;
            } else {
                v[l] = 0.0f;
            }
        }
#pragma unroll
        for (int m = 16; m >= 1; m >>= 1)
#pragma unroll
            for (int l = 0; l < m; ++l) v[l] = v[l] + v[l + m];
    }
    return rs ? 0.0f : v[0];
}
// the block's sum of the partials (TG_PAPER_T7_BLK of them, env order, double);
// PUB (the one-launch step, PaperPost): stored with agent scope, the store
// waited for, then the block's arrival added to *cnt (paper_t7_wait_sum)
template <bool PUB = false>
__device__ __forceinline__ void paper_t7_block(const PaperPre &pp, const float *part, int blk,
                                               unsigned *cnt = nullptr) {
    double s = 0.0;
    {
#pragma clang fp reassociate(off) contract(off)
#pragma unroll
        for (int i = 0; i < TG_PAPER_T7_BLK; ++i) s = s + (double)part[i];
    }
    if constexpr (PUB) {
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(pp.t7 + blk),
                           (unsigned long long)__double_as_longlong(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        pp.t7[blk] = s;
    }
}

template <class M>
__device__ __forceinline__ void rb_force_env(const float *root, const float *dof, const float *comp, int e,
                                             const float *mass_scale, const float *forces, const float *torques,
                                             int space, float *out, int lane, float (*T)[12], float (*F)[10],
                                             const float *props, int N);

// a compile-time loop over groups G = B .. E-1: f(GroupC<G>{})
template <int N> struct GroupC {
    static constexpr int value = N;
};
template <int B, int E, class Fn> __device__ __forceinline__ void rbf_for_groups(Fn &&f) {
    if constexpr (B < E) {
        f(GroupC<B>{});
        rbf_for_groups<B + 1, E>(f);
    }
}

// one wavefront's compose scratch
template <class M> struct ComposeLds {
    float T[M::NL][12];        // link pose in its group-root frame: R (9), p (3)
    float LM[M::NL + 1][10];   // link mass, com (group frame), inertia about com; row NL = 0
    int GL[M::NG][M::MAXGL];   // group links, padded with NL (the zero row): branch-free sums
};

// compose env e with the 64 lanes of a wavefront (cs: the wave's LDS scratch)
template <class M> __device__ __forceinline__ void compose_env(const StepArgs &a, int e, int lane, ComposeLds<M> &cs) {
    TG_CPROF_INIT
    using CL = CompLayout<M>;
    static_assert(M::NL <= 64 && M::NG <= 64 && M::NS <= 64, "compose: one lane per link / group / shape");
    float(&T)[M::NL][12] = cs.T;
    float(&LM)[M::NL + 1][10] = cs.LM;
    int(&GL)[M::NG][M::MAXGL] = cs.GL;
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    wsync();   // a previous compose of this wave is done with the scratch
    auto ldT = [&](int l, M3 &R, V3 &P) {
#pragma unroll
        for (int k = 0; k < 9; ++k) R.a[k] = T[l][k];
        P = v3(T[l][9], T[l][10], T[l][11]);
    };
    auto ld9 = [](const float *o) { return M3{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}}; };
    // ---- every model constant and per-env input this lane needs, loaded up
    // front as one batch (the level loop below then runs on LDS only while
    // the group / shape loads are still in flight)
    for (int i = lane; i < M::NG * M::MAXGL; i += 64) {
        const int k = M::group_links[i / M::MAXGL][i % M::MAXGL];
        GL[i / M::MAXGL][i % M::MAXGL] = k < 0 ? M::NL : k;
    }
    if (lane < 10) LM[M::NL][lane] = 0.f;
    const int l = lane;                      // lane = link
    const bool lact = l < M::NL;
    M3 Rl = eye3();
    V3 tl = v3(0, 0, 0);
    int lev = -1, par = 0;
    float msc = 1.f, lin[10];
    if (lact) {
        lev = M::link_level[l];
        par = M::link_parent[l];
#pragma unroll
        for (int k = 0; k < 10; ++k) lin[k] = M::link_inertia[l][k];
        if (lev > 0) {
            const float *o = M::link_origin[l];
            Rl = ld9(o);
            tl = v3(o[9], o[10], o[11]);
            const int d = M::link_dof[l];
            if (d >= 0) {
                const float lo = prop(a, TG_PROP_LOWER, e, d), hi = prop(a, TG_PROP_UPPER, e, d);
                const float q = 0.5f * (lo + hi);
                // a locked joint is rigid at its window centre: a wider window
                // (props set as if the joint were free) is reported by tg_sync
                if (a.err && !(hi - lo <= TG_LOCK_WINDOW_MAX)) atomicOr(a.err, 1);
                const float *ax = M::link_axis[l];
                if (M::link_jtype[l] == TG_JOINT_REVOLUTE) Rl = mul(Rl, rot_axis(ax[0], ax[1], ax[2], q));
                else if (M::link_jtype[l] == TG_JOINT_PRISMATIC) tl = tl + q * mul(Rl, v3(ax[0], ax[1], ax[2]));
            }
        }
        if (a.mass_scale) msc = a.mass_scale[(size_t)e * M::NL + l];
    }
    const int g = lane;                      // lane = group
    const bool gact = g < M::NG;
    int gnl = 0, gpl = 0;
    M3 Qg = eye3(), Qp = eye3(), Rgo = eye3();
    V3 tgo = v3(0, 0, 0);
    if (gact) {
        gnl = M::group_nlinks[g];
        Qg = ld9(M::gq[g]);
        if (g > 0) {
            Qp = ld9(M::gq[M::parent[g]]);
            const int r = M::group_root[g];
            gpl = M::link_parent[r];
            Rgo = ld9(M::link_origin[r]);
            tgo = v3(M::link_origin[r][9], M::link_origin[r][10], M::link_origin[r][11]);
        }
    }
    const int sh = lane;                     // lane = shape
    const bool sact = sh < M::NS;
    int sl = 0;
    M3 Qs = eye3(), Rso = eye3();
    V3 tso = v3(0, 0, 0);
    if (sact) {
        sl = M::shape_link[sh];
        Qs = ld9(M::gq[M::shape_group[sh]]);
        Rso = ld9(M::shape_pose[sh]);
        tso = v3(M::shape_pose[sh][9], M::shape_pose[sh][10], M::shape_pose[sh][11]);
    }
    TG_CPROF(0)
    // ---- link poses in their group-root frame, level by level (LDS only)
    M3 R = eye3();
    V3 P = v3(0, 0, 0);
    for (int lv = 0; lv <= M::NLEV; ++lv) {
        if (lev == lv) {
            if (lv > 0) {
                M3 Rp;
                V3 Pp;
                ldT(par, Rp, Pp);
                R = mul(Rp, Rl);
                P = Pp + mul(Rp, tl);
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) T[l][k] = R.a[k];
            T[l][9] = P.x; T[l][10] = P.y; T[l][11] = P.z;
        }
        wsync();
    }
    if (lact) {   // per-link mass terms
        const float s = msc;
        const V3 cg = mul(R, v3(lin[1], lin[2], lin[3])) + P;
        const M3 Il{{lin[4] * s, lin[7] * s, lin[8] * s, lin[7] * s, lin[5] * s, lin[9] * s, lin[8] * s, lin[9] * s,
                     lin[6] * s}};
        const M3 RI = mul(mul(R, Il), transpose(R));
        LM[l][0] = lin[0] * s;
        LM[l][1] = cg.x; LM[l][2] = cg.y; LM[l][3] = cg.z;
        LM[l][4] = RI.a[0]; LM[l][5] = RI.a[4]; LM[l][6] = RI.a[8];
        LM[l][7] = RI.a[1]; LM[l][8] = RI.a[2]; LM[l][9] = RI.a[5];
        if constexpr (M::LCOM) {   // the link's com in its group's joint-aligned frame
            const float *qg = M::gq[M::link_group[l]];
            const V3 cq = mulT(M3{{qg[0], qg[1], qg[2], qg[3], qg[4], qg[5], qg[6], qg[7], qg[8]}}, cg);
            float *lc = a.comp + (size_t)e * M::KC + CL::lcom(l);
            lc[0] = cq.x; lc[1] = cq.y; lc[2] = cq.z;
        }
    }
    wsync();
    TG_CPROF(1)
    // ---- group sums in link order (deterministic, the order of
    // oracle/physics_ref.c), written to the cache in joint-aligned group
    // frames (axis e_z, codegen gq): v' = Q^T v, I' = Q^T I Q, placements
    // R' = Q_p^T R Q_g, t' = Q_p^T t
    float *c = a.comp + (size_t)e * M::KC;
    // large groups (the scooter's root group holds the locked rider: 55 links)
    // by wave reductions over lane = link, in tree order; the others by their
    // own lane in link order
    float bm = 0.f, bI[6] = {0, 0, 0, 0, 0, 0};
    V3 bc = v3(0, 0, 0);
#pragma unroll
    for (int gb = 0; gb < M::NG; ++gb) {
        if constexpr (M::MAXGL > COMPOSE_SERIAL_MAX) {
            if (M::group_nlinks[gb] <= COMPOSE_SERIAL_MAX) continue;
            const bool mine = lact && M::link_group[l] == gb;
            float v4[4] = {0.f, 0.f, 0.f, 0.f};
            if (mine) { v4[0] = LM[l][0]; v4[1] = LM[l][0] * LM[l][1]; v4[2] = LM[l][0] * LM[l][2]; v4[3] = LM[l][0] * LM[l][3]; }
            wave_sum_n<4>(v4);
            const float im = v4[0] > 0.f ? 1.0f / v4[0] : 0.f;
            const V3 gcb = v3(v4[1] * im, v4[2] * im, v4[3] * im);
            float v6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (mine) {
                const float ml = LM[l][0];
                const V3 dd = v3(LM[l][1], LM[l][2], LM[l][3]) - gcb;
                const float d2 = dot(dd, dd);
                v6[0] = LM[l][4] + ml * (d2 - dd.x * dd.x);
                v6[1] = LM[l][5] + ml * (d2 - dd.y * dd.y);
                v6[2] = LM[l][6] + ml * (d2 - dd.z * dd.z);
                v6[3] = LM[l][7] - ml * dd.x * dd.y;
                v6[4] = LM[l][8] - ml * dd.x * dd.z;
                v6[5] = LM[l][9] - ml * dd.y * dd.z;
            }
            wave_sum_n<6>(v6);
            if (lane == gb) {
                bm = v4[0];
                bc = gcb;
#pragma unroll
                for (int k = 0; k < 6; ++k) bI[k] = v6[k];
            }
        }
    }
    if (gact) {
        float gm = 0.f;
        V3 gc = v3(0, 0, 0);
        float gI[6] = {0, 0, 0, 0, 0, 0};
        constexpr int SM = max_small_group<M>();
        if (gnl > COMPOSE_SERIAL_MAX) {
            gm = bm;
            gc = bc;
#pragma unroll
            for (int k = 0; k < 6; ++k) gI[k] = bI[k];
        } else {
#pragma unroll
            for (int i = 0; i < SM; ++i) {   // unrolled and branch-free (padding = the zero row)
                const int k = GL[g][i];
                gm += LM[k][0];
                gc = gc + LM[k][0] * v3(LM[k][1], LM[k][2], LM[k][3]);
            }
            gc = (gm > 0.f ? 1.0f / gm : 0.f) * gc;
#pragma unroll
            for (int i = 0; i < SM; ++i) {
                const int k = GL[g][i];
                const float ml = LM[k][0];
                const V3 dd = v3(LM[k][1], LM[k][2], LM[k][3]) - gc;
                const float d2 = dot(dd, dd);
                gI[0] += LM[k][4] + ml * (d2 - dd.x * dd.x);
                gI[1] += LM[k][5] + ml * (d2 - dd.y * dd.y);
                gI[2] += LM[k][6] + ml * (d2 - dd.z * dd.z);
                gI[3] += LM[k][7] - ml * dd.x * dd.y;
                gI[4] += LM[k][8] - ml * dd.x * dd.z;
                gI[5] += LM[k][9] - ml * dd.y * dd.z;
            }
        }
        const V3 gcq = mulT(Qg, gc);
        float gIq[6];
        sym_from(gIq, mul(mul(transpose(Qg), sym_to(gI)), Qg));
        float *ci = c + CL::inertia(g);
        ci[0] = gm;
        ci[1] = gcq.x; ci[2] = gcq.y; ci[3] = gcq.z;
#pragma unroll
        for (int k = 0; k < 6; ++k) ci[4 + k] = gIq[k];
        ci[10] = 0.f;
        ci[11] = 0.f;
        if (g > 0) {
            M3 Rp;
            V3 Pp;
            ldT(gpl, Rp, Pp);
            const M3 Rx = mul(mul(transpose(Qp), mul(Rp, Rgo)), Qg);
            const V3 t = mulT(Qp, Pp + mul(Rp, tgo));
            float *cx = c + CL::xtree(g);
#pragma unroll
            for (int k = 0; k < 9; ++k) cx[k] = Rx.a[k];
            cx[9] = t.x; cx[10] = t.y; cx[11] = t.z;
            if constexpr (M::NTL > 0) {   // composed placement of a group below a translating lock
#pragma unroll
                for (int j = 0; j < M::NAG; ++j)
                    if (M::ag_group[j] == g) {
                        c[CL::xag(j)] = t.x; c[CL::xag(j) + 1] = t.y; c[CL::xag(j) + 2] = t.z;
                    }
            }
        }
    }
    if constexpr (M::NTL > 0) {
        // translating-lock extension: the lock group's mass moments (pre-Q
        // group frame) and, per lock, the moments of the links below it
        constexpr int NV = 10 + 4 * M::NTL;
        float v[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = 0.f;
        if (lact && M::link_group[l] == M::tl_group) {
            const float ml = LM[l][0];
            const V3 pc = v3(LM[l][1], LM[l][2], LM[l][3]);
            const float d2 = dot(pc, pc);
            v[0] = ml;
            v[1] = ml * pc.x; v[2] = ml * pc.y; v[3] = ml * pc.z;
            v[4] = LM[l][4] + ml * (d2 - pc.x * pc.x);
            v[5] = LM[l][5] + ml * (d2 - pc.y * pc.y);
            v[6] = LM[l][6] + ml * (d2 - pc.z * pc.z);
            v[7] = LM[l][7] - ml * pc.x * pc.y;
            v[8] = LM[l][8] - ml * pc.x * pc.z;
            v[9] = LM[l][9] - ml * pc.y * pc.z;
#pragma unroll
            for (int k = 0; k < M::NTL; ++k)
                if ((M::link_tl[l] >> k) & 1) {
                    v[10 + 4 * k] = ml;
                    v[11 + 4 * k] = ml * pc.x; v[12 + 4 * k] = ml * pc.y; v[13 + 4 * k] = ml * pc.z;
                }
        }
        wave_sum_n<NV>(v);
        if (lane == 0) {
            float *x = c + CL::ext();
#pragma unroll
            for (int k = 0; k < 10; ++k) x[k] = v[k];
#pragma unroll
            for (int k = 0; k < M::NTL; ++k) {
                const int lk = M::tl_link[k], dk = M::tl_dof[k];
                M3 Rp;
                V3 Pp;
                ldT(M::link_parent[lk], Rp, Pp);
                const float *o = M::link_origin[lk];
                const float *ax = M::link_axis[lk];
                const V3 w = mul(Rp, mul(ld9(o), v3(ax[0], ax[1], ax[2])));
                float *xk = c + CL::xk(k);
                xk[0] = 0.5f * (prop(a, TG_PROP_LOWER, e, dk) + prop(a, TG_PROP_UPPER, e, dk));   // as the FK above
                xk[1] = v[10 + 4 * k];
                xk[2] = v[11 + 4 * k]; xk[3] = v[12 + 4 * k]; xk[4] = v[13 + 4 * k];
                xk[5] = w.x; xk[6] = w.y; xk[7] = w.z;
            }
        }
    }
    TG_CPROF(2)
    if (sact) {   // shape poses in their group frame
        M3 Rsl;
        V3 Psl;
        ldT(sl, Rsl, Psl);
        const M3 Rx = mul(transpose(Qs), mul(Rsl, Rso));
        const V3 t = mulT(Qs, Psl + mul(Rsl, tso));
        float *cs = c + CL::shape(sh);
#pragma unroll
        for (int k = 0; k < 9; ++k) cs[k] = Rx.a[k];
        cs[9] = t.x; cs[10] = t.y; cs[11] = t.z;
        if constexpr (M::NTL > 0) {   // composed pose of a lock-group shape below a translating lock
#pragma unroll
            for (int j = 0; j < M::NASH; ++j)
                if (M::ash_shape[j] == sh) {
                    c[CL::xash(j)] = t.x; c[CL::xash(j) + 1] = t.y; c[CL::xash(j) + 2] = t.z;
                }
        }
    }
    if (lane == 0) a.dirty[e] = 0;
    TG_CPROF(3)
}

// After a full compose: is every env's composite block the same as env 0's?
// One wavefront per env; a mismatch clears the flag (set to 1 before the
// launch).  NaN compares unequal: never uniform.  (The DOF property rows are
// not shared: the step kernel reads each env's own, so writes through the
// dof_props view need no re-check.)
template <class M> __global__ __launch_bounds__(64) void uniform_check_kernel(StepArgs a) {
    const int e = blockIdx.x, lane = threadIdx.x;
    if (e == 0 || e >= a.N) return;
    bool bad = false;
    const float *c = a.comp + (size_t)e * M::KC;
    for (int k = lane; k < M::KC; k += 64) bad |= c[k] != a.comp[k];
    if (__any(bad) && lane == 0) atomicExch(a.cuni, 0);
}

template <class M> __global__ __launch_bounds__(64 * COMPOSE_WPB) void compose_kernel(StepArgs a) {
    const int wv = threadIdx.x / 64;
    const int e = blockIdx.x * COMPOSE_WPB + wv;
    const bool dirty = e < a.N && a.dirty[e] != 0;   // read before the prologue: one memory latency
    if (a.cnext && blockIdx.x == 0 && threadIdx.x == 0) *a.cnext = 0;   // the reset list the next epilogue fills
    if (a.pm_actions && !a.pm_in_step && e < a.N) target_prologue(a, e, threadIdx.x % 64);
    if (a.gp.actions && !a.gp_in_step && e < a.N && threadIdx.x % 64 == 0) gogoro_pre_prologue(a.gp, e, a.D);
    if (a.pp.actions && !a.pp_in_step && e < a.N) paper_pre_prologue(a.pp, e, a.D, threadIdx.x % 64);
    __shared__ ComposeLds<M> cs[COMPOSE_WPB];
    if (dirty) compose_env<M>(a, e, threadIdx.x % 64, cs[wv]);
    if (a.rbf_forces && e < a.N)   // a pending apply_rigid_body_force_tensors, on the fresh composite
        rb_force_env<M>(a.root, a.dof, a.comp, e, a.mass_scale, a.rbf_forces, a.rbf_torques, a.rbf_space, a.rbf_out,
                        threadIdx.x % 64, cs[wv].T, cs[wv].LM, a.props, a.N);
}

// Compose of the envs a fused task epilogue reset (tg_gogoro_step): the
// previous step kernel appended their ids to a.clist / *a.ccount, so no wave
// reads all N dirty flags.  One wavefront per workgroup, COMPOSE_WPB envs per
// wave: first the task's pre-physics prologue on lanes 0..COMPOSE_WPB-1 (one
// lane per env), then wave b composes list entry b (b + grid, ... for longer
// lists); zeroes the count the coming epilogue appends to.
template <class M> __global__ __launch_bounds__(64) void compose_list_kernel(StepArgs a) {
    const int lane = threadIdx.x;
    const int n = a.ccount ? *a.ccount : 0;   // issued first: its latency overlaps the prologue
    if (a.cnext && blockIdx.x == 0 && lane == 0) *a.cnext = 0;
    const int e0 = blockIdx.x * COMPOSE_WPB + lane;
    if (a.gp.actions && !a.gp_in_step && lane < COMPOSE_WPB && e0 < a.N) gogoro_pre_prologue(a.gp, e0, a.D);
    if ((int)blockIdx.x >= n) return;
    __shared__ ComposeLds<M> cs;
    for (int i = blockIdx.x; i < n; i += gridDim.x) compose_env<M>(a, a.clist[i], lane, cs);
}

// ---------------------------------------------------------------- rigid-body states
// World state of every link (acquire/refresh_rigid_body_state_tensor): one
// wavefront per env, links level by level (lane = link): R_l = R_p Ro Rj(q),
// p_l = p_p + R_p (to + q s), w_l = w_p + qd R_p Ro a (revolute),
// v_l = v_p + w_p x (p_l - p_p) + qd R_p Ro a (prismatic), v_l at the link
// origin; out[e][l] = (p_l, quat(R_l) xyzw, v_l + w_l x R_l c_l, w_l).
// The same function as oracle/physics_ref.c oracle_rigid_body_states.
__device__ __forceinline__ void m3_to_quat(const M3 &R, float &x, float &y, float &z, float &w) {
    const float m00 = R.a[0], m11 = R.a[4], m22 = R.a[8], tr = m00 + m11 + m22;
    if (tr > 0.f) {
        const float s = 0.5f / sqrtf(tr + 1.f);
        w = 0.25f / s; x = (R.a[7] - R.a[5]) * s; y = (R.a[2] - R.a[6]) * s; z = (R.a[3] - R.a[1]) * s;
    } else if (m00 > m11 && m00 > m22) {
        const float s = 2.f * sqrtf(1.f + m00 - m11 - m22);
        w = (R.a[7] - R.a[5]) / s; x = 0.25f * s; y = (R.a[1] + R.a[3]) / s; z = (R.a[2] + R.a[6]) / s;
    } else if (m11 > m22) {
        const float s = 2.f * sqrtf(1.f + m11 - m00 - m22);
        w = (R.a[2] - R.a[6]) / s; x = (R.a[1] + R.a[3]) / s; y = 0.25f * s; z = (R.a[5] + R.a[7]) / s;
    } else {
        const float s = 2.f * sqrtf(1.f + m22 - m00 - m11);
        w = (R.a[3] - R.a[1]) / s; x = (R.a[2] + R.a[6]) / s; y = (R.a[5] + R.a[7]) / s; z = 0.25f * s;
    }
}

template <class M> __global__ __launch_bounds__(64) void body_state_kernel(const float *root, const float *dof, int n,
                                                                           float *out) {
    const int e = blockIdx.x;
    if (e >= n) return;
    __shared__ float T[M::NL][18];   // R (9), p (3), w (3), v at the origin (3)
    const int lane = threadIdx.x;
    const float *r = root + 13 * (size_t)e;
    const float *q = dof + 2 * (size_t)e * M::ND;
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (int lev = 0; lev <= M::NDEPTH; ++lev) {
        for (int l = lane; l < M::NL; l += 64) {
            if (M::link_depth[l] != lev) continue;
            M3 R;
            V3 P, W, V;
            if (M::link_parent[l] < 0) {
                float qx = r[3], qy = r[4], qz = r[5], qw = r[6];
                const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
                R = quat_to_m3(qx * in, qy * in, qz * in, qw * in);
                P = v3(r[0], r[1], r[2]);
                W = v3(r[10], r[11], r[12]);
                const V3 c = v3(M::link_inertia[l][1], M::link_inertia[l][2], M::link_inertia[l][3]);
                V = v3(r[7], r[8], r[9]) - cross(W, mul(R, c));   // root state: velocity of the root link's com
            } else {
                const int pl = M::link_parent[l];
                M3 Rp;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rp.a[k] = T[pl][k];
                const V3 Pp = v3(T[pl][9], T[pl][10], T[pl][11]);
                const V3 Wp = v3(T[pl][12], T[pl][13], T[pl][14]), Vp = v3(T[pl][15], T[pl][16], T[pl][17]);
                const float *o = M::link_origin[l];
                M3 Ro{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}};
                V3 to = v3(o[9], o[10], o[11]);
                const int d = M::link_dof[l];
                const float qq = d >= 0 ? q[2 * d] : 0.f, qd = d >= 0 ? q[2 * d + 1] : 0.f;
                const float *ax = M::link_axis[l];
                const V3 axw = mul(Rp, mul(Ro, v3(ax[0], ax[1], ax[2])));   // joint axis, world
                W = Wp;
                if (M::link_jtype[l] == TG_JOINT_REVOLUTE) {
                    Ro = mul(Ro, rot_axis(ax[0], ax[1], ax[2], qq));
                    W = W + qd * axw;
                } else if (M::link_jtype[l] == TG_JOINT_PRISMATIC) {
                    to = to + qq * mul(Ro, v3(ax[0], ax[1], ax[2]));
                }
                R = mul(Rp, Ro);
                P = Pp + mul(Rp, to);
                V = Vp + cross(Wp, P - Pp);
                if (M::link_jtype[l] == TG_JOINT_PRISMATIC) V = V + qd * axw;
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) T[l][k] = R.a[k];
            T[l][9] = P.x; T[l][10] = P.y; T[l][11] = P.z;
            T[l][12] = W.x; T[l][13] = W.y; T[l][14] = W.z;
            T[l][15] = V.x; T[l][16] = V.y; T[l][17] = V.z;
        }
        wsync();
    }
    for (int l = lane; l < M::NL; l += 64) {
        M3 R;
#pragma unroll
        for (int k = 0; k < 9; ++k) R.a[k] = T[l][k];
        const V3 W = v3(T[l][12], T[l][13], T[l][14]);
        const V3 c = v3(M::link_inertia[l][1], M::link_inertia[l][2], M::link_inertia[l][3]);
        const V3 vc = v3(T[l][15], T[l][16], T[l][17]) + cross(W, mul(R, c));
        float qx, qy, qz, qw;
        m3_to_quat(R, qx, qy, qz, qw);
        float *o = out + ((size_t)e * M::NL + l) * 13;
        o[0] = T[l][9]; o[1] = T[l][10]; o[2] = T[l][11];
        o[3] = qx; o[4] = qy; o[5] = qz; o[6] = qw;
        o[7] = vc.x; o[8] = vc.y; o[9] = vc.z;
        o[10] = W.x; o[11] = W.y; o[12] = W.z;
    }
}

// ---------------------------------------------------------------- rigid-body forces
// apply_rigid_body_force_tensors (reference call site
// tasks/gogoro_realistic_turning_sim_paper.py:457): per-link forces [N*L,3] at
// the link coms and optional torques [N*L,3], world (space 0) or link frame
// (space 1), reduced to the step kernel's group wrenches [N,G,6] (world force,
// torque about the group com): F_g = sum f_l, T_g = sum t_l + (p_l - c_g) x f_l,
// c_g the mass-weighted (per-env mass scale) com of the group's links.  One
// wavefront per env: link poses level by level (lane = link), then lane = group
// sums its links in link order.  The same function as oracle/physics_ref.c
// oracle_rigid_body_force_wrench.
// env e with the 64 lanes of a wavefront; T, F: the wave's LDS scratch
template <class M> constexpr int group_depth(int g) {
    int d = 0;
    while (M::parent[g] >= 0) {
        g = M::parent[g];
        ++d;
    }
    return d;
}
template <class M> constexpr int max_group_depth() {
    int d = 0;
    for (int g = 0; g < M::NG; ++g) d = group_depth<M>(g) > d ? group_depth<M>(g) : d;
    return d;
}

template <class M>
__device__ __forceinline__ void rb_force_env(const float *root, const float *dof, const float *comp, int e,
                                             const float *mass_scale, const float *forces, const float *torques,
                                             int space, float *out, int lane, float (*T)[12], float (*F)[10],
                                             const float *props, int N) {
    const float *r = root + 13 * (size_t)e;
    const float *q = dof + 2 * (size_t)e * M::ND;
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    wsync();   // the scratch may have been in use by this wave
    if constexpr (M::LCOM && M::NL <= 64 && M::NG <= 64) {
        if (comp && space == 0) {
            // world forces, one link and one group per lane: every input of the
            // env is issued in one batch -- the lane's link force / torque, its
            // com and its group's com (composite cache), the lane's group
            // placement and joint position, the root orientation, the lock
            // windows -- so the wave waits on memory once; then the arms
            // arm_l = W_g (c_l - c_g) from the group orientations W_g (group
            // kinematics through LDS, a few levels) and the group sums
            using CL = CompLayout<M>;
            const float *c = comp + (size_t)e * M::KC;
            const bool hl = lane < M::NL;
            const int l = hl ? lane : 0;
            const int gl = M::link_group[l];
            const size_t i = (size_t)e * M::NL + l;
            V3 f = v3(0, 0, 0), t = v3(0, 0, 0), lc = v3(0, 0, 0), gc = v3(0, 0, 0);
            if (hl) {
                f = v3(forces[3 * i], forces[3 * i + 1], forces[3 * i + 2]);
                if (torques) t = v3(torques[3 * i], torques[3 * i + 1], torques[3 * i + 2]);
                lc = v3(c[CL::lcom(l)], c[CL::lcom(l) + 1], c[CL::lcom(l) + 2]);
                gc = v3(c[CL::inertia(gl) + 1], c[CL::inertia(gl) + 2], c[CL::inertia(gl) + 3]);
            }
            const bool hg = lane > 0 && lane < M::NG;
            const int g = hg ? lane : 1 % M::NG;
            M3 Rpc;
            float qj = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) Rpc.a[k] = hg ? c[CL::xtree(g) + k] : 0.f;
            if (hg && M::jtype[g] == TG_JOINT_REVOLUTE) qj = q[2 * M::gdof[g]];
            const float qx = r[3], qy = r[4], qz = r[5], qw = r[6];
            V3 ush[M::NTL > 0 ? M::NTL : 1];
            if constexpr (M::NTL > 0) {   // lock displacements since the compose (tl_update, above)
                const size_t ND = (size_t)N * M::ND;
#pragma unroll
                for (int k = 0; k < M::NTL; ++k) {
                    const size_t id = (size_t)e * M::ND + M::tl_dof[k];
                    const float qc = 0.5f * (props[TG_PROP_LOWER * ND + id] + props[TG_PROP_UPPER * ND + id]);
                    const float *xk = c + CL::xk(k);
                    ush[k] = (qc - xk[0]) * v3(xk[5], xk[6], xk[7]);
                }
            }
            const bool act = f.x != 0.f || f.y != 0.f || f.z != 0.f || t.x != 0.f || t.y != 0.f || t.z != 0.f;
            if (!__any(act)) {   // no force and no torque on any link: zero wrenches
                for (int k = lane; k < 6 * M::NG; k += 64) out[(size_t)e * 6 * M::NG + k] = 0.f;
                return;
            }
            if (hg && M::jtype[g] == TG_JOINT_REVOLUTE) {   // Rpc Rz(q), as step pass 1a
                float sq, cq;
                tg_sincos(qj, &sq, &cq);
#pragma unroll
                for (int rr = 0; rr < 3; ++rr) {
                    const float c0 = Rpc.a[3 * rr], c1 = Rpc.a[3 * rr + 1];
                    Rpc.a[3 * rr] = c0 * cq + c1 * sq;
                    Rpc.a[3 * rr + 1] = c1 * cq - c0 * sq;
                }
            }
            constexpr int GD = max_group_depth<M>();
            for (int lev = 0; lev <= GD; ++lev) {
                if (lev == 0 && lane == 0) {
                    const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
                    const M3 W = mul(quat_to_m3(qx * in, qy * in, qz * in, qw * in),
                                     M3{{M::gq[0][0], M::gq[0][1], M::gq[0][2], M::gq[0][3], M::gq[0][4],
                                         M::gq[0][5], M::gq[0][6], M::gq[0][7], M::gq[0][8]}});
#pragma unroll
                    for (int k = 0; k < 9; ++k) T[0][k] = W.a[k];
                } else if (lev > 0 && hg && group_depth<M>(g) == lev) {
                    M3 Wp;
#pragma unroll
                    for (int k = 0; k < 9; ++k) Wp.a[k] = T[M::parent[g]][k];
                    const M3 W = mul(Wp, Rpc);
#pragma unroll
                    for (int k = 0; k < 9; ++k) T[g][k] = W.a[k];
                }
                wsync();
            }
            if (hl) {
                M3 W;
#pragma unroll
                for (int k = 0; k < 9; ++k) W.a[k] = T[gl][k];
                if constexpr (M::NTL > 0) {
                    if (gl == M::tl_group && M::link_tl[l]) {
                        V3 sh = v3(0, 0, 0);
#pragma unroll
                        for (int k = 0; k < M::NTL; ++k)
                            if ((M::link_tl[l] >> k) & 1) sh = sh + ush[k];
                        const float *qg = M::gq[gl];
                        lc = lc + mulT(M3{{qg[0], qg[1], qg[2], qg[3], qg[4], qg[5], qg[6], qg[7], qg[8]}}, sh);
                    }
                }
                const V3 tq = t + cross(mul(W, lc - gc), f);
                F[l][0] = f.x; F[l][1] = f.y; F[l][2] = f.z;
                F[l][3] = tq.x; F[l][4] = tq.y; F[l][5] = tq.z;
            }
            wsync();
            // group sums in link order, one lane per (group, component): the
            // group loop is unrolled at compile time so every link index is an
            // immediate LDS offset (a lane-indexed walk of the group-link table
            // would wait on a table load per link)
            for (int j = lane; j < 6 * M::NG; j += 64) {
                float acc = 0.f;
                const int gsel = j / 6, cmp = j % 6;
                rbf_for_groups<0, M::NG>([&](auto G) {
                    constexpr int gg = decltype(G)::value;
                    if (gsel == gg) {
#pragma unroll
                        for (int k = 0; k < M::group_nlinks[gg]; ++k) acc += F[M::group_links[gg][k]][cmp];
                    }
                });
                out[(size_t)e * 6 * M::NG + j] = acc;
            }
            return;
        }
    }
    // an env with no force and no torque on any link gets zero wrenches without
    // the link kinematics (the paper task pushes only its first 2048 envs)
    bool any = false;
    for (int l = lane; l < M::NL; l += 64) {
        const size_t i = 3 * ((size_t)e * M::NL + l);
        any = any || forces[i] != 0.f || forces[i + 1] != 0.f || forces[i + 2] != 0.f;
        if (torques) any = any || torques[i] != 0.f || torques[i + 1] != 0.f || torques[i + 2] != 0.f;
    }
    if (!__any(any)) {
        for (int k = lane; k < 6 * M::NG; k += 64) out[(size_t)e * 6 * M::NG + k] = 0.f;
        return;
    }
    if constexpr (M::LCOM) {
        if (comp && space == 0) {
            // world forces: the moment arms from the composite cache -- each
            // link's com and its group's com in the group's joint-aligned frame
            // -- rotated by the group's world orientation (group kinematics, a
            // few levels), no link kinematics: arm_l = W_g (c_l - c_g)
            using CL = CompLayout<M>;
            const float *c = comp + (size_t)e * M::KC;
            float qx = r[3], qy = r[4], qz = r[5], qw = r[6];
            const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
            const M3 Rr = quat_to_m3(qx * in, qy * in, qz * in, qw * in);
            constexpr int GD = max_group_depth<M>();
            for (int lev = 0; lev <= GD; ++lev) {
                for (int g = lane; g < M::NG; g += 64) {
                    if (group_depth<M>(g) != lev) continue;
                    M3 W;
                    if (g == 0) {
                        W = mul(Rr, M3{{M::gq[0][0], M::gq[0][1], M::gq[0][2], M::gq[0][3], M::gq[0][4], M::gq[0][5],
                                        M::gq[0][6], M::gq[0][7], M::gq[0][8]}});
                    } else {
                        M3 Wp, Rpc;
#pragma unroll
                        for (int k = 0; k < 9; ++k) {
                            Wp.a[k] = T[M::parent[g]][k];
                            Rpc.a[k] = c[CL::xtree(g) + k];
                        }
                        if (M::jtype[g] == TG_JOINT_REVOLUTE) {   // Rpc Rz(q), as step pass 1a
                            float sq, cq;
                            tg_sincos(q[2 * M::gdof[g]], &sq, &cq);
#pragma unroll
                            for (int rr = 0; rr < 3; ++rr) {
                                const float c0 = Rpc.a[3 * rr], c1 = Rpc.a[3 * rr + 1];
                                Rpc.a[3 * rr] = c0 * cq + c1 * sq;
                                Rpc.a[3 * rr + 1] = c1 * cq - c0 * sq;
                            }
                        }
                        W = mul(Wp, Rpc);
                    }
#pragma unroll
                    for (int k = 0; k < 9; ++k) T[g][k] = W.a[k];
                }
                wsync();
            }
            // models whose resets move translating locks in place (tl_update):
            // the link coms below a lock are the composed ones shifted by the
            // lock's displacement since that compose, from the current window
            V3 ush[M::NTL > 0 ? M::NTL : 1];
            if constexpr (M::NTL > 0) {
                const size_t ND = (size_t)N * M::ND;
#pragma unroll
                for (int k = 0; k < M::NTL; ++k) {
                    const size_t i = (size_t)e * M::ND + M::tl_dof[k];
                    const float qc = 0.5f * (props[TG_PROP_LOWER * ND + i] + props[TG_PROP_UPPER * ND + i]);
                    const float *xk = c + CL::xk(k);
                    ush[k] = (qc - xk[0]) * v3(xk[5], xk[6], xk[7]);
                }
            }
            for (int l = lane; l < M::NL; l += 64) {
                const int g = M::link_group[l];
                M3 W;
#pragma unroll
                for (int k = 0; k < 9; ++k) W.a[k] = T[g][k];
                V3 lc = v3(c[CL::lcom(l)], c[CL::lcom(l) + 1], c[CL::lcom(l) + 2]);
                if constexpr (M::NTL > 0) {
                    if (g == M::tl_group && M::link_tl[l]) {
                        V3 sh = v3(0, 0, 0);
#pragma unroll
                        for (int k = 0; k < M::NTL; ++k)
                            if ((M::link_tl[l] >> k) & 1) sh = sh + ush[k];
                        const float *qg = M::gq[g];
                        lc = lc + mulT(M3{{qg[0], qg[1], qg[2], qg[3], qg[4], qg[5], qg[6], qg[7], qg[8]}}, sh);
                    }
                }
                const V3 d = lc - v3(c[CL::inertia(g) + 1], c[CL::inertia(g) + 2], c[CL::inertia(g) + 3]);
                const V3 arm = mul(W, d);
                const size_t i = (size_t)e * M::NL + l;
                const V3 f = v3(forces[3 * i], forces[3 * i + 1], forces[3 * i + 2]);
                const V3 t = torques ? v3(torques[3 * i], torques[3 * i + 1], torques[3 * i + 2]) : v3(0, 0, 0);
                const V3 tq = t + cross(arm, f);
                F[l][0] = f.x; F[l][1] = f.y; F[l][2] = f.z;
                F[l][3] = tq.x; F[l][4] = tq.y; F[l][5] = tq.z;
            }
            wsync();
            for (int g = lane; g < M::NG; g += 64) {
                V3 fs = v3(0, 0, 0), ts = v3(0, 0, 0);
                for (int k = 0; k < M::group_nlinks[g]; ++k) {
                    const int l = M::group_links[g][k];
                    fs = fs + v3(F[l][0], F[l][1], F[l][2]);
                    ts = ts + v3(F[l][3], F[l][4], F[l][5]);
                }
                float *o = out + ((size_t)e * M::NG + g) * 6;
                o[0] = fs.x; o[1] = fs.y; o[2] = fs.z;
                o[3] = ts.x; o[4] = ts.y; o[5] = ts.z;
            }
            return;
        }
    }
    for (int lev = 0; lev <= M::NDEPTH; ++lev) {
        for (int l = lane; l < M::NL; l += 64) {
            if (M::link_depth[l] != lev) continue;
            M3 R;
            V3 P;
            if (M::link_parent[l] < 0) {
                float qx = r[3], qy = r[4], qz = r[5], qw = r[6];
                const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
                R = quat_to_m3(qx * in, qy * in, qz * in, qw * in);
                P = v3(r[0], r[1], r[2]);
            } else {
                const int pl = M::link_parent[l];
                M3 Rp;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rp.a[k] = T[pl][k];
                const V3 Pp = v3(T[pl][9], T[pl][10], T[pl][11]);
                const float *o = M::link_origin[l];
                M3 Ro{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}};
                V3 to = v3(o[9], o[10], o[11]);
                const int d = M::link_dof[l];
                const float qq = d >= 0 ? q[2 * d] : 0.f;
                const float *ax = M::link_axis[l];
                if (M::link_jtype[l] == TG_JOINT_REVOLUTE) Ro = mul(Ro, rot_axis(ax[0], ax[1], ax[2], qq));
                else if (M::link_jtype[l] == TG_JOINT_PRISMATIC) to = to + qq * mul(Ro, v3(ax[0], ax[1], ax[2]));
                R = mul(Rp, Ro);
                P = Pp + mul(Rp, to);
            }
#pragma unroll
            for (int k = 0; k < 9; ++k) T[l][k] = R.a[k];
            T[l][9] = P.x; T[l][10] = P.y; T[l][11] = P.z;
        }
        wsync();
    }
    for (int l = lane; l < M::NL; l += 64) {
        M3 R;
#pragma unroll
        for (int k = 0; k < 9; ++k) R.a[k] = T[l][k];
        const V3 pc = v3(T[l][9], T[l][10], T[l][11]) +
                      mul(R, v3(M::link_inertia[l][1], M::link_inertia[l][2], M::link_inertia[l][3]));
        const size_t i = (size_t)e * M::NL + l;
        V3 f = v3(forces[3 * i], forces[3 * i + 1], forces[3 * i + 2]);
        V3 t = torques ? v3(torques[3 * i], torques[3 * i + 1], torques[3 * i + 2]) : v3(0, 0, 0);
        if (space == 1) {
            f = mul(R, f);
            t = mul(R, t);
        }
        F[l][0] = pc.x; F[l][1] = pc.y; F[l][2] = pc.z;
        F[l][3] = M::link_inertia[l][0] * (mass_scale ? mass_scale[i] : 1.f);
        F[l][4] = f.x; F[l][5] = f.y; F[l][6] = f.z;
        F[l][7] = t.x; F[l][8] = t.y; F[l][9] = t.z;
    }
    wsync();
    for (int g = lane; g < M::NG; g += 64) {
        float gm = 0.f;
        V3 gc = v3(0, 0, 0);
        for (int k = 0; k < M::group_nlinks[g]; ++k) {
            const int l = M::group_links[g][k];
            gm += F[l][3];
            gc = gc + F[l][3] * v3(F[l][0], F[l][1], F[l][2]);
        }
        const int rl = M::group_links[g][0];
        gc = gm > 0.f ? (1.0f / gm) * gc : v3(T[rl][9], T[rl][10], T[rl][11]);
        V3 fs = v3(0, 0, 0), ts = v3(0, 0, 0);
        for (int k = 0; k < M::group_nlinks[g]; ++k) {
            const int l = M::group_links[g][k];
            const V3 f = v3(F[l][4], F[l][5], F[l][6]);
            fs = fs + f;
            ts = ts + v3(F[l][7], F[l][8], F[l][9]) + cross(v3(F[l][0], F[l][1], F[l][2]) - gc, f);
        }
        float *o = out + ((size_t)e * M::NG + g) * 6;
        o[0] = fs.x; o[1] = fs.y; o[2] = fs.z;
        o[3] = ts.x; o[4] = ts.y; o[5] = ts.z;
    }
}

template <class M> __global__ __launch_bounds__(64 * COMPOSE_WPB) void rb_force_kernel(const float *root, const float *dof,
                                                                         const float *comp, int n,
                                                                         const float *mass_scale, const float *forces,
                                                                         const float *torques, int space, float *out,
                                                                         const float *props) {
    // COMPOSE_WPB envs per workgroup, one wavefront each (N single-wave
    // workgroups would be dispatch-bound)
    const int wv = threadIdx.x / 64;
    const int e = blockIdx.x * COMPOSE_WPB + wv;
    if (e >= n) return;
    __shared__ float T[COMPOSE_WPB][M::NL][12];   // link pose: R (9), p (3)
    __shared__ float F[COMPOSE_WPB][M::NL][10];   // link com (3), mass, force (3), torque (3)
    rb_force_env<M>(root, dof, comp, e, mass_scale, forces, torques, space, out, threadIdx.x % 64, T[wv], F[wv],
                    props, n);
}

// ---------------------------------------------------------------- contact row layout
// rows of shape s: shape_nrows[s] normal rows, then friction t1, t2 and --
// for a patch of several points -- torsion.  A one-point patch (torus,
// sphere) has no torsional friction: its torsion radius is the points' mean
// distance from their centroid, 0 (PhysX, too, applies none without a
// torsional patch radius, which the reference does not set)
template <class M> __device__ __forceinline__ constexpr int shape_nfric(int s) {
    return M::shape_nrows[s] == 1 ? 2 : 3;
}
template <class M> __device__ __forceinline__ constexpr int row_shape(int i) {
    int base = 0;
    for (int s = 0; s < M::NS; ++s) {
        if (i < base + M::shape_nrows[s] + shape_nfric<M>(s)) return s;
        base += M::shape_nrows[s] + shape_nfric<M>(s);
    }
    return 0;
}
// the contact group of row i (lane-dependent i): compares and selects against
// the model's row ranges, no table load
template <class M> __device__ __forceinline__ int row_cg(int i) {
    int r = M::shape_cg[0], base = 0;
#pragma unroll
    for (int sh = 0; sh < M::NS; ++sh) {
        r = i >= base ? M::shape_cg[sh] : r;
        base += M::shape_nrows[sh] + shape_nfric<M>(sh);
    }
    return r;
}
// the contact group's GROUP of row i (lane-dependent i): compares and
// selects, no table load
template <class M> __device__ __forceinline__ int row_group(int i) {
    int r = M::cgroup[M::shape_cg[0]], base = 0;
#pragma unroll
    for (int sh = 0; sh < M::NS; ++sh) {
        r = i >= base ? M::cgroup[M::shape_cg[sh]] : r;
        base += M::shape_nrows[sh] + shape_nfric<M>(sh);
    }
    return r;
}
// the most contact points (normal rows) of any shape of the model
template <class M> __device__ __forceinline__ constexpr int max_shape_rows() {
    int m = 0;
    for (int s = 0; s < M::NS; ++s) m = M::shape_nrows[s] > m ? M::shape_nrows[s] : m;
    return m;
}
// the shape of row i (lane-dependent i): compares and selects, no table load
template <class M> __device__ __forceinline__ int row_shape_sel(int i) {
    int r = 0, base = 0;
#pragma unroll
    for (int sh = 0; sh < M::NS; ++sh) {
        r = i >= base ? sh : r;
        base += M::shape_nrows[sh] + shape_nfric<M>(sh);
    }
    return r;
}
template <class M> __device__ __forceinline__ constexpr int row_base(int s) {
    int base = 0;
    for (int k = 0; k < s; ++k) base += M::shape_nrows[k] + shape_nfric<M>(k);
    return base;
}
// row k is a normal row (lane-dependent k): compares against the model's row ranges
template <class M> __device__ __forceinline__ bool row_normal(int k) {
    bool r = false;
    int base = 0;
#pragma unroll
    for (int sh = 0; sh < M::NS; ++sh) {
        r = (k >= base && k < base + M::shape_nrows[sh]) ? true : r;
        base += M::shape_nrows[sh] + shape_nfric<M>(sh);
    }
    return r;
}
// a normal row's velocity lower bound over a step dt at separation phi: the
// speculative approach bound above the rest offset, the Baumgarte push-out
// capped by max_depenetration_velocity below it (oracle/physics_ref.c row_target)
__device__ __forceinline__ float contact_target(const StepArgs &a, float phi, float dt) {
    return phi > a.rest ? -(phi - a.rest) / dt : fminf(a.baumgarte * (a.rest - phi) / dt, a.max_depen);
}
// physx.contact_offset: PhysX's pair rule (round 6).  A point
// generates a contact -- a speculative normal row -- only while its separation
// is below the pair's contact distance, the sum of the two shapes' offsets:
// the shape's and the ground plane's, both the scene's contact_offset, so 2 x
// contact_offset.  Beyond it the separation becomes TG_NO_ROW, whose target
// (-TG_NO_ROW / h) no row velocity reaches, so its multiplier stays 0 in every
// sweep (PGS and TGS sub-steps alike) and its patch's friction limit counts
// nothing from it.  Round 5's rule (one offset plus the point's free approach
// over the substep) gated rows in exactly where they start to matter: a foot
// corner whose free approach just reached the gate took a 1.15 N s impulse
// when present and none when absent, a discontinuity that rounding alone
// crossed (a GPU-only 0.2 rad/s outlier at 16384 envs, 24 of 48 one-ulp
// perturbed oracle replays on either side).  Distance alone
// gates at a separation no foot or wheel closes within a substep.
// oracle/physics_ref.c collect_rows applies the same rule.
#define TG_NO_ROW 1e30f
__device__ __forceinline__ float contact_row_phi(const StepArgs &a, float phi) {
    return (a.coff > 0.f && !(phi < 2.f * a.coff)) ? TG_NO_ROW : phi;
}

}  // namespace tg

#include "step_par.h"

namespace tg {

// ---------------------------------------------------------------- fused walk post-physics
// tg_walk_step's last simulate: the ThormangWalk post-physics step
// (walk_task.hip walk_post_kernel: progress, masked resets, observations,
// reward, termination, timeouts, pushes) as the step kernel's epilogue, LPE
// lanes per env (lane = dof mod LPE) on the final state the kernel holds, so
// the state is stored once (reset values for a reset env) and the separate
// launch disappears.  Same operations as walk_env; the fp contraction and
// reassociation are off here as in walk_task.hip, the transcendentals are this
// translation unit's (fast-math) ones.
struct WalkPost {
    static constexpr bool on = true;
    static constexpr bool T7_SYNC = false;
    static constexpr int NPRE = 0;
    static constexpr bool PM_OUT = true;   // stores the pre-physics' actions / targets (pm_in_step) below
    static constexpr bool TOUCH = true;
    using Args = WalkPostArgs;
    // the line of the epilogue's inputs lane `sub` touches in the last
    // substep (step_par.h EPI_TOUCH): progress, reset flag, last actions (two
    // lines), commands, the reset root state; the other lanes the first
    template <class M, int LPE>
    static __device__ __forceinline__ const float *touch_addr(const Args &pa, const StepArgs &, int e, int sub) {
        const tg_walk_buffers &b = pa.b;
        constexpr int D = M::ND;
        const float *la = b.last_actions + (size_t)e * D;
        switch (sub) {
        case 1: return reinterpret_cast<const float *>(b.reset_buf + e);
        case 2: return la;
        case 3: return la + (D - 1);
        case 4: return b.commands + 3 * (size_t)e;
        case 5: return b.root_reset + 13 * (size_t)e;
        default: return reinterpret_cast<const float *>(b.progress_buf + e);
        }
    }
    static __device__ __forceinline__ float clampw(float x, float lo, float hi) {
        return x < lo ? lo : (x > hi ? hi : x);
    }
    template <class M, int LPE>
    static __device__ __forceinline__ void epilogue(const Args &pa, const StepArgs &a, const LE &s, int e, bool owner,
                                                    int sub, const float *rt0, float *root, float *dofs,
                                                    const float *) {
#pragma clang fp contract(off) reassociate(off)
        constexpr int D = M::ND;
        constexpr int NR = (D + LPE - 1) / LPE;
        const tg_walk_params &p = pa.p;
        const tg_walk_buffers &b = pa.b;
        const uint32_t c_lo = pa.c_lo, c_hi = pa.c_hi;
        const bool lead = sub == 0;
        const size_t eD = (size_t)e * D;
        // every input of the env in one batch
        const int64_t prog1 = b.progress_buf[e] + 1;
        const bool reset = b.reset_buf[e] != 0;
        float q[NR], qd[NR], act[NR], la[NR], pt[NR], cmd[3], rt[13];
        // (the per-dof constants too: kernel-argument arrays indexed by lane
        // are memory loads, which would otherwise be issued where they are
        // used -- inside the reset branch and after it)
        float dpos[NR], kst[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int d = sub + LPE * r;
            q[r] = qd[r] = act[r] = la[r] = pt[r] = dpos[r] = kst[r] = 0.f;
            if (d < D) {
                dpos[r] = p.default_pos[d];
                kst[r] = p.stiffness[d];
                const int g = dof_group<M>(d);
                if (g > 0) {
                    q[r] = s(g * GF + F_Q);
                    qd[r] = s(g * GF + F_QD);
                } else {
                    q[r] = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
                }
                if (a.pm_in_step) {   // the pre-physics ran inside this kernel (pass 2a's targets)
                    act[r] = pm_clamp(a, a.pm_actions[eD + d]);
                    pt[r] = pm_target(a, d, act[r]);
                    if (owner) {   // pre_physics_step's outputs (a reset below zeroes the actions again)
                        a.pm_act_out[eD + d] = act[r];
                        a.pm_tgt_out[eD + d] = pt[r];
                    }
                } else {
                    act[r] = b.actions[eD + d];
                    pt[r] = b.pos_target[eD + d];
                }
                la[r] = b.last_actions[eD + d];
            }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) cmd[k] = b.commands[3 * (size_t)e + k];
        float tpl[2] = {0.f, 0.f};   // a reset's spawn (x, y)
        if (lead) {
            tpl[0] = b.root_reset[13 * (size_t)e];
            tpl[1] = b.root_reset[13 * (size_t)e + 1];
        }
#pragma unroll
        for (int k = 0; k < 13; ++k) rt[k] = rt0[k];
        const int64_t prog = reset ? 0 : prog1;
        if (reset) {
            // the env's 4 + 2D reset draws (walk_draw): Philox block j (draws
            // 4j .. 4j + 3) computed once, on lane j mod LPE, and staged in the
            // Delassus slots (dead after the contact solve) -- rather than one
            // block per draw on the lane that uses it
            using PL = ParLayout<M>;
            constexpr int NRD = 4 + 2 * D, NB = (NRD + 3) / 4;
            constexpr bool STAGE = PL::K * PL::K >= 4 * NB;
            if (STAGE && !pa.reset_draws) {
                for (int j = sub; j < NB; j += LPE) {
                    const U4 x = philox(U4{(uint32_t)e, c_lo, c_hi, 0x57524530u + (uint32_t)j}, (uint32_t)p.seed,
                                        (uint32_t)(p.seed >> 32));
                    s(PL::W + 4 * j) = u01(x.x);
                    s(PL::W + 4 * j + 1) = u01(x.y);
                    s(PL::W + 4 * j + 2) = u01(x.z);
                    s(PL::W + 4 * j + 3) = u01(x.w);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the env's lanes share a wavefront
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            auto rdraw = [&](int k) {
                if (!STAGE || pa.reset_draws) return walk_draw(p, pa.reset_draws, e, k, c_lo, c_hi);
                return s(PL::W + k);
            };
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int d = sub + LPE * r;
                if (d < D) {
                    q[r] = dpos[r] + (rdraw(4 + d) * 2.0f - 1.0f) * p.joint_noise;
                    qd[r] = 0.1f * (rdraw(4 + D + d) * 2.0f - 1.0f);
                    act[r] = la[r] = 0.f;
                    if (owner) b.actions[eD + d] = 0.f;
                }
            }
            if (lead) {
                float r4[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) r4[k] = rdraw(k);
                cmd[0] = p.cmd_vx[0] + r4[0] * (p.cmd_vx[1] - p.cmd_vx[0]);
                cmd[1] = p.cmd_vy[0] + r4[1] * (p.cmd_vy[1] - p.cmd_vy[0]);
                cmd[2] = p.cmd_wz[0] + r4[2] * (p.cmd_wz[1] - p.cmd_wz[0]);
                const float yaw = (r4[3] * 2.0f - 1.0f) * 3.14159265358979323846f;
                rt[0] = tpl[0];
                rt[1] = tpl[1];
                rt[2] = p.spawn_height;
                rt[3] = 0.0f;
                rt[4] = 0.0f;
                rt[5] = sinf(0.5f * yaw);
                rt[6] = cosf(0.5f * yaw);
#pragma unroll
                for (int k = 7; k < 13; ++k) rt[k] = 0.0f;
                if (owner) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) b.commands[3 * (size_t)e + k] = cmd[k];
                }
            }
        }
        // dof observations and the per-dof reward terms
        float *o = b.obs_buf + (size_t)p.num_obs * e;
        const float co = p.clip_obs;
        float rate = 0.0f, vel2 = 0.0f, tq = 0.0f;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int d = sub + LPE * r;
            if (d < D) {
                if (owner) {
                    o[13 + d] = clampw((q[r] - dpos[r]) * p.dof_pos_scale, -co, co);
                    o[13 + D + d] = clampw(qd[r] * p.dof_vel_scale, -co, co);
                    o[13 + 2 * D + d] = clampw(act[r], -co, co);
                    b.last_actions[eD + d] = act[r];   // (pm_in_step: actions / targets stored above)
                }
                rate += (act[r] - la[r]) * (act[r] - la[r]);
                vel2 += qd[r] * qd[r];
                const float tt = kst[r] * (pt[r] - q[r]);
                tq += tt * tt;
            }
        }
        rate = sum_lanes<LPE>(rate);
        vel2 = sum_lanes<LPE>(vel2);
        tq = sum_lanes<LPE>(tq);
        if (owner) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int d = sub + LPE * r;
                if (d < D) {
                    dofs[2 * d] = q[r];
                    dofs[2 * d + 1] = qd[r];
                }
            }
        }
        if (!lead || !owner) return;
#pragma unroll
        for (int k = 0; k < 13; ++k) root[k] = rt[k];
        b.progress_buf[e] = prog;
        const float x = rt[3], y = rt[4], z = rt[5], w = rt[6];
        const float Rw[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                             2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                             2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
        float vb[3], wb[3], gb[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            vb[k] = Rw[k] * rt[7] + Rw[3 + k] * rt[8] + Rw[6 + k] * rt[9];
            wb[k] = Rw[k] * rt[10] + Rw[3 + k] * rt[11] + Rw[6 + k] * rt[12];
            gb[k] = -Rw[6 + k];
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
        if (!b.body_force) return;
        // push wrench for the next simulate (walk_post_kernel)
        float *f = b.body_force + (size_t)6 * p.num_groups * e;
        const bool push = p.push_force > 0.0f && p.push_interval > 0 && prog > 0 && (prog % p.push_interval) == 0;
        float u[3] = {0.5f, 0.5f, 0.5f};
        if (pa.push_draws) {
#pragma unroll
            for (int k = 0; k < 3; ++k) u[k] = pa.push_draws[3 * (size_t)e + k];
        } else if (push) {   // (the block only where it is used)
            const U4 xx = philox(U4{(uint32_t)e, c_lo, c_hi, 0x50555348u}, (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
            u[0] = u01(xx.x); u[1] = u01(xx.y); u[2] = u01(xx.z);
        }
        f[0] = push ? p.push_force * (u[0] * 2.0f - 1.0f) : 0.0f;
        f[1] = push ? p.push_force * (u[1] * 2.0f - 1.0f) : 0.0f;
        f[2] = push ? 0.25f * p.push_force * (u[2] * 2.0f - 1.0f) : 0.0f;
        f[3] = 0.0f; f[4] = 0.0f; f[5] = 0.0f;
    }
};

// ---------------------------------------------------------------- translating locks
// The lock group's composite and the placements below its translating locks
// (CompLayout ext) at new lock positions q[k], from the moments the last
// compose stored -- what a compose at those positions would write, without
// re-composing the env.  Moving lock k by dq_k translates the links below it
// by u_k = dq_k w_k, so with D_l = sum of the u_k above link l:
//   S'  = S + sum_k m_k u_k
//   Io' = Io + sum_k [2 (S_k . u_k) E - (S_k u_k^T + u_k S_k^T)]
//            + sum_{k,k'} m_{max(k,k')} ((u_k . u_k') E - u_k u_k'^T)
// (nested locks: the links below both are the deeper one's), c' = S'/m,
// I_com = Io' - m (|c'|^2 E - c' c'^T); placements and shape poses below a lock
// move by the sum of its u_k, in the joint-aligned frame of the lock group.
// c: the env's composite cache (written); xe: its extension (read)
template <class M> __device__ __forceinline__ void tl_update(float *c, const float *xe, const float *q) {
    using CL = CompLayout<M>;
    constexpr int gt = M::tl_group;
    const float *x = xe;
    auto X = [&](int off) { return xe + (off - CL::ext()); };
    const float m = x[0];
    V3 S = v3(x[1], x[2], x[3]);
    float Io[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) Io[k] = x[4 + k];
    V3 u[M::NTL];
    float mk[M::NTL];
#pragma unroll
    for (int k = 0; k < M::NTL; ++k) {
        const float *xk = X(CL::xk(k));
        const float dq = q[k] - xk[0];
        mk[k] = xk[1];
        const V3 Sk = v3(xk[2], xk[3], xk[4]);
        u[k] = dq * v3(xk[5], xk[6], xk[7]);
        S = S + mk[k] * u[k];
        const float su = dot(Sk, u[k]);
        Io[0] += 2.f * (su - Sk.x * u[k].x);
        Io[1] += 2.f * (su - Sk.y * u[k].y);
        Io[2] += 2.f * (su - Sk.z * u[k].z);
        Io[3] -= Sk.x * u[k].y + u[k].x * Sk.y;
        Io[4] -= Sk.x * u[k].z + u[k].x * Sk.z;
        Io[5] -= Sk.y * u[k].z + u[k].y * Sk.z;
    }
#pragma unroll
    for (int k = 0; k < M::NTL; ++k)
#pragma unroll
        for (int j = 0; j < M::NTL; ++j) {
            const float mm = mk[k > j ? k : j];
            const float uu = dot(u[k], u[j]);
            Io[0] += mm * (uu - u[k].x * u[j].x);
            Io[1] += mm * (uu - u[k].y * u[j].y);
            Io[2] += mm * (uu - u[k].z * u[j].z);
            Io[3] -= mm * u[k].x * u[j].y;
            Io[4] -= mm * u[k].x * u[j].z;
            Io[5] -= mm * u[k].y * u[j].z;
        }
    const V3 cc = (m > 0.f ? 1.0f / m : 0.f) * S;
    const float c2 = dot(cc, cc);
    float gI[6] = {Io[0] - m * (c2 - cc.x * cc.x), Io[1] - m * (c2 - cc.y * cc.y), Io[2] - m * (c2 - cc.z * cc.z),
                   Io[3] + m * cc.x * cc.y, Io[4] + m * cc.x * cc.z, Io[5] + m * cc.y * cc.z};
    const M3 Q = M3{{M::gq[gt][0], M::gq[gt][1], M::gq[gt][2], M::gq[gt][3], M::gq[gt][4], M::gq[gt][5],
                     M::gq[gt][6], M::gq[gt][7], M::gq[gt][8]}};
    const V3 cq = mulT(Q, cc);
    float gIq[6];
    sym_from(gIq, mul(mul(transpose(Q), sym_to(gI)), Q));
    float *ci = c + CL::inertia(gt);
    ci[0] = m;
    ci[1] = cq.x; ci[2] = cq.y; ci[3] = cq.z;
#pragma unroll
    for (int k = 0; k < 6; ++k) ci[4 + k] = gIq[k];
    auto shift = [&](int mask) {
        V3 d = v3(0, 0, 0);
#pragma unroll
        for (int k = 0; k < M::NTL; ++k)
            if ((mask >> k) & 1) d = d + u[k];
        return mulT(Q, d);
    };
#pragma unroll
    for (int j = 0; j < M::NAG; ++j) {
        const V3 t = v3(X(CL::xag(j))[0], X(CL::xag(j))[1], X(CL::xag(j))[2]) + shift(M::ag_mask[j]);
        float *cx = c + CL::xtree(M::ag_group[j]);
        cx[9] = t.x; cx[10] = t.y; cx[11] = t.z;
    }
#pragma unroll
    for (int j = 0; j < M::NASH; ++j) {
        const V3 t = v3(X(CL::xash(j))[0], X(CL::xash(j))[1], X(CL::xash(j))[2]) + shift(M::ash_mask[j]);
        float *cs = c + CL::shape(M::ash_shape[j]);
        cs[9] = t.x; cs[10] = t.y; cs[11] = t.z;
    }
}

// ---------------------------------------------------------------- fused Gogoro post-physics
// tg_gogoro_step's last simulate: gogoro_task.hip post_kernel (progress,
// masked resets with their property writes and dirty flag, observations,
// reward, sensor noise, command resampling, timeouts) as the step kernel's
// epilogue, LPE lanes per env on the final state it holds: the 9 Philox
// blocks run on the env's lanes at once (lane l block l, the lead lane also
// block 8) and reach the lead lane by DPP row broadcasts; a reset env's dof
// rows are written by all its lanes; the lead lane does the task math.  The
// state is stored once (the reset state for a reset env), and the separate
// post launch and its re-read of the state disappear.  Same counters, draws
// and fp32 operations (gogoro_math.h) as post_kernel.
struct GogoroPost {
    static constexpr bool on = true;
    static constexpr bool T7_SYNC = false;
    static constexpr bool PM_OUT = false;
    static constexpr bool TOUCH = false;
    using Args = GogoroPostArgs;
    // the translating-lock extension of an env the previous step reset (its
    // reset happens in this epilogue), LPE lanes x NPRE floats, loaded at
    // kernel start so its latency hides behind the whole step
    static constexpr int NPRE = 5;
    template <class M, int LPE>
    static __device__ __forceinline__ void prefetch(const Args &pa, const StepArgs &a, int e, int sub, float *x) {
#pragma unroll
        for (int k = 0; k < NPRE; ++k) x[k] = 0.f;
        if constexpr (M::NTL > 0) {
            static_assert(M::KX <= NPRE * LPE, "extension prefetch: KX <= NPRE x LPE");
            if (pa.tl_inplace && pa.b.reset_buf[e] != 0) {
                const float *xs = a.comp + (size_t)e * M::KC + CompLayout<M>::ext();
#pragma unroll
                for (int k = 0; k < NPRE; ++k) {
                    const int i = sub * NPRE + k;
                    if (i < M::KX) x[k] = xs[i];
                }
            }
        }
    }
    template <class M, int LPE>
    static __device__ __forceinline__ void epilogue(const Args &pa, const StepArgs &a, const LE &s, int e, bool owner,
                                                    int sub, const float *rt0, float *root, float *dofs,
                                                    const float *xpre) {
#pragma clang fp contract(off) reassociate(off)
        constexpr int D = M::ND;
        constexpr int NR = (D + LPE - 1) / LPE;
        static_assert(LPE >= 8, "the 9 draw blocks need 8 lanes per env");
        const tg_gogoro_params &p = pa.p;
        const tg_gogoro_buffers &b = pa.b;
        const bool lead = sub == 0;
        const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
        // ---- the prefetched extension to the env's dead Delassus slots (read
        // by the lead lane if the env resets)
        if constexpr (M::NTL > 0) {
#pragma unroll
            for (int k = 0; k < NPRE; ++k) {
                const int i = sub * NPRE + k;
                if (i < M::KX) s(ParLayout<M>::W + i) = xpre[k];
            }
            static_assert(M::KX <= ParLayout<M>::K * ParLayout<M>::K + 8 * ParLayout<M>::K,
                          "the extension fits the dead Delassus / row slots");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the env's lanes share a wavefront
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // ---- inputs, one batch
        const int64_t prog1 = b.progress_buf[e] + 1;
        const bool rflag = b.reset_buf[e] != 0;
        float rt[13], ah[5];
#pragma unroll
        for (int k = 0; k < 13; ++k) rt[k] = rt0[k];
        float cmdc;
        if constexpr (ParLayout<M>::TPON) {
            if (a.gp_in_step) {   // this kernel's pre-physics values (LDS), not yet-unflushed HBM
#pragma unroll
                for (int k = 0; k < 5; ++k) ah[k] = s(ParLayout<M>::TP + k);
                cmdc = s(ParLayout<M>::TP + 5);
            } else {
#pragma unroll
                for (int k = 0; k < 5; ++k) ah[k] = b.action_history[5 * (size_t)e + k];
                cmdc = b.curent_command[e];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 5; ++k) ah[k] = b.action_history[5 * (size_t)e + k];
            cmdc = b.curent_command[e];
        }
        float yawc = b.yaw_command[e], imu = b.imu_offsets[e];
        float tpl[3];   // a reset's spawn (x, y, z) and pose, with the other inputs rather than inside the reset branch
#pragma unroll
        for (int k = 0; k < 3; ++k) tpl[k] = b.root_reset[13 * (size_t)e + k];
        float pose[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) pose[rr] = sub + LPE * rr < D ? b.thormang_pose[sub + LPE * rr] : 0.f;
        // ---- draws: lane l < 8 block l, the lead lane also block 8 (command resample)
        float v[3], v8[3];
        gogoro_post_block(sub < 8 ? sub : 7, e, pa.c_lo, pa.c_hi, k0, k1, v);
        gogoro_post_block(8, e, pa.c_lo, pa.c_hi, k0, k1, v8);
        auto slot = [&](int x) {   // exchange slot x = 3 l + j of block l, from lane l
            const int l = x / 3, j = x % 3;
            return env_bcast<LPE>(j == 0 ? v[0] : (j == 1 ? v[1] : v[2]), l, sub);
        };
        float r[TG_GOGORO_RESET_DRAWS], nd[5];
#pragma unroll
        for (int k = 0; k < TG_GOGORO_RESET_DRAWS; ++k) r[k] = slot(GOGORO_RSLOT[k]);
#pragma unroll
        for (int k = 0; k < 5; ++k) nd[k] = slot(GOGORO_NSLOT[k]);
        float su = v8[0], yu = v8[1];
        // replayed draws (parity tests: the reference's recorded stream) in
        // place of the Philox values, the same arithmetic after this point
        if (pa.reset_draws && rflag) {
#pragma unroll
            for (int k = 0; k < TG_GOGORO_RESET_DRAWS; ++k) r[k] = pa.reset_draws[(size_t)e * TG_GOGORO_RESET_DRAWS + k];
        }
        if (pa.obs_draws) {
#pragma unroll
            for (int k = 0; k < 5; ++k) nd[k] = pa.obs_draws[(size_t)e * 5 + k];
        }
        if (pa.speed_draws) {
            su = pa.speed_draws[e];
            yu = pa.yaw_draws[e];
        }
        int64_t prog = prog1;
        if (rflag) {
            // reset_env: dof rows (every lane), the rest on the lead lane
            if (owner) {
#pragma unroll
                for (int rr = 0; rr < NR; ++rr) {
                    const int d = sub + LPE * rr;
                    if (d < D) {
                        dofs[2 * d] = pose[rr];
                        dofs[2 * d + 1] = 0.0f;
                    }
                }
            }
            const float target = (r[3] * 2.0f - 1.0f) * F_PI;
            const float rot = target + u_aff(-1.57f, 1.57f, r[4]);
            const float hh = rot / 2.0f;
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
            if (owner && lead) {
                b.curent_speed[e] = u_aff(p.speed_range[0], p.speed_range[1], r[0]);
                b.speed_offset[e] = u_aff(p.speed_sensor_offset[0], p.speed_sensor_offset[1], r[2]);
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
                prop[TG_PROP_DAMPING * ND + st] =
                    u_aff(p.steering_damping_range[0], p.steering_damping_range[1], r[10]);
                prop[TG_PROP_EFFORT * ND + st] = p.steer_effort;
                prop[TG_PROP_VELOCITY * ND + st] = p.steer_velocity;
                bool inplace = false;
                if constexpr (M::NTL > 0) inplace = pa.tl_inplace != 0;
                if (inplace) {
                    // the new seat windows only translate the rider: update the
                    // composite in place (tl_update) -- no compose for this env
                    constexpr int NT = M::NTL > 0 ? M::NTL : 1;
                    float qn[NT];
#pragma unroll
                    for (int k = 0; k < M::NTL; ++k) {
                        qn[k] = 0.f;
#pragma unroll
                        for (int j = 0; j < 3; ++j)
                            if (seat[j] == M::tl_dof[k]) qn[k] = 0.5f * (cv[j] + (cv[j] + 0.0001f));
                    }
                    if constexpr (M::NTL > 0) tl_update<M>(a.comp + (size_t)e * M::KC, s.b + ParLayout<M>::W, qn);
                } else {
                    b.env_dirty[e] = 1;
                    if (pa.reset_list) pa.reset_list[atomicAdd(pa.reset_count, 1)] = e;   // for compose_list_kernel
                }
                b.curent_command[e] = 0.0f;
#pragma unroll
                for (int k = 0; k < 5; ++k) b.action_history[5 * (size_t)e + k] = 0.0f;
            }
            prog = 0;
        } else if (owner) {
            // the simulated state: active dofs from LDS, locked ones at their window centre
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int d = sub + LPE * rr;
                if (d < D) {
                    const int g = dof_group<M>(d);
                    if (g > 0) {
                        dofs[2 * d] = s(g * GF + F_Q);
                        dofs[2 * d + 1] = s(g * GF + F_QD);
                    } else {
                        dofs[2 * d] = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
                        dofs[2 * d + 1] = 0.f;
                    }
                }
            }
        }
        if (!lead || !owner) return;
#pragma unroll
        for (int k = 0; k < 13; ++k) root[k] = rt[k];
        float o[6];
        observation(rt, yawc, cmdc, o);
        bool felt;
        const float rew = gogoro_reward(o, ah, felt);
        const bool finished = prog >= p.max_episode_length - 1;
        const int64_t reset = (finished || felt) ? 1 : 0;
        float rr[6];
        noisy_observation(p, o, nd, imu, rr);
        float yc = yawc;
        if (prog == p.yaw_freq_update) yc = u_aff(-F_PI, F_PI, yu);
        if (yc > F_PI) yc = yc - F_2PI;
        if (yc < -F_PI) yc = yc + F_2PI;
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
};

}  // namespace tg

#include "paper_math.h"

namespace tg {

// ---------------------------------------------------------------- fused paper post-physics
// Reward term 7 inside the step launch (PaperPost): every workgroup published
// its block sum in the prologue (paper_t7_block<true>: an agent-scope store,
// its completion waited for, then one agent-scope add to the arrival
// counter).  Each wavefront polls the counter from one lane until every block
// of this launch has arrived -- bounded: a timeout raises bit 2 of the sticky
// error word (tg_sync reports it) and the sum goes on with what is there, so
// no wave can spin forever -- then reads the block sums with agent-scope loads
// (MI355X_MICROARCH.md's hand-off form: scope-1 stores, a waited store before
// the counter add, scope-1 loads after the matched poll) and adds them in
// t7_batch_sum's canonical order: virtual thread t < TG_PAPER_T7_THREADS adds
// blocks t, t + TG_PAPER_T7_THREADS, ...; an xor butterfly per virtual
// wavefront; the wavefront sums in order (the post launch's total bit for bit).
// (A/B, profiles/r6/paper_one_launch_ab.txt: reading the count a substep
// ahead measured no gain)
// (c0: the count as lane 0 read it before, with the epilogue's first batch)
__device__ __forceinline__ double paper_t7_wait_sum(const double *t7, unsigned *cnt, unsigned target, int nblk,
                                                    int *err, unsigned c0) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        unsigned it = 0, c = c0;
        while ((int)(c - target) < 0) {
            if (++it > (1u << 20)) {   // ~1 s: a workgroup never became resident
                if (err) atomicOr(err, 2);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    constexpr int VW = TG_PAPER_T7_THREADS / 64;
    const unsigned long long *src = reinterpret_cast<const unsigned long long *>(t7);
    double v[VW];
#pragma unroll
    for (int w = 0; w < VW; ++w) {
        const int c = lane + 64 * w;
        v[w] = c < nblk ? __longlong_as_double((long long)__hip_atomic_load(src + c, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT))
                        : 0.0;
    }
    double tot = 0.0;
    {
#pragma clang fp contract(off) reassociate(off)
#pragma unroll
        for (int w = 0; w < VW; ++w) {
            double x = 0.0;
            x += v[w];   // (a virtual thread's one block: nblk <= TG_PAPER_T7_THREADS, checked by the host)
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
            tot += x;
        }
    }
    return tot;
}

// b.rb_forces [N*L,3] (world forces at the link coms) reduced to env e's
// group wrenches [G,6] by the env's LN lanes -- rb_force_env's composite-cache
// path (link = lane mod LN, group = lane), the same operations per link and
// the same link order per group sum.  load(): the inputs no epilogue store
// changes (the lane's link forces and coms, its group's joint placement, the
// lock extension); finish(): the state the epilogue's stores change -- root
// orientation, joint angles, lock windows -- and the one force row the
// epilogue itself rewrote (the head push, plink: its link, -1 none), all read
// after the stores (fence before); T: 9 x NG, F: 6 x NL floats of the env's
// LDS.
template <class M, int LN> struct RbLanes {
    static_assert(M::LCOM && M::NG <= LN, "one group per lane");
    static constexpr int NLL = (M::NL + LN - 1) / LN;
    static constexpr int NT = M::NTL > 0 ? M::NTL : 1;
    using CL = CompLayout<M>;
    V3 f[NLL], lc[NLL], gc[NLL];
    M3 Rpc;
    float xk0[NT];
    V3 xka[NT];
    __device__ __forceinline__ void load(const float *comp, int e, const float *forces, int sub) {
        const float *c = comp + (size_t)e * M::KC;
#pragma unroll
        for (int k = 0; k < NLL; ++k) {
            const int l = sub + LN * k;
            f[k] = lc[k] = gc[k] = v3(0, 0, 0);
            if (l < M::NL) {
                const int gl = M::link_group[l];
                const size_t i = (size_t)e * M::NL + l;
                f[k] = v3(forces[3 * i], forces[3 * i + 1], forces[3 * i + 2]);
                lc[k] = v3(c[CL::lcom(l)], c[CL::lcom(l) + 1], c[CL::lcom(l) + 2]);
                gc[k] = v3(c[CL::inertia(gl) + 1], c[CL::inertia(gl) + 2], c[CL::inertia(gl) + 3]);
            }
        }
        const bool hg = sub > 0 && sub < M::NG;
        const int g = hg ? sub : 1 % M::NG;
#pragma unroll
        for (int k = 0; k < 9; ++k) Rpc.a[k] = hg ? c[CL::xtree(g) + k] : 0.f;
        if constexpr (M::NTL > 0) {
#pragma unroll
            for (int k = 0; k < M::NTL; ++k) {
                const float *xk = c + CL::xk(k);
                xk0[k] = xk[0];
                xka[k] = v3(xk[5], xk[6], xk[7]);
            }
        }
    }
    __device__ __forceinline__ void finish(const float *root, const float *dof, const float *forces, int plink,
                                           int e, float *out, int sub, float *T, float *F, const float *props, int N,
                                           bool store) {
#pragma clang fp contract(off) reassociate(off)
        auto wsync = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        const float *r = root + 13 * (size_t)e;
        const float *q = dof + 2 * (size_t)e * M::ND;
        const bool hg = sub > 0 && sub < M::NG;
        const int g = hg ? sub : 1 % M::NG;
        float qj = 0.f;
        if (hg && M::jtype[g] == TG_JOINT_REVOLUTE) qj = q[2 * M::gdof[g]];
        const float qx = r[3], qy = r[4], qz = r[5], qw = r[6];
        if (plink >= 0) {   // the row this epilogue rewrote, re-read by the lane that holds it
            const size_t i = (size_t)e * M::NL + (plink < M::NL ? plink : 0);
            const bool mine = plink % LN == sub;
            const V3 fp = mine ? v3(forces[3 * i], forces[3 * i + 1], forces[3 * i + 2]) : v3(0, 0, 0);
#pragma unroll
            for (int k = 0; k < NLL; ++k) {   // (selects: a per-k branch folds to a dynamically indexed store)
                const bool hit = mine && sub + LN * k == plink;
                f[k].x = hit ? fp.x : f[k].x;
                f[k].y = hit ? fp.y : f[k].y;
                f[k].z = hit ? fp.z : f[k].z;
            }
        }
        V3 ush[NT];
        if constexpr (M::NTL > 0) {
            const size_t ND = (size_t)N * M::ND;
#pragma unroll
            for (int k = 0; k < M::NTL; ++k) {
                const size_t id = (size_t)e * M::ND + M::tl_dof[k];
                const float qc = 0.5f * (props[TG_PROP_LOWER * ND + id] + props[TG_PROP_UPPER * ND + id]);
                ush[k] = (qc - xk0[k]) * xka[k];
            }
        }
        bool act = false;
#pragma unroll
        for (int k = 0; k < NLL; ++k)
            act = act || f[k].x != 0.f || f[k].y != 0.f || f[k].z != 0.f;
        // the env's lanes: any force at all (else zero wrenches, no kinematics)
        const unsigned long long envm = ((LN == 64) ? ~0ull : ((1ull << LN) - 1)) << ((threadIdx.x & 63) / LN * LN);
        if ((__ballot(act) & envm) == 0) {
            if (store)
                for (int k = sub; k < 6 * M::NG; k += LN) out[(size_t)e * 6 * M::NG + k] = 0.f;
            return;
        }
        M3 R = Rpc;
        if (hg && M::jtype[g] == TG_JOINT_REVOLUTE) {   // Rpc Rz(q), as step pass 1a
            float sq, cq;
            tg_sincos(qj, &sq, &cq);
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const float c0 = R.a[3 * rr], c1 = R.a[3 * rr + 1];
                R.a[3 * rr] = c0 * cq + c1 * sq;
                R.a[3 * rr + 1] = c1 * cq - c0 * sq;
            }
        }
        constexpr int GD = max_group_depth<M>();
        for (int lev = 0; lev <= GD; ++lev) {
            if (lev == 0 && sub == 0) {
                const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
                const M3 W = mul(quat_to_m3(qx * in, qy * in, qz * in, qw * in),
                                 M3{{M::gq[0][0], M::gq[0][1], M::gq[0][2], M::gq[0][3], M::gq[0][4], M::gq[0][5],
                                     M::gq[0][6], M::gq[0][7], M::gq[0][8]}});
#pragma unroll
                for (int k = 0; k < 9; ++k) T[k] = W.a[k];
            } else if (lev > 0 && hg && group_depth<M>(g) == lev) {
                M3 Wp;
#pragma unroll
                for (int k = 0; k < 9; ++k) Wp.a[k] = T[9 * M::parent[g] + k];
                const M3 W = mul(Wp, R);
#pragma unroll
                for (int k = 0; k < 9; ++k) T[9 * g + k] = W.a[k];
            }
            wsync();
        }
#pragma unroll
        for (int k = 0; k < NLL; ++k) {
            const int l = sub + LN * k;
            if (l < M::NL) {
                const int gl = M::link_group[l];
                M3 W;
#pragma unroll
                for (int j = 0; j < 9; ++j) W.a[j] = T[9 * gl + j];
                V3 lck = lc[k];
                if constexpr (M::NTL > 0) {
                    if (gl == M::tl_group && M::link_tl[l]) {
                        V3 sh = v3(0, 0, 0);
#pragma unroll
                        for (int j = 0; j < M::NTL; ++j)
                            if ((M::link_tl[l] >> j) & 1) sh = sh + ush[j];
                        const float *qg = M::gq[gl];
                        lck = lck + mulT(M3{{qg[0], qg[1], qg[2], qg[3], qg[4], qg[5], qg[6], qg[7], qg[8]}}, sh);
                    }
                }
                const V3 tq = v3(0, 0, 0) + cross(mul(W, lck - gc[k]), f[k]);
                F[6 * l + 0] = f[k].x; F[6 * l + 1] = f[k].y; F[6 * l + 2] = f[k].z;
                F[6 * l + 3] = tq.x; F[6 * l + 4] = tq.y; F[6 * l + 5] = tq.z;
            }
        }
        wsync();
        for (int j = sub; j < 6 * M::NG; j += LN) {
            float acc = 0.f;
            const int gsel = j / 6, cmp = j % 6;
            rbf_for_groups<0, M::NG>([&](auto G) {
                constexpr int gg = decltype(G)::value;
                if (gsel == gg) {
#pragma unroll
                    for (int k = 0; k < M::group_nlinks[gg]; ++k) acc += F[6 * M::group_links[gg][k] + cmp];
                }
            });
            if (store) out[(size_t)e * 6 * M::NG + j] = acc;
        }
    }
};

// tg_paper_step's simulate when the whole launch is resident at once: the
// GogoroPaper post-physics (gogoro_paper_task.hip paper_post_kernel: masked
// reset_idx, the 20-step clean / noisy histories, rewards with reward term 7's
// batch mean, command changes, head pushes, the push tensor reduced to the
// next simulate's group wrenches) as the step kernel's epilogue, LPE lanes per
// env (lane = history entry / dof / link mod LPE) on the final state the
// kernel holds: the whole GogoroPaper step in one launch.
// The same helpers (paper_math.h), Philox blocks and sum order as the post
// kernel; this unit's transcendentals and the physics' fp contraction in the
// link kinematics are the differences (tests/test_gpu_paper.py).
#ifndef TG_PAPER_T7_END
#define TG_PAPER_T7_END 1   // developer switch: 0 = reward term 7's batch sum before the histories (A/B)
#endif
struct PaperPost {
    static constexpr bool on = true;
    static constexpr bool PM_OUT = false;
    static constexpr bool TOUCH = false;
    static constexpr bool T7_SYNC = true;
    using Args = PaperPostArgs;
    // the translating-lock extension of an env the previous step flagged for
    // reset (its reset happens in this epilogue), as GogoroPost
    static constexpr int NPRE = 5, NXP = 5;
    template <class M, int LPE>
    static __device__ __forceinline__ void prefetch(const Args &pa, const StepArgs &a, int e, int sub, float *x) {
#pragma unroll
        for (int k = 0; k < NPRE; ++k) x[k] = 0.f;
        if constexpr (M::NTL > 0) {
            static_assert(M::KX <= NXP * LPE, "extension prefetch: KX <= NXP x LPE");
            if (pa.b.reset_buf[e] != 0) {
                const float *xs = a.comp + (size_t)e * M::KC + CompLayout<M>::ext();
#pragma unroll
                for (int k = 0; k < NXP; ++k) {
                    const int i = sub * NXP + k;
                    if (i < M::KX) x[k] = xs[i];
                }
            }
        }
    }
    template <class M, int LPE>
    static __device__ __forceinline__ void epilogue(const Args &pa, const StepArgs &a, const LE &s, int e, bool owner,
                                                    int sub, const float *rt0, float *root, float *dofs,
                                                    const float *xpre) {
        using namespace paper;
        constexpr int D = M::ND;
        constexpr int NR = (D + LPE - 1) / LPE;     // dof rows per lane
        constexpr int NH = (PHO + LPE - 1) / LPE;   // history entries per lane
        static_assert(LPE >= 8, "the 8 Philox blocks need 8 lanes per env");
        static_assert(M::NTL > 0 && (M::FUSED & 4), "in-place seat composites (the paper model)");
        using PL = ParLayout<M>;
        // the env's LDS after the state stores: the extension at W (reset
        // envs), the draws / newest entries after it; the force reduction's
        // T / F from 0 once those are consumed
        constexpr int XO = PL::W, SX = PL::W + ((M::KX + 3) & ~3);
        constexpr int DR = SX, OB = SX + 32, NZ = SX + 40;
        static_assert(NZ + PO <= PL::ES && 9 * M::NG + 6 * M::NL <= PL::ES, "epilogue scratch in the env's LDS");
        const tg_paper_params &p = pa.p;
        const tg_paper_buffers &b = pa.b;
        const bool lead = sub == 0;
        auto wsync = [] {   // the env's lanes share a wavefront
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        // ---- inputs, one batch
        const bool rflag = b.reset_buf[e] != 0;
        const int64_t prog0 = b.progress_buf[e] + 1;
        float *bo = b.buffer_obs + (size_t)PHO * e, *bn = b.buffer_obs_noisy + (size_t)PHO * e;
        float vc[NH], vn[NH];
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int i = sub + LPE * j;
            vc[j] = vn[j] = 0.0f;
            if (i < PHO - PO) {
                vc[j] = bo[i + PO];
                vn[j] = bn[i + PO];
            }
        }
        float pose[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
            const int d = sub + LPE * rr;
            pose[rr] = d < D ? b.thormang_pose[(size_t)e * D + d] : 0.f;
        }
        PaperLead L;
        float tpl[13], old6 = 0.0f;
#pragma unroll
        for (int k = 0; k < 13; ++k) L.root[k] = rt0[k];
        L.speed = L.speed_off = L.imu_off = L.yaw_cmd = L.cmd = 0.f;
        L.delay = 0;
        if (lead) {
            const float *tp = b.root_reset + 13 * (size_t)e;
#pragma unroll
            for (int k = 0; k < 13; ++k) tpl[k] = tp[k];
            L.speed = b.curent_speed[e];
            L.speed_off = b.curent_speed_offset[e];
            L.imu_off = b.curent_imu_x_offset[e];
            L.yaw_cmd = b.yaw_command[e];
            L.cmd = b.curent_command[e];
            L.delay = b.steer_delay[e];
            old6 = bo[(PH - 1) * PO + 6];
        }
        // the step's 8 Philox blocks (reset 3, noise 2, speed, yaw, push), block l on lane l
        float dv[4] = {0.f, 0.f, 0.f, 0.f};
        if (sub < 8) {
            const U4 x = philox(U4{(uint32_t)e, pa.c_lo, pa.c_hi, post_block_tag(sub)}, (uint32_t)p.seed,
                                (uint32_t)(p.seed >> 32));
            dv[0] = u01(x.x);
            dv[1] = u01(x.y);
            dv[2] = u01(x.z);
            dv[3] = u01(x.w);
        }
        // reward term 7's batch sum (every workgroup's prologue published its block)
        // the term-7 arrival count, read with the first batch; the batch sum
        // itself waits until the end (TG_PAPER_T7_END), where its loads overlap
        // the epilogue's store drain
        const unsigned c0 = (threadIdx.x & 63) == 0 ? __hip_atomic_load(pa.t7_count, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) : 0u;
        double tot = 0.0;
        if (!TG_PAPER_T7_END) tot = paper_t7_wait_sum(a.pp.t7, pa.t7_count, pa.t7_target, pa.nblk, a.err, c0);
        // ---- the extension and the draws to the env's LDS
        if constexpr (M::NTL > 0) {
#pragma unroll
            for (int k = 0; k < NXP; ++k) {
                const int i = sub * NXP + k;
                if (i < M::KX) s(XO + i) = xpre[k];
            }
        }
        if (sub < 8) {
#pragma unroll
            for (int k = 0; k < 4; ++k) s(DR + 4 * sub + k) = dv[k];
        }
        wsync();
        auto draw = [&](int k, int blk) { return s(DR + 4 * (blk + (k >> 2)) + (k & 3)); };
        const int64_t prog = rflag ? 0 : prog0;
        // ---- the state: a reset env's reset values, else the simulated state
        if (rflag) {
            if (owner) {
#pragma unroll
                for (int rr = 0; rr < NR; ++rr) {
                    const int d = sub + LPE * rr;
                    if (d < D) {
                        dofs[2 * d] = pose[rr];
                        dofs[2 * d + 1] = 0.0f;
                    }
                }
                for (int i = sub; i < PC; i += LPE) b.command_history[PC * (size_t)e + i] = 0.0f;
            }
#pragma unroll
            for (int j = 0; j < NH; ++j) vc[j] = vn[j] = 0.0f;
            if (lead) {
                float r[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) r[k] = draw(k, 0);
                if (owner) reset_lead<M>(p, b, e, r, tpl, L, a.comp, &s(XO));
                old6 = 0.0f;
            }
        } else if (owner) {
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int d = sub + LPE * rr;
                if (d < D) {
                    const int g = dof_group<M>(d);
                    if (g > 0) {
                        dofs[2 * d] = s(g * GF + F_Q);
                        dofs[2 * d + 1] = s(g * GF + F_QD);
                    } else {
                        dofs[2 * d] = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
                        dofs[2 * d + 1] = 0.f;
                    }
                }
            }
            if (lead) {
#pragma unroll
                for (int k = 0; k < 13; ++k) root[k] = rt0[k];
                b.progress_buf[e] = prog0;
            }
        }
        // ---- the newest clean / noisy entries (lead lane) through LDS
        if (lead) {
            float u[6], o[PO], l[PO];
#pragma unroll
            for (int k = 0; k < 6; ++k) u[k] = draw(k, 3);
            entries(p, L, old6, u, o, l);
#pragma unroll
            for (int k = 0; k < PO; ++k) {
                s(OB + k) = o[k];
                s(NZ + k) = l[k];
            }
            if (owner) b.speed_no_noise[e] = o[4];
        }
        wsync();
        // ---- both histories shifted by one entry, the new one appended
#pragma unroll
        for (int j = 0; j < NH; ++j) {
            const int i = sub + LPE * j;
            if (i < PHO) {
                if (i >= PHO - PO) {
                    vc[j] = s(OB + i - (PHO - PO));
                    vn[j] = s(NZ + i - (PHO - PO));
                }
                if ((i % PO) == 1) vn[j] = 0.0f;   // noisy[:, :, 1] = 0
                if (owner) {
                    bo[i] = vc[j];
                    bn[i] = vn[j];
                    b.obs_buf[(size_t)PHO * e + i] = vn[j];
                }
            }
        }
        // ---- rewards, resets, time_outs, command changes, pushes (lead lane)
        float rew = 0.f, tilt = 0.f;
        if (lead && owner) {
            float last[PO];
#pragma unroll
            for (int k = 0; k < PO; ++k) last[k] = s(OB + k);
            rew = reward15(p, last);
            tilt = last[0];
            if (!TG_PAPER_T7_END) finish_env(p, b, e, tot, tilt, prog, rew);
            commands(p, b, e, prog, L, last, draw(0, 5), draw(0, 6), draw(0, 7), draw(1, 7));
        }
        if (b.body_force && owner) {
            float *wr = b.body_force + (size_t)6 * p.num_groups * e;
            for (int i = 6 + sub; i < 6 * p.num_groups; i += LPE) wr[i] = 0.0f;
        }
        // ---- the push tensor reduced to the next simulate's group wrenches,
        // on this epilogue's root / dofs / seat windows / pushes
        if (pa.rb_out) {
            // the head-push row, when the push tensor holds it (the task's
            // [N, L, 3] tensor; perturbation = its head_p_link rows)
            const long off = (long)(b.perturbation + (size_t)(p.perturbation_stride ? p.perturbation_stride : 3) * e -
                                    (b.rb_forces + (size_t)3 * M::NL * e));
            const int plink = (off >= 0 && off < 3 * M::NL && off % 3 == 0) ? (int)(off / 3) : -1;
            wsync();   // (the LDS scratch above is consumed)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // (every input after the stores: the static ones with the
            // epilogue's first batch, or behind the history stores, measured
            // +0.45 us each, paper_one_launch_ab.txt)
            RbLanes<M, LPE> rb;
            rb.load(a.comp, e, b.rb_forces, sub);
            rb.finish(b.root, b.dof_state, b.rb_forces, plink, e, pa.rb_out, sub, s.b, s.b + 9 * M::NG, b.dof_props,
                      p.num_envs, owner);
        }
        if (TG_PAPER_T7_END) {   // reward term 7's batch sum, then the rewards / resets / time-outs
            tot = paper_t7_wait_sum(a.pp.t7, pa.t7_count, pa.t7_target, pa.nblk, a.err, c0);
            if (lead && owner) finish_env(p, b, e, tot, tilt, prog, rew);
        }
    }
};

}  // namespace tg
