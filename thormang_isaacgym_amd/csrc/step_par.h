// step_par.h -- tree-parallel, LDS-resident articulation step (included by
// articulation.hip after the shared helpers).  The algorithm of
// oracle/physics_ref.c (Featherstone ABA with a floating base, implicit drives,
// patch-friction PGS contact), evaluated in the ROOT-BODY FRAME: every spatial
// quantity of every group (pose, velocity, inertia, articulated inertia, bias
// force, acceleration, contact Jacobian) is expressed at the root-body origin
// in the root body's coordinates frozen at the start of the substep (an
// inertial frame).  The oracle works in group frames with a spatial transform
// per tree edge; here pass 1 places each group in the root frame once, and the
// backward pass, the forward pass, the Delassus columns and the impulse
// application become transform-free: a child's articulated inertia and bias
// force add into its parent's as they are, and a parent's acceleration is its
// child's before the joint term.  The motion subspace of a group is
// S = (a, P x a) (revolute) or (0, a) (prismatic), a = the group's joint axis
// (its frame's e_z, joint-aligned frames from model/codegen.py), P its origin.
//
// Layout: EPB envs per workgroup, LPE lanes per env (LPE consecutive lanes of
// one wavefront).  Each env's articulated state (per group: pose R,P; v, I^A,
// p^A, U, D^-1, u, q, qd, qds) lives in LDS at lds[env * ES + group * GF +
// field] with 16-byte aligned field blocks.  At 16 envs x 2370 floats the
// Thormang block uses 148 KB of the 160 KB LDS of a CU; 4096 envs = 256
// workgroups = one per CU.
//
// Parallelism inside an env: model/codegen.py list-schedules the non-root
// groups onto the LPE lanes (M::sched[step][lane], parents at earlier steps).
//   pass 1 (root-frame poses, velocities, inertias, bias forces) -- schedule forward
//   pass 2 (articulated inertias)               -- schedule backward; a group
//          gathers its children's contributions (each child leaves its
//          I^a and p^a in its own I^A / p^A slots), so lanes never
//          accumulate into the same address
//   pass 3 (accelerations), impulse application -- forward / backward again
//   Delassus columns                            -- one column per lane, the
//          impulse's up-walk kept in registers (path-restricted: only the
//          ancestors of the contact group and the root->contact-group paths)
//   PGS                                         -- all LPE lanes: W columns and
//          the multipliers in registers, row sums by DPP reduction
//   terrain (HF instantiation)                  -- ground_at: heightfield
//          trimesh height/normal under each shape, rows along that normal
// The root (group 0) quantities that every lane needs (pose, base velocity,
// root LDL factor) are computed redundantly in all lanes of the env.
#pragma once

namespace tg {

#ifdef TG_SECTION_PROF
// developer build only: per-section cycle counts summed over thread 0 of every block
static __device__ unsigned long long tg_prof_acc[24];   // [16..]: sub-sections (see scripts/section_prof.py)
// (round 6: the per-block sums accumulate in LDS and reach the global
// counters once, at the kernel's end -- a global atomic per stamp made every
// block wait on the same address after the synchronised stamps, which
// inflated the section after them, pass 1a of substeps 2 and 3 most)
#define TG_PROF_INIT                                                            \
    __shared__ unsigned long long tg_prof_l[24];                                \
    if (threadIdx.x == 0)                                                       \
        for (int k_ = 0; k_ < 24; ++k_) tg_prof_l[k_] = 0ull;                   \
    unsigned long long tg_t0 = clock64();
#define TG_PROF(k)                                                              \
    {                                                                           \
        const unsigned long long t1 = clock64();                               \
        if (threadIdx.x == 0) tg_prof_l[k] += t1 - tg_t0;                       \
        tg_t0 = t1;                                                             \
    }
#define TG_PROF_FLUSH                                                           \
    if (threadIdx.x == 0)                                                       \
        for (int k_ = 0; k_ < 24; ++k_) atomicAdd(&tg_prof_acc[k_], tg_prof_l[k_]);
#elif defined(TG_STOP_AT)
// developer build only: the kernel ends at the first stamp TG_STOP_AT (every
// wave at the same point), so PMC counters of successive stop points
// attribute LDS bank conflicts to sections (scripts/dev/lds_attrib.sh)
#define TG_PROF_INIT
#define TG_PROF_FLUSH
#define TG_PROF(k)                                                              \
    {                                                                           \
        if ((k) == TG_STOP_AT) return;                                          \
    }
#else
#define TG_PROF_INIT
#define TG_PROF_FLUSH
#define TG_PROF(k)
#endif

// a compile-time int argument (std::integral_constant without <type_traits>,
// which a hipRTC unit, jit.cpp, does not have)
template <int N> struct IntC {
    static constexpr int value = N;
};
// f(IntC<I>), ..., f(IntC<N-1>): a loop whose index is a compile-time constant
template <int I, int N, class F> __device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(IntC<I>{});
        static_for<I + 1, N>(f);
    }
}

#ifdef TG_DUMP_ENV
// developer build (scripts/dev/contact_dump.py): the contact solve of one env
// in the first substep of a launch -- Delassus matrix, free row velocities,
// rows, multipliers -- for a side-by-side with the oracle's (oracle_dump_*)
static __device__ int tg_dump_env = -1, tg_dump_sub = 0;
static __device__ float tg_dump_buf[4096];
#endif

// one env's LDS state
struct LE {
    float *b;
    __device__ __forceinline__ float &operator()(int i) const { return b[i]; }
};

// per-group field offsets (GF floats per group)
// (16-byte aligned blocks: pose [0,12), v [12,18), I^A [20,41), p^A [44,50),
// so the compiler can move them with ds_read/write_b128).  F_RT holds the
// group->root rotation R column-major (= R^T row-major), so the joint axis
// (column 2) and the origin P are the 6 contiguous floats [6,12).
// F_CL: drive-clamp scratch (te, K, effort) between the two solves.
enum : int {
    F_RT = 0, F_AX = 6, F_P = 9, F_V = 12, F_Q = 18, F_QD = 19, F_IA = 20, F_DINV = 41, F_UU = 42, F_QDS = 43,
    F_PA = 44, F_U = 50, F_CL = 56, F_C1 = 59, GF = 60
};

__device__ __forceinline__ V3 ldv3(const LE &s, int o) { return v3(s(o), s(o + 1), s(o + 2)); }
__device__ __forceinline__ void stv3(const LE &s, int o, V3 v) { s(o) = v.x; s(o + 1) = v.y; s(o + 2) = v.z; }
__device__ __forceinline__ SV ldsv(const LE &s, int o) { return SV{ldv3(s, o), ldv3(s, o + 3)}; }
__device__ __forceinline__ void stsv(const LE &s, int o, const SV &v) { stv3(s, o, v.w); stv3(s, o + 3, v.v); }
__device__ __forceinline__ M3 ldm3(const LE &s, int o) {
    M3 m;
#pragma unroll
    for (int k = 0; k < 9; ++k) m.a[k] = s(o + k);
    return m;
}
__device__ __forceinline__ void stm3(const LE &s, int o, const M3 &m) {
#pragma unroll
    for (int k = 0; k < 9; ++k) s(o + k) = m.a[k];
}
__device__ __forceinline__ SI ldsi(const LE &s, int o) {
    SI I;
#pragma unroll
    for (int k = 0; k < 6; ++k) { I.A[k] = s(o + k); I.C[k] = s(o + 15 + k); }
#pragma unroll
    for (int k = 0; k < 9; ++k) I.B[k] = s(o + 6 + k);
    return I;
}
__device__ __forceinline__ void stsi(const LE &s, int o, const SI &I) {
#pragma unroll
    for (int k = 0; k < 6; ++k) { s(o + k) = I.A[k]; s(o + 15 + k) = I.C[k]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) s(o + 6 + k) = I.B[k];
}
// scratch float x of the contact phase, laid over the groups' I^A slots
__device__ __forceinline__ int scr(int x) { return (x / 21) * GF + F_IA + x % 21; }
// group g's pose in the root frame: rotation (group -> root) and origin
__device__ __forceinline__ M3 ldR(const LE &s, int g) { return transpose(ldm3(s, g * GF + F_RT)); }
__device__ __forceinline__ void stR(const LE &s, int g, const M3 &R) { stm3(s, g * GF + F_RT, transpose(R)); }

// round 6: leaf groups' joint-space inertia from their local rigid inertia
// (step_par_kernel d0l); 0 = pass 2b's root-origin form for every group (A/B)
#ifndef TG_LEAF_D0
#define TG_LEAF_D0 1
#endif

// per-group model table in LDS (ints; axis as float bits), built once per block
enum : int { GI_PARENT = 0, GI_DOF = 1, GI_JT = 2, GI_NCH = 3, GI_CH = 4 };

template <class M> struct ParLayout {
    static constexpr int K = M::NROWS;
    static constexpr int GIW = GI_CH + M::MAXC;
    // per-env floats
    static constexpr int W = M::NG * GF;             // K*K Delassus
    static constexpr int ROW = W + K * K;            // K * 8: Jacobian (6) target on
    static constexpr int VFREE = ROW + K * 8;
    static constexpr int LAM = VFREE + K;
    static constexpr int SHP = LAM + K;              // per shape: mu, reff
    static constexpr int CGP = SHP + 2 * M::NSA;     // per contact group: world R (9), p - root origin (3)
    static constexpr int CGV = CGP + 12 * M::NCG;    // per contact group: free velocity (6)
    static constexpr int FLG = CGV + 6 * M::NCG;     // a drive exceeded its effort limit
    // the Gogoro pre-physics values computed in the step kernel (models with
    // the fused Gogoro epilogue): action history (5), command, steering target,
    // rear-wheel velocity target -- in the root group's U / clamp slots, which
    // the root never uses (its articulated inertia is solved by the LDL), so
    // the env stride and with it the LDS bank pattern stay as they were
    static constexpr bool TPON = (M::FUSED & 6) != 0;
    static constexpr int TP = F_U;
    static_assert(F_U + 8 <= GF, "pre-physics values in the root group's slots");
    // per-block ints after the env area
    static constexpr int T_GI = 0;
    static constexpr int T_CPATH = T_GI + M::NG * GIW;                 // [NCG][MAXD]
    // per (schedule step, lane) descriptor, one int4 (see step_desc)
    static constexpr int T_DESC = (T_CPATH + M::NCG * M::MAXD + 3) & ~3;
    static constexpr int T_PACK = T_DESC + 4 * M::NSTEP * M::LPE;     // PackTab words [NPW][LPE]
    static constexpr int T_ZERO = T_PACK + (M::NSTEP + 1) / 2 * M::LPE;  // 32 zero floats (PackTab NPW)
    // GogoroPaper (FUSED bit 4): the envs' reward-term-7 partials
    static constexpr int T_T7 = T_ZERO + 32;
    static constexpr int T_TOTAL = T_T7 + ((M::FUSED & 4) ? M::EPB : 0);
    // SEPC (when the LDS has room): pass 2 writes each group's contribution to
    // its parent (I^a 21 at +0, p^a 6 at +24) and pass 3 its acceleration (+0)
    // into a separate 32-float block, so pass 1's rigid inertias and bias
    // forces survive and the drive-clamp rerun starts at pass 2
    static constexpr int CB = (FLG + 1 + 3) & ~3;
    static constexpr bool SEPC = ((size_t)M::EPB * (CB + 32 * M::NG) + T_TOTAL) * 4 <= 160 * 1024;
    static constexpr int TOTAL0 = SEPC ? CB + 32 * M::NG : FLG + 1;
    // Woodbury drive-clamp update (small trees, one lane per non-root group,
    // impulse application by superposition): instead of re-running passes 2-3
    // with the saturated drives explicit, the first solve is corrected by the
    // unit-torque responses of up to WCM clamped drives.  Per env: G (the
    // responses' joint accelerations per group), R (root accelerations), A
    // (contact-group accelerations), J (row velocities, = J G), Minv
#ifdef TG_NO_SUPER   // developer build: the bottom-up impulse application (A/B)
    static constexpr bool SUPER = false;
#else
    static constexpr bool SUPER = K > 0 && K * (M::MAXD + 6) <= M::NG * 21;
#endif
#ifdef TG_NO_WOOD   // developer build: the drive-clamp rerun instead (A/B)
    static constexpr bool WOOD = false;
#else
    static constexpr bool WOOD = M::NG <= 8 && M::NG - 1 <= M::LPE && (SUPER || K == 0);
#endif
    static constexpr int WCM = 2;
    static constexpr int WB_G = (TOTAL0 + 3) & ~3;          // [WCM][8]
    static constexpr int WB_R = WB_G + WCM * 8;             // [WCM][6]
    static constexpr int WB_A = WB_R + WCM * 6;             // [WCM][NCG][6]
    static constexpr int WB_J = WB_A + WCM * 6 * M::NCG;    // [WCM][K]
    static constexpr int WB_M = WB_J + WCM * (K > 0 ? K : 1);   // [WCM][WCM]
    static constexpr int TOTAL1 = WOOD ? WB_M + WCM * WCM : TOTAL0;
    // superposition scratch past the group slots (humanoid trees with more
    // Delassus columns than groups, the whole-body model): columns NG .. K-1,
    // 21 floats each, when the LDS has room (step_par_kernel swa)
    static constexpr int SWX = (TOTAL1 + 3) & ~3;
    static constexpr bool SWXON = SUPER && K > M::NG && M::NG >= 16 && M::MAXD + 6 <= 21 &&
                                  ((size_t)M::EPB * (SWX + 21 * (K - M::NG) + 4) + T_TOTAL) * 4 <= 160 * 1024;
    static constexpr int TOTAL = SWXON ? SWX + 21 * (K - M::NG) : TOTAL1;
    // env stride.  Large trees (Thormang): 2 mod 4 floats, so the two envs
    // of a 32-lane b32/b64 bank group fall on disjoint bank classes (bank
    // conflicts 27 % -> 17 % of LDS cycles, kernel -0.25 %; the env base is
    // then 8-byte aligned and 16-byte moves become b64 pairs).  The scooters
    // keep 16-byte strides (2 mod 4 measured +1.9 % on 8 lanes per env and
    // +2.5 % / +1.5 % Gogoro / paper on lane pairs; profiles/r3/lds_*, ablations_r3)
#ifdef TG_ES_PAD   // developer experiment: extra floats per env (LDS bank pattern)
    static constexpr int ESPAD = TG_ES_PAD;
#else
    static constexpr int ESPAD = M::NG >= 16 ? 2 : 0;
#endif
    static constexpr int ES = ((TOTAL + 3) & ~3) + ESPAD;
    template <int EPB> static constexpr size_t bytes() { return ((size_t)EPB * ES + T_TOTAL) * 4; }
};

struct GInfo {
    int parent, dof, jt;
};

// the T at a 32-bit byte offset from a uniform base pointer (every per-env
// buffer is far below 4 GiB)
template <class T> __device__ __forceinline__ const T &at_u32(const float *base, unsigned byte_off) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + byte_off);
}

// a table value known to lie in [lo, hi): lets the compiler form LDS / HBM
// offsets from it with 24-bit multiplies instead of v_mad_u64_u32
__device__ __forceinline__ int bounded(int v, int lo, int hi) {
    __builtin_assume(v >= lo && v < hi);
    return v;
}

template <class M> __device__ __forceinline__ GInfo ginfo(const int *gi, int g) {
    const int *p = gi + bounded(g, 0, M::NG) * ParLayout<M>::GIW;
    return GInfo{p[GI_PARENT], p[GI_DOF], p[GI_JT]};
}

// Chain schedule (round 5; TG_CHAIN, the lane-pair trees): one
// schedule slot per root-to-leaf chain of the group tree -- slot s runs, at
// step t, the group at depth t + 1 on the path from the root to its leaf --
// so in every tree pass a group's parent (forward passes) or first child
// (pass 2b) was computed by the same lane one step earlier and its values
// are still in that lane's registers: pass 1a, pass 3 and the impulse
// top-down pass read no parent pose / velocity / acceleration from LDS and
// store none of the last two, and pass 2b gathers from LDS only the children
// after the first (the chains that branch off).  A group shared by several
// chains (the chest, the wrists) is computed by each of their slots in the
// forward passes (identical values) and stored by its OWNER, the slot of its
// first-child chain; pass 2b runs each group on its owner only, which keeps
// the children's summation order (own + child 0 + child 1 + ...), so every
// result is bit-identical to the list schedule's.  Leaves are the slots
// (Thormang: 7 of 8), in depth-first order, children in child-list order.
#ifndef TG_CHAIN
#define TG_CHAIN 1   // developer switch: 0 = the list schedule for every tree (A/B)
#endif
// chain schedule: the forward passes have no LDS dependence between their
// steps, pass 2b only where a group gathers another chain's head; 0 = a
// wave-scope sync only there (and after each pass), 1 = after every step
#ifndef TG_CHAIN_SYNC
#define TG_CHAIN_SYNC 1
#endif
// the passes that use the chain registers (1 pass 1a, 2 pass 2b, 4 pass 3,
// 8 the impulse top-down pass); the others run their list-schedule form over
// the chain schedule (duplicates then load and store like owners: the same
// values).  All four by default, bit-identical to the list schedule
// (scripts/dev/r5_chain_mask.sh, scripts/dev/bitcmp_libs.py, profiles/r5/).
// (The impulse pass stores the joint velocities from every lane of a group,
// owners and duplicates alike: gating that store on ownership changed how the
// compiler contracted the stored sum, and with it the rounding.)
#ifndef TG_CHAIN_MASK
#define TG_CHAIN_MASK 15
#endif
// every lane-pair tree with at least this many groups (the scooters' 6-group
// trees gain too: Gogoro 44.9 -> 43.3 us, GogoroPaper 36.6 -> 35.4 us,
// bit-identical, profiles/r5/scooter_chain_ab.txt; 16 = the humanoids only)
#ifndef TG_CHAIN_MIN_NG
#define TG_CHAIN_MIN_NG 2
#endif

template <class M> struct Chain {
    struct Tab {
        int g[M::NSTEP][M::SL];             // group at (step, slot), -1 idle
        unsigned char own[M::NSTEP][M::SL]; // the slot owns that group
        unsigned char st[M::NG];            // pass 2b stores the group's contribution (its parent is another slot's or the root)
        int nleaf, depth;
    };
    static constexpr Tab make() {
        Tab x{};
        int leaf[M::NG > 0 ? M::NG : 1] = {}, stack[M::NG > 0 ? M::NG : 1] = {};
        int sp = 0, nl = 0;
        stack[sp++] = 0;
        while (sp > 0) {   // depth-first, children in child-list order
            const int g = stack[--sp];
            if (g != 0 && M::nchild[g] == 0) leaf[nl++] = g;
            for (int c = M::nchild[g] - 1; c >= 0; --c) stack[sp++] = M::child[g][c];
        }
        x.nleaf = nl;
        for (int t = 0; t < M::NSTEP; ++t)
            for (int s = 0; s < M::SL; ++s) x.g[t][s] = -1;
        if (nl > M::SL) return x;
        int owner[M::NG > 0 ? M::NG : 1] = {};
        for (int g = 0; g < M::NG; ++g) owner[g] = -1;
        for (int s = 0; s < nl; ++s) owner[leaf[s]] = s;
        for (int g = M::NG - 1; g >= 1; --g)   // parents precede children (topological numbering)
            if (M::nchild[g] > 0) owner[g] = owner[M::child[g][0]];
        for (int s = 0; s < nl; ++s) {
            int path[M::NG > 0 ? M::NG : 1] = {}, n = 0;
            for (int g = leaf[s]; g > 0; g = M::parent[g]) path[n++] = g;
            if (n > x.depth) x.depth = n;
            if (n > M::NSTEP) return x;
            for (int t = 0; t < n; ++t) {
                const int g = path[n - 1 - t];
                x.g[t][s] = g;
                x.own[t][s] = owner[g] == s ? 1 : 0;
            }
        }
        for (int g = 1; g < M::NG; ++g) x.st[g] = (M::parent[g] == 0 || owner[M::parent[g]] != owner[g]) ? 1 : 0;
        return x;
    }
    static constexpr Tab tab = make();
    static constexpr bool ON = TG_CHAIN && M::PAIR && M::NG >= TG_CHAIN_MIN_NG && M::NG <= 128 && tab.nleaf <= M::SL &&
                               tab.depth <= M::NSTEP;
};
// the group (step t, slot) runs (chain: only its owner counts, for the gather widths)
template <class M> constexpr int sched_at(int t, int slot) {
    if constexpr (Chain<M>::ON) return Chain<M>::tab.g[t][slot];
    else return M::sched[t][slot];
}
template <class M> constexpr bool sched_own(int t, int slot) {
    if constexpr (Chain<M>::ON) return Chain<M>::tab.own[t][slot] != 0;
    else return M::sched[t][slot] > 0;
}

// Schedule descriptor of (step t, lane): everything a lane needs about the
// group it handles, in one ds_read_b128 (prefetched a step ahead):
//   x = group (0: idle), y = parent, z = dof | jt << 16 | own << 24 | st << 25
//   (chain schedule: the lane owns the group; pass 2b stores its contribution),
//   w = nch | smax << 4 | child_c << (8 + 8c)  (smax: the step's max nch over lanes)
struct alignas(16) I4 {
    int x, y, z, w;
};
template <class M> constexpr I4 step_desc(int t, int lane) {
    // lane pairs (M::PAIR): lanes sub and sub + SL run schedule slot sub
    const int slot = lane % M::SL;
    const int g = (lane < M::SL || M::PAIR) ? sched_at<M>(t, slot) : -1;
    if (g <= 0) return I4{0, 0, 0, 0};
    int smax = 0;
    for (int l = 0; l < M::SL; ++l)
        if (sched_own<M>(t, l) && M::nchild[sched_at<M>(t, l)] > smax) smax = M::nchild[sched_at<M>(t, l)];
    int w = M::nchild[g] | smax << 4;
    for (int c = 0; c < M::nchild[g]; ++c) w |= M::child[g][c] << (8 + 8 * c);
    int z = M::gdof[g] | M::jtype[g] << 16;
    if constexpr (Chain<M>::ON) z |= (sched_own<M>(t, slot) ? 1 : 0) << 24 | Chain<M>::tab.st[g] << 25;
    return I4{g, M::parent[g], z, w};
}
// the largest child count among schedule step t's groups (the gather width
// of pass 2b at that step, a compile-time constant)
template <class M> constexpr int step_smax(int t) {
    int m = 0;
    for (int l = 0; l < M::SL; ++l)
        if (sched_own<M>(t, l) && M::nchild[sched_at<M>(t, l)] > m) m = M::nchild[sched_at<M>(t, l)];
    return m;
}
// pass 2b's step t gathers from LDS under the chain schedule (a group with
// children after its first)
template <class M> constexpr bool step_gathers(int t) { return step_smax<M>(t) >= 2; }
template <class M> constexpr int max_nonroot_children() {
    int m = 0;
    for (int g = 1; g < M::NG; ++g) m = M::nchild[g] > m ? M::nchild[g] : m;
    return m;
}
template <class M> struct DescTab {
    static_assert(max_nonroot_children<M>() <= 3 && M::NG <= 255, "descriptor packs 3 children of 8 bits");
    struct Arr {
        I4 d[M::NSTEP * M::LPE];
    };
    static constexpr Arr make() {
        Arr a{};
        for (int i = 0; i < M::NSTEP * M::LPE; ++i) a.d[i] = step_desc<M>(i / M::LPE, i % M::LPE);
        return a;
    }
    static constexpr Arr tab = make();
};
// The tree passes' (group, parent, joint type) of every schedule step of a
// lane, packed 16 bits per step (g | jt == prismatic << 7 | parent << 8), two
// steps per 32-bit word, held in registers for the whole launch: the forward
// passes form their next step's LDS / HBM addresses with one bit-field
// extract instead of a descriptor read from LDS, which sat behind the
// previous step's stores in the in-order LDS queue (NG <= 128)
template <class M> struct PackTab {
    static constexpr bool ON = M::NG <= 128;
    static constexpr int NPW = (M::NSTEP + 1) / 2;
    struct Arr {
        int v[NPW * M::LPE];
    };
    static constexpr Arr make() {
        Arr a{};
        for (int w = 0; w < NPW; ++w)
            for (int lane = 0; lane < M::LPE; ++lane) {
                int x = 0;
                for (int k = 0; k < 2; ++k) {
                    const int t = 2 * w + k;
                    if (t >= M::NSTEP) break;
                    const I4 d = step_desc<M>(t, lane);
                    const int jp = ((d.z >> 16) & 255) == TG_JOINT_PRISMATIC ? 1 : 0;
                    // (chain schedule: bit 15 the owner flag, the parent in bits 8-14)
                    const int py = Chain<M>::ON ? ((d.y & 127) | ((d.z >> 24) & 1) << 7) : (d.y & 255);
                    x |= ((d.x & 127) | jp << 7 | py << 8) << (16 * k);
                }
                a.v[w * M::LPE + lane] = x;
            }
        return a;
    }
    static constexpr Arr tab = make();
};
__device__ __forceinline__ int d_dof(const I4 &d) { return d.z & 0xFFFF; }
__device__ __forceinline__ int d_jt(const I4 &d) { return (d.z >> 16) & 255; }
__device__ __forceinline__ bool d_own(const I4 &d) { return (d.z >> 24) & 1; }
__device__ __forceinline__ bool d_store(const I4 &d) { return (d.z >> 25) & 1; }
__device__ __forceinline__ int d_nch(const I4 &d) { return d.w & 15; }
__device__ __forceinline__ int d_smax(const I4 &d) { return (d.w >> 4) & 15; }
__device__ __forceinline__ int d_child(const I4 &d, int c) { return (d.w >> (8 + 8 * c)) & 255; }

// motion subspace of a joint in the root frame from its axis a and origin P:
// (a, P x a) for a revolute joint, (0, a) for a prismatic one
__device__ __forceinline__ SV motion_S(int jt, V3 ax, V3 P) {
    const bool rev = jt == TG_JOINT_REVOLUTE;
    const V3 pa = cross(P, ax);
    return SV{rev ? ax : v3(0, 0, 0), rev ? pa : ax};
}
__device__ __forceinline__ SV ldS(const LE &s, int g, int jt) {
    return motion_S(jt, ldv3(s, g * GF + F_AX), ldv3(s, g * GF + F_P));
}
// models whose every joint group is revolute (Thormang, the scooters: their
// prismatic joints are locked seat joints inside the root group): the joint
// type drops out of every pass -- no per-lane select or branch on it
template <class M> constexpr bool all_revolute() {
    for (int g = 1; g < M::NG; ++g)
        if (M::jtype[g] != TG_JOINT_REVOLUTE) return false;
    return true;
}
template <class M> __device__ __forceinline__ SV motion_Sm(int jt, V3 ax, V3 P) {
    if constexpr (all_revolute<M>()) return SV{ax, cross(P, ax)};
    else return motion_S(jt, ax, P);
}
template <class M> __device__ __forceinline__ SV ldSm(const LE &s, int g, int jt) {
    return motion_Sm<M>(jt, ldv3(s, g * GF + F_AX), ldv3(s, g * GF + F_P));
}
// Contact quantities at the contact group's own origin (round 6).  The passes
// carry spatial vectors about the ROOT origin; a contact group far from it (a
// scooter wheel 0.8 m away, a humanoid foot 0.9 m below the pelvis) then has
// a linear velocity dominated by its joint's qd (P x a) term, which the
// contact point's r x w cancels again when a row velocity is formed -- the
// fp32 digits lost there made the kernel's Delassus matrix and free row
// velocities 4-6x less accurate than the fp32 oracle's, which works in group
// frames (profiles/r6/gogoro_dump_stats*.txt).  So the rows' Jacobians are
// (r_l x d, d) with r_l the point about the contact group's origin pc, and the
// velocities they meet are formed at pc term by term: the root's shifted by
// w0 x pc, each path joint's as qd (a, a x (pc - P)) -- a wheel's own spin
// adds nothing to its centre's velocity, exactly.
// (w, v) about the root origin -> (w, v + w x pc)
__device__ __forceinline__ SV shift_to(const SV &x, V3 pc) { return SV{x.w, x.v + cross(x.w, pc)}; }
// a joint's motion subspace about pc (its axis a through P): (a, a x (pc - P))
// revolute, (0, a) prismatic
template <class M> __device__ __forceinline__ SV motion_at(int jt, V3 ax, V3 P, V3 pc) {
    if constexpr (all_revolute<M>()) return SV{ax, cross(ax, pc - P)};
    else return jt == TG_JOINT_REVOLUTE ? SV{ax, cross(ax, pc - P)} : SV{v3(0, 0, 0), ax};
}

// The LPE lanes of an env are consecutive lanes of one wavefront, whose LDS
// operations execute in program order: an env-level "barrier" only has to stop
// the compiler from moving LDS accesses across it (no s_barrier, and no
// s_waitcnt on the prefetched global loads still in flight).
// sum over the 8 lanes of an env with DPP moves (row half-mirror, then quad
// swaps): every lane ends with the total, no LDS round trip
// (every lane of the permutations used here has a valid source, so the old
// operand is dead: mov_dpp with bound_ctrl needs no zero-initialised
// destination and lets the compiler fold the move into the add; round 5,
// 103 moves fewer in the walk kernel, bit-identical, profiles/r5/dpp_ab.txt)
template <int CTRL> __device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float sum8(float v) {
    v += dpp<0x141>(v);   // row_half_mirror: lane i <-> 7 - i
    v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
    return v;
}
// over the 16 lanes of a DPP row: the two 8-lane halves, then row_ror:8
__device__ __forceinline__ float sum16(float v) {
    v = sum8(v);
    return v + dpp<0x128>(v);
}
template <int L> __device__ __forceinline__ float sum_lanes(float v) {
    static_assert(L == 8 || L == 16, "env lanes: 8 or 16");
    if constexpr (L == 8) return sum8(v);
    else return sum16(v);
}
// lane n of the env's LPE lanes, on every lane of the env: DPP row_newbcast
// (lane n of each 16-lane row to the whole row); an 8-lane env takes its
// half's lane
template <int L> __device__ __forceinline__ float env_bcast(float v, int n, int sub) {
    static_assert(L == 8 || L == 16, "env lanes: 8 or 16");
    auto bc = [&](int m) {
        switch (m) {
        case 0: return dpp<0x150>(v); case 1: return dpp<0x151>(v); case 2: return dpp<0x152>(v);
        case 3: return dpp<0x153>(v); case 4: return dpp<0x154>(v); case 5: return dpp<0x155>(v);
        case 6: return dpp<0x156>(v); case 7: return dpp<0x157>(v); case 8: return dpp<0x158>(v);
        case 9: return dpp<0x159>(v); case 10: return dpp<0x15A>(v); case 11: return dpp<0x15B>(v);
        case 12: return dpp<0x15C>(v); case 13: return dpp<0x15D>(v); case 14: return dpp<0x15E>(v);
        default: return dpp<0x15F>(v);
        }
    };
    if constexpr (L == 16) return bc(n);
    else return (threadIdx.x & 8) ? bc(n + 8) : bc(n);
}
// the partner lane's value (lane pairs sub, sub + 8 of a 16-lane row)
__device__ __forceinline__ float pair_swap(float v) { return dpp<0x128>(v); }

// a contact row without response: its Delassus diagonal at most this (real
// rows have 1e-3 .. 1e1, inverse effective masses; this only catches the
// rounding residue of an exact 0)
#define TG_W_DEAD 1e-9f
// (the 8-lane PGS's inverse diagonal: 0 for such a row, no impulse)
__device__ __forceinline__ float inv_diag(float w) { return w > TG_W_DEAD ? 1.0f / w : 0.f; }

#define TG_SYNC()                                          \
    do {                                                   \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                   \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)

// Ground surface under world (x, y): the heightfield trimesh of
// tg_set_heightfield (vertex (i,j) at (ox + i hs, oy + j hs, vs h[i][j]);
// cell triangles (i,j)-(i+1,j+1)-(i,j+1) for fv >= fu and
// (i,j)-(i+1,j)-(i+1,j+1) for fu >= fv) or the z = 0 plane, whichever is
// higher.  Returns the height, the unit normal in n and whether the terrain
// is the surface.  oracle/physics_ref.c ground_at is the same function.
__device__ __forceinline__ float ground_at(const StepArgs &a, float x, float y, V3 &n, bool &on_hf) {
    n = v3(0, 0, 1);
    on_hf = false;
    const float u = (x - a.hf_ox) / a.hf_hs, v = (y - a.hf_oy) / a.hf_hs;
    if (!(u >= 0.f && v >= 0.f && u <= (float)(a.hf_rows - 1) && v <= (float)(a.hf_cols - 1))) return 0.f;
    const int i = min((int)u, a.hf_rows - 2), j = min((int)v, a.hf_cols - 2);
    const float fu = u - (float)i, fv = v - (float)j;
    const float *r0 = a.hf + (size_t)i * a.hf_cols + j, *r1 = r0 + a.hf_cols;
    const float h00 = a.hf_vs * r0[0], h01 = a.hf_vs * r0[1], h10 = a.hf_vs * r1[0], h11 = a.hf_vs * r1[1];
    float H, gx, gy;
    if (fu >= fv) { gx = h10 - h00; gy = h11 - h10; H = h00 + fu * gx + fv * gy; }
    else          { gx = h11 - h01; gy = h01 - h00; H = h00 + fu * gx + fv * gy; }
    if (!(H > 0.f)) return 0.f;
    gx /= a.hf_hs;
    gy /= a.hf_hs;
    const float inv = 1.f / sqrtf(gx * gx + gy * gy + 1.f);
    n = v3(-gx * inv, -gy * inv, inv);
    on_hf = true;
    return H;
}

// Optional fused epilogue P: a task's post-physics step run by the step
// kernel on the final state (still in registers / LDS) instead of a separate
// launch that re-reads it; P::epilogue then also stores the state.  NoPost:
// plain store.
struct NoPost {
    struct Args {};
    static constexpr bool on = false;
    static constexpr int NPRE = 0;   // floats per lane an epilogue prefetches at kernel start
    static constexpr bool PM_OUT = false;   // the epilogue stores the walk pre-physics outputs itself
    static constexpr bool TOUCH = false;    // touch_addr: a line of the epilogue's inputs per lane (below)
    static constexpr bool T7_SYNC = false;  // publishes the term-7 block sum for an in-launch batch sum (PaperPost)
};

// inverse of the group -> dof map: group of dof d, -1 for a locked dof
template <class M> struct DofGroup {
    struct Arr {
        int g[M::ND > 0 ? M::ND : 1];
    };
    static constexpr Arr make() {
        Arr x{};
        for (int d = 0; d < M::ND; ++d) x.g[d] = -1;
        for (int g = 1; g < M::NG; ++g) x.g[M::gdof[g]] = g;
        return x;
    }
    static constexpr Arr tab = make();
};
// dof of group g in [1, NG) (lane-dependent g): g + OFF when the model
// numbers them that way, else a select chain over the model's table
template <class M> constexpr int group_dof_offset() {
    const int off = M::NG > 1 ? M::gdof[1] - 1 : 0;
    for (int g = 1; g < M::NG; ++g)
        if (M::gdof[g] != g + off) return -1000;
    return off;
}
template <class M> __device__ __forceinline__ int group_dof(int g) {
    constexpr int off = group_dof_offset<M>();
    if constexpr (off != -1000) {
        return g + off;
    } else {
        int d = M::gdof[M::NG > 1 ? 1 : 0];
#pragma unroll
        for (int k = 2; k < M::NG; ++k) d = g == k ? M::gdof[k] : d;
        return d;
    }
}
// group of dof d (lane-dependent d): d + OFF when the model numbers its
// groups that way (an add, no table load), else the table
template <class M> constexpr int dof_group_offset() {
    constexpr auto t = DofGroup<M>::make();
    const int off = M::ND > 0 ? t.g[0] - 0 : 0;
    for (int d = 0; d < M::ND; ++d)
        if (t.g[d] != d + off) return -1000;
    return off;
}
template <class M> __device__ __forceinline__ int dof_group(int d) {
    constexpr int off = dof_group_offset<M>();
    if constexpr (off != -1000) return d + off;
    else return DofGroup<M>::tab.g[d];
}

// TG_ALIAS_DEV (developer timing experiment, wrong results): the lane-pair
// trees' envs share TG_ALIAS_DEV LDS slots and the kernel is compiled for two
// waves per SIMD, so two workgroups fit a CU -- what a per-env LDS footprint
// half the size would buy
// TG_GHOST_DEV (developer timing prototype, VERDICT r4 item 1, results
// exact): the lane-pair trees run two envs per wavefront instead of four --
// lanes 0-31 two real envs, lanes 32-63 their "ghost" twins, which compute
// the same env on the same LDS slot and never store -- so 4096 envs are 2048
// waves, and with half the LDS slots per workgroup and the kernel compiled
// for two waves per SIMD two workgroups share a CU: two waves per SIMD, each
// carrying the whole per-env chain for half the envs.  What a second wave
// per SIMD buys when the env's work is NOT split across more lanes (the
// 32-lane design's lower end)
#if defined(TG_ALIAS_DEV)
template <class M> constexpr int alias_slots(int epb) { return M::PAIR && TG_ALIAS_DEV < epb ? TG_ALIAS_DEV : epb; }
#define TG_STEP_BOUNDS(M, EPB) __launch_bounds__(EPB * M::LPE, M::PAIR ? 2 : 1)
#elif defined(TG_GHOST_DEV)
template <class M> constexpr int alias_slots(int epb) { return (M::PAIR && M::NG >= 16) ? epb / 2 : epb; }
#define TG_STEP_BOUNDS(M, EPB) __launch_bounds__(EPB * M::LPE, (M::PAIR && M::NG >= 16) ? 2 : 1)
#else
template <class M> constexpr int alias_slots(int epb) { return epb; }
#define TG_STEP_BOUNDS(M, EPB) __launch_bounds__(EPB * M::LPE)
#endif
template <class M, int EPB, bool HF, class P = NoPost>
__global__ TG_STEP_BOUNDS(M, EPB) void step_par_kernel(StepArgs a, typename P::Args pa) {
    constexpr int LPE = M::LPE;
    static_assert(64 % LPE == 0, "an env's lanes must share a wavefront");
    using CL = CompLayout<M>;
    using PL = ParLayout<M>;
    constexpr int K = PL::K;
    constexpr int GIW = PL::GIW;
    // Impulse application by superposition: each Delassus column j leaves its
    // up-walk joint impulses du_j (path order) and root response a_j in the
    // I^A slots (dead between pass 2's root solve and the next substep), and
    // the application becomes u_g = sum_j lam_j du_j, da0 = sum_j lam_j a_j,
    // then the top-down pass.  Models whose columns do not fit keep the
    // bottom-up pass.
    constexpr int SW = M::MAXD + 6;
    // column j's superposition scratch (its up-walk impulses, then its root
    // response), element x: one dead I^A slot per column when every column
    // has its own group slot -- the address is then affine in x, one base
    // register plus an immediate per element (round 6: the packed form's
    // (jSW+x)/21 per element made the apply loop hoist a register per row,
    // the whole-body model's spills); else packed across the slots.  Humanoid
    // trees only: A/B (profiles/r6/sw_slot_ab.txt) walk 49.25 -> 48.4 us, AGPRs
    // 59 -> 39; Gogoro 43.1 -> 43.8 us, so the scooters keep the packed form
    constexpr bool SW_SLOT = (K <= M::NG || PL::SWXON) && SW <= 21 && M::NG >= 16;
    auto swa = [](int j, int x) {
        return SW_SLOT ? (j < M::NG ? j * GF + F_IA + x : PL::SWX + 21 * (j - M::NG) + x) : scr(j * SW + x);
    };
#ifdef TG_NO_SUPER
    constexpr bool SUPER = false;
#else
    constexpr bool SUPER = K > 0 && K * SW <= M::NG * 21;
#endif
    constexpr bool SEPC = PL::SEPC;
    auto ia_c = [](int g) { return SEPC ? PL::CB + 32 * g : g * GF + F_IA; };        // pass-2 contribution I^a
    auto pa_c = [](int g) { return SEPC ? PL::CB + 32 * g + 24 : g * GF + F_PA; };   // pass-2 contribution p^a
    auto ac_s = [](int g) { return SEPC ? PL::CB + 32 * g : g * GF + F_PA; };        // pass-3 acceleration
    extern __shared__ __attribute__((aligned(16))) float lds_raw[];
    int *tab = reinterpret_cast<int *>(lds_raw + alias_slots<M>(EPB) * PL::ES);
    const int *gi = tab + PL::T_GI;
    const I4 *desc = reinterpret_cast<const I4 *>(tab + PL::T_DESC);   // [NSTEP][LPE]
    const float *zeros = reinterpret_cast<const float *>(tab + PL::T_ZERO);
    const int *cpath = tab + PL::T_CPATH;
    const int tid = threadIdx.x;
    const int le = tid / LPE, sub = tid % LPE;
    auto dsc = [&](int t) {
        I4 d = desc[t * LPE + sub];
        d.x = bounded(d.x, 0, M::NG);
        d.y = bounded(d.y, 0, M::NG);
        return d;
    };
    // XCD-aware chunk order: workgroups are dispatched round-robin over the 8
    // XCDs, so workgroup b takes env chunk (b % 8) * (nb / 8) + b / 8 and each
    // XCD's L2 sees a contiguous env range (the [KC][N] composite cache rows
    // of neighbouring chunks share 128-B lines)
    const int nb = gridDim.x;
    const int chunk = (nb % 8 == 0) ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
#ifdef TG_GHOST_DEV
    // (lanes 32-63 of a wave: the ghost twins of lanes 0-31's envs)
    constexpr bool GH = M::PAIR && LPE == 16 && M::NG >= 16;
    constexpr int EPR = GH ? EPB / 2 : EPB;   // real envs per workgroup
    const int lr = GH ? (le >> 2) * 2 + (le & 1) : le;
    const int e = min(chunk * EPR + lr, a.N - 1);
    const bool owner = (!GH || (le & 3) < 2) && chunk * EPR + lr < a.N;
#else
    const int lr = le;
    const int e = min(chunk * EPB + le, a.N - 1);   // tail lanes redo the last env, never store
    const bool owner = chunk * EPB + le < a.N;
#endif
    TG_PROF_INIT

    // the per-block tables, copied from the model's constants.  When every
    // table fits one entry per thread (every compiled model), all the loads are
    // issued before the first LDS store: one memory round trip instead of one
    // per table (the stores would otherwise pin each table's loads behind the
    // previous one's)
    // the env's state (root, joint positions and velocities), loaded early
    // for one-round trees (EARLY) or, for the larger trees with an affine
    // group -> dof map, inside the table fill (OVL, round 4: its round trip
    // overlaps the table's; ThormangWalk -0.3 us, three A/B rounds,
    // profiles/r4/state_overlap_ab.txt)
#ifndef TG_STATE_OVERLAP
#define TG_STATE_OVERLAP 1   // developer switch: 0 = the state loads after the table barrier (A/B)
#endif
#ifndef TG_EARLY_STATE
#define TG_EARLY_STATE 0   // developer switch: 1 = every tree with an affine group -> dof map
#endif
    constexpr int NGR = (M::NG - 1 + LPE - 1) / LPE;
    // one-round trees: the env's state issued before the barrier (group ->
    // dof from the model's constants, not the LDS table) so its latency
    // overlaps the table fill's (larger trees: measured no gain, more live
    // registers across the barrier)
    constexpr bool EARLY = NGR == 1 || (TG_EARLY_STATE && group_dof_offset<M>() != -1000);
    float q0[NGR > 0 ? NGR : 1], qd0[NGR > 0 ? NGR : 1], rt0[13];
    const float *st_root = a.root + (size_t)e * 13;
    const float *st_dofs = a.dof + (size_t)e * a.D * 2;
    constexpr int NT = EPB * M::LPE;
    constexpr bool ONE = M::NG <= NT && M::NSTEP * LPE <= NT && PackTab<M>::NPW * LPE <= NT &&
                         M::NCG * M::MAXD <= NT && 32 <= NT;
    // (inside the one-pass table fill only: the whole-body model's 8-env
    // workgroups fill the table in loops and load the state after the barrier)
    constexpr bool OVL = TG_STATE_OVERLAP && ONE && !EARLY && group_dof_offset<M>() != -1000;
    if constexpr (ONE) {
        const int ig = tid < M::NG ? tid : 0, idd = tid < M::NSTEP * LPE ? tid : 0,
                  ipk = tid < PackTab<M>::NPW * LPE ? tid : 0, icp = tid < M::NCG * M::MAXD ? tid : 0;
        int gv[GIW];
        gv[GI_PARENT] = M::parent[ig];
        gv[GI_DOF] = M::gdof[ig];
        gv[GI_JT] = M::jtype[ig];
        gv[GI_NCH] = M::nchild[ig];
#pragma unroll
        for (int c = 0; c < M::MAXC; ++c) gv[GI_CH + c] = M::child[ig][c];
        const I4 dv = DescTab<M>::tab.d[idd];
        const int pv = PackTab<M>::tab.v[ipk];
        const int cv = M::cpath[icp / M::MAXD][icp % M::MAXD];
        if constexpr (OVL) {
            // the env's state issued here, between the table loads and their
            // stores: its memory round trip overlaps the table's instead of
            // following the barrier (the group -> dof map from the model's
            // constants)
#pragma unroll
            for (int r = 0; r < NGR; ++r) {
                const int d = group_dof<M>(min(1 + sub + r * LPE, M::NG - 1));
                q0[r] = st_dofs[2 * d];
                qd0[r] = st_dofs[2 * d + 1];
            }
#pragma unroll
            for (int k = 0; k < 13; ++k) rt0[k] = st_root[k];
        }
        if (tid < M::NG) {
#pragma unroll
            for (int k = 0; k < GIW; ++k) tab[PL::T_GI + tid * GIW + k] = gv[k];
        }
        if (tid < M::NSTEP * LPE) {
            int *p = tab + PL::T_DESC + 4 * tid;
            p[0] = dv.x; p[1] = dv.y; p[2] = dv.z; p[3] = dv.w;
        }
        if (tid < PackTab<M>::NPW * LPE) tab[PL::T_PACK + tid] = pv;
        if (tid < 32) tab[PL::T_ZERO + tid] = 0;
        if (tid < M::NCG * M::MAXD) tab[PL::T_CPATH + tid] = cv;
    } else {
    for (int i = tid; i < M::NG; i += EPB * LPE) {
        int *p = tab + PL::T_GI + i * GIW;
        p[GI_PARENT] = M::parent[i];
        p[GI_DOF] = M::gdof[i];
        p[GI_JT] = M::jtype[i];
        p[GI_NCH] = M::nchild[i];
        for (int c = 0; c < M::MAXC; ++c) p[GI_CH + c] = M::child[i][c];
    }
    for (int i = tid; i < M::NSTEP * LPE; i += EPB * LPE) {
        const I4 d = DescTab<M>::tab.d[i];
        int *p = tab + PL::T_DESC + 4 * i;
        p[0] = d.x; p[1] = d.y; p[2] = d.z; p[3] = d.w;
    }
    for (int i = tid; i < PackTab<M>::NPW * LPE; i += EPB * LPE) tab[PL::T_PACK + i] = PackTab<M>::tab.v[i];
    for (int i = tid; i < 32; i += EPB * LPE) tab[PL::T_ZERO + i] = 0;
    for (int i = tid; i < M::NCG * M::MAXD; i += EPB * LPE) tab[PL::T_CPATH + i] = M::cpath[i / M::MAXD][i % M::MAXD];
    }
    const LE s{lds_raw + (lr % alias_slots<M>(EPB)) * PL::ES};
    const size_t N = a.N;
    const int D = a.D;
    const float h = a.h;
    const bool fix_base = a.fix_base != 0;
    const float *comp = a.comp;
#ifdef TG_EXP_HOT   // developer experiment: every env reads env (e % 64)'s inputs (cache-resident)
    const int ein = e % 64;
#else
    // every env reads env 0's composite block while all blocks are equal
    // (a.cuni, uniform_check_kernel): one shared, cache-resident copy.  The
    // composites change only through a compose, which re-runs the check; the
    // DOF property rows are read per env always, so a write through the
    // zero-copy dof_props view takes effect at the next step as it does
    // without the shared cache
    const int ein = (a.cuni && *a.cuni) ? 0 : e;
#endif
    // per-env inputs through 32-bit element offsets from the uniform base
    // pointers (scalar base + vector offset addressing, no 64-bit address math)
    const unsigned cbase = (unsigned)ein * M::KC;
    // (byte offsets formed in 32 bits: the loads take the scalar-base +
    // 32-bit vector-offset form, no 64-bit address arithmetic per load)
    auto CP = [&](int k) { return at_u32<float>(comp, (cbase + (unsigned)k) * 4u); };
    auto CP4 = [&](int k) { return at_u32<float4>(comp, (cbase + (unsigned)k) * 4u); };
    const unsigned ND = (unsigned)N * (unsigned)D, pbase = (unsigned)e * (unsigned)D;
    auto PR = [&](int f, int d) { return at_u32<float>(a.props, ((unsigned)f * ND + pbase + (unsigned)d) * 4u); };
    const bool lead = sub == 0;

    // the Gogoro pre-physics (tg_gogoro_step) on the env's lead lane, first of
    // all so its input latency overlaps the state loads
    if constexpr (PL::TPON) {
        if ((M::FUSED & 2) && a.gp_in_step && lead) {   // the Gogoro pre-physics (tg_gogoro_step) on the env's lead lane
            float ah[5], cmd, ts, vr;
            gogoro_pre_values(a.gp, e, ah, cmd, ts, vr);
#pragma unroll
            for (int k = 0; k < 5; ++k) s(PL::TP + k) = ah[k];
            s(PL::TP + 5) = cmd;
            s(PL::TP + 6) = ts;
            s(PL::TP + 7) = vr;
            if (owner) gogoro_pre_store(a.gp, e, a.D, ah, cmd, ts, vr);
        }
        if ((M::FUSED & 4) && a.pp_in_step && lead) {   // the GogoroPaper pre-physics (tg_paper_step), as paper_pre_prologue
            const PaperPre &pp = a.pp;
            constexpr int PC = TG_PAPER_CMD_HIST;
            float *hh = pp.command_history + PC * (size_t)e;
            const float act = pp.actions[e];
            const float ac = act < -1.0f ? -1.0f : (act > 1.0f ? 1.0f : act);
            const float cmd = ac * pp.max_steering;
            float hv[PC];
#pragma unroll
            for (int k = 0; k < PC - 1; ++k) hv[k] = hh[k + 1];
            hv[PC - 1] = cmd;
            const int64_t delay = pp.use_steer_delay ? pp.steer_delay[e] : 0;
            const float speed = pp.curent_speed[e];
            int idx = PC - 3;
            if (pp.use_steer_delay) idx = delay == 0 ? 0 : (int)(PC - delay);   // command_history[:, -steer_delay]
            float steer = 0.f;
#pragma unroll
            for (int k = 0; k < PC; ++k) steer = k == idx ? hv[k] : steer;
            s(PL::TP + 6) = steer;
            s(PL::TP + 7) = speed;
            if (owner) {
#pragma unroll
                for (int k = 0; k < PC; ++k) hh[k] = hv[k];
                pp.curent_command[e] = cmd;
            }
            if (pp.t7) {   // the env's partial into the workgroup's slots, summed after the barrier
                static_assert(EPB == TG_PAPER_T7_BLK, "a term-7 block is one workgroup");
                reinterpret_cast<float *>(tab + PL::T_T7)[le] = owner ? paper_t7_partial(pp, e, cmd) : 0.0f;
            }
        }
    }
    // the walk pre-physics (tg_walk_step): the env's clamped actions and drive
    // targets written once, lane = dof mod LPE; pass 2a reads the targets back
    // like pos_tgt (the barrier below orders them within the workgroup)
    // (an epilogue that stores them itself, WalkPost, skips this: its
    // targets come from the actions where pass 2a loads them, and the kernel
    // start then waits on no store)
    if (!P::PM_OUT && a.pm_in_step && owner) {
        for (int d = sub; d < D; d += LPE) {
            const unsigned ed = (unsigned)e * (unsigned)D + (unsigned)d;
            const float c = pm_clamp(a, a.pm_actions[ed]);
            a.pm_act_out[ed] = c;
            a.pm_tgt_out[ed] = pm_target(a, d, c);
        }
    }
    float *root = a.root + (size_t)e * 13;
    float *dofs = a.dof + (size_t)e * D * 2;
    if constexpr (EARLY) {
#pragma unroll
        for (int r = 0; r < NGR; ++r) {
            const int g = 1 + sub + r * LPE;
            q0[r] = qd0[r] = 0.f;
            if (g < M::NG) {
                const int d = group_dof<M>(g);
                q0[r] = dofs[2 * d];
                qd0[r] = dofs[2 * d + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < 13; ++k) rt0[k] = root[k];
    }
    __syncthreads();   // group tables (shared by both wavefronts)
    constexpr int NPW = PackTab<M>::NPW;
    int pkw[NPW];
#pragma unroll
    for (int w = 0; w < NPW; ++w) pkw[w] = tab[PL::T_PACK + w * LPE + sub];
    // step t's (group, parent, joint type) from the packed words (descriptor
    // fields x, y and z's joint type), or the LDS descriptor for NG > 128
#ifndef TG_PACK_MASK
#define TG_PACK_MASK 15   // passes using the packed words: 1 pass 1a, 2 pass 2b, 4 pass 3, 8 impulse top-down
#endif
    auto pdsc_on = [&](int t, auto PASS) {
        if constexpr (PackTab<M>::ON && (TG_PACK_MASK & decltype(PASS)::value)) {
            // (laundered through an empty volatile asm, which stays between the
            // wave barriers around it: the loads this step's fields address are
            // then issued where the pass issues them, a step or two ahead, not
            // hoisted to the start of the pass with all their registers live)
            int wv = pkw[t / 2];
            __asm__ volatile("" : "+v"(wv));
            const int v = (wv >> (16 * (t % 2))) & 0xFFFF;
            const int jz = ((v >> 7) & 1 ? TG_JOINT_PRISMATIC : TG_JOINT_REVOLUTE) << 16;
            if constexpr (Chain<M>::ON)   // (bit 15: the lane owns the group)
                return I4{bounded(v & 127, 0, M::NG), bounded((v >> 8) & 127, 0, M::NG), jz | ((v >> 15) & 1) << 24, 0};
            else
                return I4{bounded(v & 127, 0, M::NG), bounded(v >> 8, 0, M::NG), jz, 0};
        } else {
            return dsc(t);
        }
    };
    auto pdsc = [&](int t) { return pdsc_on(t, IntC<1>{}); };
    auto pdsc2 = [&](int t) { return pdsc_on(t, IntC<2>{}); };
    auto pdsc3 = [&](int t) { return pdsc_on(t, IntC<4>{}); };
    auto pdsc4 = [&](int t) { return pdsc_on(t, IntC<8>{}); };
    if constexpr ((M::FUSED & 4) != 0) {
        if (a.pp_in_step && a.pp.t7 && tid == 0) {
            if constexpr (P::T7_SYNC)
                paper_t7_block<true>(a.pp, reinterpret_cast<const float *>(tab + PL::T_T7), chunk, pa.t7_count);
            else
                paper_t7_block(a.pp, reinterpret_cast<const float *>(tab + PL::T_T7), chunk);
        }
    }
    if constexpr (!EARLY && !OVL) {
#pragma unroll
        for (int k = 0; k < 13; ++k) rt0[k] = root[k];
    }
    if constexpr (PL::TPON) {
        if ((M::FUSED & 4) && a.pp_in_step && owner) {   // the paper's drive target rows: steering and rear wheel, 0 elsewhere
            float *pt = a.pp.pos_target + (size_t)D * e, *vt = a.pp.vel_target + (size_t)D * e;
            for (int d = sub; d < D; d += LPE) {
                pt[d] = d == a.pp.dof_steer ? s(PL::TP + 6) : 0.0f;
                vt[d] = d == a.pp.dof_rear ? s(PL::TP + 7) : 0.0f;
            }
        }
    }
    if constexpr (EARLY || OVL) {
#pragma unroll
        for (int r = 0; r < NGR; ++r) {
            const int g = 1 + sub + r * LPE;
            if (g < M::NG) {
                s(g * GF + F_Q) = q0[r];
                s(g * GF + F_QD) = qd0[r];
            }
        }
    } else {
        // every round's dof index, then every load, then the stores: one
        // memory round trip (a store between them would pin the next round's
        // loads behind it)
        int dix[NGR > 0 ? NGR : 1];
        float qv[NGR > 0 ? NGR : 1], qdv[NGR > 0 ? NGR : 1];
#pragma unroll
        for (int r = 0; r < NGR; ++r) {
            const int g = min(1 + sub + r * LPE, M::NG - 1);
            if constexpr (group_dof_offset<M>() != -1000) dix[r] = group_dof<M>(g);
            else dix[r] = bounded(gi[g * GIW + GI_DOF], 0, 1 << 16);
        }
#pragma unroll
        for (int r = 0; r < NGR; ++r) {
            qv[r] = dofs[2 * dix[r]];
            qdv[r] = dofs[2 * dix[r] + 1];
        }
#pragma unroll
        for (int r = 0; r < NGR; ++r) {
            const int g = 1 + sub + r * LPE;
            if (g < M::NG) {
                s(g * GF + F_Q) = qv[r];
                s(g * GF + F_QD) = qdv[r];
            }
        }
    }
    if (sub == 0) {   // the root group's pose in its own frame (never rewritten)
        stR(s, 0, eye3());
        stv3(s, F_P, v3(0, 0, 0));
    }
    V3 pos = v3(rt0[0], rt0[1], rt0[2]);
    float qx = rt0[3], qy = rt0[4], qz = rt0[5], qw = rt0[6];
    {
        const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
        qx *= in; qy *= in; qz *= in; qw *= in;
    }
    M3 R = quat_to_m3(qx, qy, qz, qw);
    const V3 c0 = v3(M::root_com[0], M::root_com[1], M::root_com[2]);
    const V3 ww = v3(rt0[10], rt0[11], rt0[12]);
    const V3 vo = v3(rt0[7], rt0[8], rt0[9]) - cross(ww, mul(R, c0));
    SV v0 = fix_base ? sv0() : SV{mulT(R, ww), mulT(R, vo)};
    const V3 grav = v3(a.gx, a.gy, a.gz);

    // rigid inertia + bias force of group g (pass 1 body) in the root frame;
    // v, the group's root-frame pose (Rg, Pg) and gravity in the root frame gr
    // already known.  cin: the group's composite inertia (m, com, Ic about the
    // com) in its own frame, from the per-env cache.
    //   c = P + R c_l, Ic_w = R Ic R^T, I = rb_inertia(m, c, Ic_w)
    //   h = m (v + w x c) (momentum), L = Ic_w w + c x h
    //   p = v x* (L, h) - (n, F),  F = m g - k_lin h + f_ext,
    //   n = c x F - k_ang Ic_w w + t_ext
    auto body_bias = [&](int g, const SV &vg, const M3 &Rg, V3 Pg, V3 gr, const float *cin) {
        const int o = g * GF;
        const float m = cin[0];
        const V3 c = Pg + mul(Rg, v3(cin[1], cin[2], cin[3]));
        float Icw[6];
        sym_rot(cin + 4, transpose(Rg), Icw);
        stsi(s, o + F_IA, rb_inertia(m, c, Icw));
        const V3 hm = m * (vg.v + cross(vg.w, c));
        const V3 Iw = symmul(Icw, vg.w);
        const V3 L = Iw + cross(c, hm);
        V3 F = m * gr - a.lin_damp * hm;
        V3 n = -a.ang_damp * Iw;
        if (a.force) {
            const float *fw = a.force + ((size_t)e * M::NG + g) * 6;
            F = F + mulT(R, v3(fw[0], fw[1], fw[2]));
            n = n + mulT(R, v3(fw[3], fw[4], fw[5]));
        }
        n = n + cross(c, F);
        const V3 bw = cross(vg.w, L) + cross(vg.v, hm), bv = cross(vg.w, hm);
        stsv(s, o + F_PA, SV{bw - n, bv - F});
    };
    // per-group per-env inputs, prefetched one schedule step ahead
    auto load_kin = [&](int g, float *x) {   // joint placement (12)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float4 v = CP4(CL::xtree(g) + 4 * k);
            x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
        }
    };
    // pass 1b: groups sub, sub + LPE, ... of the env (all lanes, no schedule)
    constexpr int NR1 = (M::NG + LPE - 1) / LPE;
#ifdef TG_DEV_R2   // developer timing probe (results wrong): the all-groups passes stop after two rounds
    constexpr int NRX = NR1 < 2 ? NR1 : 2;
#else
    constexpr int NRX = NR1;
#endif
    auto load_inertia = [&](float (*x)[12]) {   // mass, com, inertia (10 + 2 pad) of the lane's groups
#pragma unroll
        for (int r = 0; r < NR1; ++r) {
            const int g = sub + r * LPE;
            if (g < M::NG) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const float4 v = CP4(CL::inertia(g) + 4 * k);
                    x[r][4 * k] = v.x; x[r][4 * k + 1] = v.y; x[r][4 * k + 2] = v.z; x[r][4 * k + 3] = v.w;
                }
            }
        }
    };
    auto load_drv = [&](int d, float *x) {   // drive / limit inputs of dof d
        x[0] = PR(TG_PROP_ARMATURE, d);
        x[1] = PR(TG_PROP_DRIVE_MODE, d);
        x[2] = PR(TG_PROP_STIFFNESS, d);
        x[3] = PR(TG_PROP_DAMPING, d);
        x[4] = PR(TG_PROP_EFFORT, d);
        x[5] = PR(TG_PROP_LOWER, d);
        x[6] = PR(TG_PROP_UPPER, d);
        const unsigned ed = (unsigned)e * (unsigned)D + (unsigned)d;
        // the walk pre-physics inside the step (tg_walk_step): its targets, formed here from the actions
        // (one load from whichever buffer is live: the actions when the
        // pre-physics runs in this kernel, the stored targets otherwise)
        const float tv = at_u32<float>(a.pm_in_step ? a.pm_actions : a.pos_tgt, ed * 4u);
        x[7] = a.pm_in_step ? pm_target(a, d, pm_clamp(a, tv)) : tv;
        x[8] = at_u32<float>(a.vel_tgt, ed * 4u);
        if constexpr (PL::TPON) {   // the Gogoro pre-physics inside the step (tg_gogoro_step)
            if ((M::FUSED & 2) && a.gp_in_step) {
                if (d == a.gp.dof_steer) x[7] = s(PL::TP + 6);
                if (d == a.gp.dof_rear) x[8] = s(PL::TP + 7);
            } else if ((M::FUSED & 4) && a.pp_in_step) {   // the paper zeroes every other target
                x[7] = d == a.pp.dof_steer ? s(PL::TP + 6) : 0.f;
                x[8] = d == a.pp.dof_rear ? s(PL::TP + 7) : 0.f;
            }
        }
        x[9] = a.act ? at_u32<float>(a.act, ed * 4u) : 0.f;
    };
    // pass 2: the children's contributions of the lane's group, n = the step's
    // largest child count: absent children read the zero block, so every load
    // is issued before the first add (one LDS round trip)
    auto gather = [&](auto NCc, const I4 &dc, SI &IA, SV &pA) {
        constexpr int n = decltype(NCc)::value;
        SI ci[n];
        SV cv[n];
#pragma unroll
        for (int c = 0; c < n; ++c) {
            const bool has = c < d_nch(dc);
            const int ch = d_child(dc, c);
            const float *pi = has ? s.b + ia_c(ch) : zeros, *pp = has ? s.b + pa_c(ch) : zeros;
            ci[c] = ldsi(LE{(float *)__builtin_assume_aligned(pi, PL::ES % 4 == 0 ? 16 : 8)}, 0);
            cv[c] = ldsv(LE{(float *)__builtin_assume_aligned(pp, PL::ES % 4 == 0 ? 16 : 8)}, 0);
        }
#pragma unroll
        for (int c = 0; c < n; ++c) {
            si_add(IA, ci[c]);
            pA = pA + cv[c];
        }
    };
    // one-round trees (the lane's group is g = sub): its drive / limit inputs
    // are constant over the launch, so they are loaded once here instead of
    // in every substep and again for the drive-clamp rerun
    float cd1[10], vlim1 = 0.f, cin1[1][12];
    if constexpr (NR1 == 1) {
        if (sub > 0 && sub < M::NG) load_drv(bounded(gi[sub * GIW + GI_DOF], 0, 1 << 16), cd1);
        // and the velocity limit of group 1 + sub, the composite of group sub
        if (1 + sub < M::NG) vlim1 = PR(TG_PROP_VELOCITY, bounded(gi[(1 + sub) * GIW + GI_DOF], 0, 1 << 16));
        load_inertia(cin1);
    }
    // one-round trees: every schedule step's joint placement too (constant
    // over the launch: the epilogue's in-place seat moves come after the last
    // substep), so pass 1a waits for them once per launch, not once per substep
#ifndef TG_KIN_ONCE
#define TG_KIN_ONCE 1   // developer switch: 0 = per-substep prefetch ring (A/B)
#endif
    constexpr bool KIN1 = NR1 == 1 && TG_KIN_ONCE;
    float kin1[KIN1 ? M::NSTEP : 1][12];
    if constexpr (KIN1) {
#pragma unroll
        for (int t = 0; t < M::NSTEP; ++t) load_kin(pdsc(t).x, kin1[t]);
    }
    // the lane's contact shape (sh = sub): its pose in the contact group's
    // frame (composite cache) and its friction, constant over the launch --
    // loaded once here instead of inside every substep's contact setup, where
    // the loads sat on the chain (Gogoro 45.4 -> 45.1 us, GogoroPaper 36.9 ->
    // 36.5 us, A/B twice)
#ifndef TG_SHAPE_ONCE
#define TG_SHAPE_ONCE 1   // developer switch: 0 = loads inside the contact setup (A/B)
#endif
    // one lane per contact ROW when every row has a lane (ROWPAR, round 4;
    // the contact setup below), else one lane per shape; either way the
    // lane's shape is loaded here
#ifndef TG_ROW_PAR
#define TG_ROW_PAR 1   // developer switch: 0 = one lane per shape builds its rows (A/B)
#endif
    // (multi-point patches only -- the box faces' 7 rows per shape: on the
    // scooters' one-point tori, 3 rows per shape, every lane redoing the
    // shape geometry measured +0.35 % (Gogoro), where Thormang gains 1.0 %,
    // profiles/r4/rowpar_ab.txt)
    constexpr bool ROWPAR = TG_ROW_PAR && M::NS > 0 && PL::K <= LPE && max_shape_rows<M>() > 1;
    constexpr bool SHP1 = TG_SHAPE_ONCE && M::NS > 0 && (ROWPAR || M::NS <= LPE);
    float shp1[SHP1 ? 12 : 1], smu1 = 0.f;
    if constexpr (SHP1) {
        const int sh = ROWPAR ? row_shape_sel<M>(sub < PL::K ? sub : 0) : (sub < M::NS ? sub : 0);
#pragma unroll
        for (int k = 0; k < 12; ++k) shp1[k] = CP(CL::shape(sh) + k);
        smu1 = a.shape_mu[(size_t)e * M::NS + sh];
    }
    // an epilogue's inputs it wants in flight for the whole step (P::prefetch)
    float xpre[P::NPRE > 0 ? P::NPRE : 1];
    if constexpr (P::NPRE > 0) P::template prefetch<M, LPE>(pa, a, e, sub, xpre);
    TG_SYNC();
    TG_PROF(0)

    // ---- Woodbury drive-clamp state of the current substep (PL::WOOD):
    // the env's clamped groups as a lane mask, their count
    unsigned wmask = 0u;
    int wn = 0;
    // the a-th clamped group of the env (ascending group order)
    auto wgroup = [&](int aidx) {
        unsigned m = wmask;
        for (int k = 0; k < aidx; ++k) m &= m - 1u;
        return 1 + (int)__builtin_ctz(m);
    };
    // LDL6 / a0 of the substep are passed in (the lambda is defined once)
    auto wood_update_impl = [&](const LDL6 &rf, SV &acc0) -> bool {
        if constexpr (PL::WOOD) {
            constexpr int WCM = PL::WCM;
            const int gl = 1 + sub;
            const bool clm = gl < M::NG && s(gl * GF + F_C1) != 0.f;
            const uint64_t bal = __ballot(clm);
            const int lw = (int)(threadIdx.x % 64);
            wmask = (unsigned)(bal >> (lw - sub)) & ((1u << LPE) - 1u);
            wn = __builtin_popcount(wmask);
            if (wn > WCM) { wn = 0; wmask = 0u; return false; }   // more than WCM saturate: the rerun
            // (1) lane aidx < wn: the response of the whole tree to a unit torque
            // at clamped group ga (the articulated inertias of the first solve):
            // up-walk along ga's ancestors, root solve, top-down over every group
            if (sub < wn) {
                const int ga = wgroup(sub);
                SV dp = sv0();
                float dus[M::NG];
                dus[0] = 0.f;
#pragma unroll
                for (int g = M::NG - 1; g >= 1; --g) {
                    // g on ga's path: g == ga or an ancestor of ga (compile-time table)
                    bool onp = false;
#pragma unroll
                    for (int k = 1; k < M::NG; ++k) onp = (ga == k) ? (M::anc[k][g] != 0) : onp;
                    const SV Ug = ldsv(s, g * GF + F_U);
                    const float di = s(g * GF + F_DINV);
                    const SV Sg = ldSm<M>(s, g, M::jtype[g]);
                    float du = g == ga ? 1.f : -dot(Sg, dp);
                    du = onp ? du : 0.f;
                    dus[g] = du;
                    dp = dp + (du * di) * Ug;
                }
                const SV ar = fix_base ? sv0() : ldl6_solve(rf, -1.0f * dp);
                SV acc[M::NG];
                float qgs[M::NG];
                acc[0] = ar;
                qgs[0] = 0.f;
#pragma unroll
                for (int g = 1; g < M::NG; ++g) {
                    const SV ap = acc[M::parent[g]];
                    const SV Ug = ldsv(s, g * GF + F_U);
                    const float di = s(g * GF + F_DINV);
                    const float qg = (dus[g] - dot(Ug, ap)) * di;
                    acc[g] = ap + qg * ldSm<M>(s, g, M::jtype[g]);
                    qgs[g] = qg;
                    s(PL::WB_G + 8 * sub + g) = qg;
                }
                stsv(s, PL::WB_R + 6 * sub, ar);
                // (the contact groups' responses about their own origins, as the rows take them)
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) {
                    const V3 pcc = ldv3(s, M::cgroup[c] * GF + F_P);
                    SV al = shift_to(ar, pcc);
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i) {
                        if (i < M::cpath_len[c]) {
                            const int hg = M::cpath[c][i];
                            al = al + qgs[hg] * motion_at<M>(M::jtype[hg], ldv3(s, hg * GF + F_AX),
                                                             ldv3(s, hg * GF + F_P), pcc);
                        }
                    }
                    stsv(s, PL::WB_A + 6 * (M::NCG * sub + c), al);
                }
            } else if (sub < WCM) {
                // the unused response slots (wn < WCM): zeros, because the
                // fixed-size WCM sums below multiply them by zero weights, and
                // 0 x whatever an earlier kernel left in this LDS is NaN when
                // that was a NaN pattern (ragged-batch Gogoro runs hit it)
#pragma unroll
                for (int g = 0; g < 8; ++g) s(PL::WB_G + 8 * sub + g) = 0.f;
                stsv(s, PL::WB_R + 6 * sub, sv0());
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) stsv(s, PL::WB_A + 6 * (M::NCG * sub + c), sv0());
            }
            TG_SYNC();
            // (2) every lane: the clamped system M = K^-1 - E^T G (wn x wn), the
            // correction w = delta + M^-1 (qdd_C + N delta), delta = +-effort - te
            float Kc[WCM], dl[WCM], qc[WCM], Nm[WCM][WCM];
            int gc[WCM];
#pragma unroll
            for (int i = 0; i < WCM; ++i) {
                gc[i] = i < wn ? wgroup(i) : 1;
                const int o = gc[i] * GF;
                const float te = s(o + F_CL), K = s(o + F_CL + 1), eff = s(o + F_CL + 2), sg = s(o + F_C1);
                Kc[i] = K;
                dl[i] = i < wn ? sg * eff - te : 0.f;
                qc[i] = s(o + F_UU);
            }
#pragma unroll
            for (int i = 0; i < WCM; ++i)
#pragma unroll
                for (int j = 0; j < WCM; ++j) Nm[i][j] = s(PL::WB_G + 8 * j + gc[i]);   // response of i's dof to torque j
            float Mm[WCM][WCM], Mi[WCM][WCM];
#pragma unroll
            for (int i = 0; i < WCM; ++i)
#pragma unroll
                for (int j = 0; j < WCM; ++j) Mm[i][j] = (i == j ? 1.0f / Kc[i] : 0.f) - Nm[i][j];
            static_assert(WCM == 2, "closed-form inverse below");
            if (wn == 1) {
                Mi[0][0] = 1.0f / Mm[0][0]; Mi[0][1] = Mi[1][0] = Mi[1][1] = 0.f;
            } else {
                const float det = Mm[0][0] * Mm[1][1] - Mm[0][1] * Mm[1][0], id = 1.0f / det;
                Mi[0][0] = Mm[1][1] * id; Mi[1][1] = Mm[0][0] * id;
                Mi[0][1] = -Mm[0][1] * id; Mi[1][0] = -Mm[1][0] * id;
            }
            float wv[WCM];
#pragma unroll
            for (int i = 0; i < WCM; ++i) {
                float r = qc[i];
#pragma unroll
                for (int j = 0; j < WCM; ++j) r += Nm[i][j] * dl[j];
                wv[i] = r;
            }
#pragma unroll
            for (int i = 0; i < WCM; ++i) {
                float z = 0.f;
#pragma unroll
                for (int j = 0; j < WCM; ++j) z += Mi[i][j] * wv[j];
                wv[i] = i < wn ? dl[i] + z : 0.f;
            }
            // (3) the corrected accelerations: qdd += G w (the lane's group), a0 += R w
            if (gl < M::NG) {
                float dq = 0.f;
#pragma unroll
                for (int i = 0; i < WCM; ++i) dq += s(PL::WB_G + 8 * i + gl) * wv[i];
                s(gl * GF + F_UU) += dq;
                s(gl * GF + F_QDS) += h * dq;
            }
#pragma unroll
            for (int i = 0; i < WCM; ++i) acc0 = acc0 + wv[i] * ldsv(s, PL::WB_R + 6 * i);
            if (sub == 0) {
#pragma unroll
                for (int i = 0; i < WCM; ++i)
#pragma unroll
                    for (int j = 0; j < WCM; ++j) s(PL::WB_M + WCM * i + j) = Mi[i][j];
            }
            TG_SYNC();
            return true;
        } else {
            (void)rf; (void)acc0;
            return false;
        }
    };
#ifndef TG_EPI_TOUCH
#define TG_EPI_TOUCH 0   // developer switch: 1 = touch the epilogue's inputs in the last substep (round 4 A/B: +0.6 us, AGPRs 54 -> 65; profiles/r4/epilogue_touch_ab.txt)
#endif
    constexpr bool EPI_TOUCH = TG_EPI_TOUCH && P::TOUCH;
    float epi_touch = 0.f;
    for (int sub_i = 0; sub_i < a.substeps; ++sub_i) {
        // Passes 1-3 run with every position/velocity drive implicit and
        // unclamped; if some drive's implicit end-of-substep torque te - K*qdd
        // exceeds its effort, they run once more with those drives as the
        // explicit torque +-effort ("implicit, then clamp", as
        // oracle/physics_ref.c aba()).  Between the two runs the F_CL slots of
        // a drive group hold (te, K, effort) and F_UU holds qdd.
        // Every schedule step below issues all its LDS loads before its first
        // LDS store (the compiler keeps LDS loads and stores in program order).
        LDL6 rootf{};
        SV a0 = sv0();
        wmask = 0u;
        wn = 0;
        auto wood_update = [&]() { return wood_update_impl(rootf, a0); };
        // velocity limits of the lane's groups (used by the integration at the
        // end of the substep), issued now so their latency is hidden
        float vlim[(M::NG + LPE - 1) / LPE];
        if constexpr (NR1 == 1) {
            vlim[0] = vlim1;
        } else {
#pragma unroll
        for (int r = 0; r < (M::NG + LPE - 1) / LPE; ++r) {
            const int g = 1 + sub + r * LPE;
            vlim[r] = g < M::NG ? PR(TG_PROP_VELOCITY, bounded(gi[g * GIW + GI_DOF], 0, 1 << 16)) : 0.f;
        }
        }
        // a leaf group's joint-space inertia D0 = S.I.S from its own rigid
        // inertia about its joint (group frame: the axis is e_z), Izz + m (cx^2
        // + cy^2) (revolute) or m (prismatic) -- pass 2b's S.(I^A S) forms it
        // from the inertia about the ROOT origin, where a wheel 0.8 m away
        // carries m |P|^2 ~ 35x its spin inertia and loses those digits
        // (round 6); -1 = not a leaf.  Formed in pass 1b, used by pass 2a.
        float d0l[NR1];
#pragma unroll
        for (int r = 0; r < NR1; ++r) d0l[r] = -1.f;
#pragma unroll 1
        for (int cp = 0; cp < 2; ++cp) {
#if defined(TG_SECTION_PROF) && defined(TG_CLAMP_COUNT)
        // counters (perturb the pass-1 timing, hence a separate switch):
        // [12] env-substeps, [13] env-substeps with the clamp rerun,
        // [14] wave-substeps, [15] wave-substeps that rerun
        if (lead && owner) atomicAdd(&tg_prof_acc[12 + cp], 1ull);
        if (tid % 64 == 0) atomicAdd(&tg_prof_acc[14 + cp], 1ull);
#endif
        // ---- pass 1: root, then the schedule forward (SEPC: not rerun, its
        // results are intact).  Descriptors run two steps ahead, the cache
        // inputs one step ahead.
        if (!SEPC || cp == 0) {
        // 1a (schedule forward): root-frame poses and velocities; 1b (every
        // group at once, LPE lanes wide): rigid inertias and bias forces,
        // which depend on the group's own pose and velocity only
        const V3 gr = mulT(R, grav);   // gravity in the root frame
        float cin[NR1][12];
        if constexpr (NR1 == 1) {
#pragma unroll
            for (int k = 0; k < 12; ++k) cin[0][k] = cin1[0][k];
        } else {
            load_inertia(cin);
        }
        if (lead) stsv(s, F_V, v0);
        TG_SYNC();
#ifndef TG_PROBE
#define TG_PROBE 0   // developer timing probes (results wrong): the tree passes' parent / child LDS traffic
#endif               // replaced by the lane's own previous-step registers (1 pass 1a, 2 pass 2b, 4 pass 3, 8 impulse)
        // (chain schedule: the parent's pose and velocity are the lane's own
        // previous step's, the root's at step 0)
        constexpr bool CH = Chain<M>::ON && (TG_CHAIN_MASK & 1);
        constexpr bool CH1 = CH || (TG_PROBE & 1);
#ifndef TG_Q_AHEAD
#define TG_Q_AHEAD 1   // pass 1a: q, qd loaded two steps ahead (0: in the step, the A/B control)
#endif
        M3 pr_R = eye3();
        V3 pr_P = v3(0, 0, 0);
        SV pr_v = v0;
        // the group's joint position / velocity, loaded two steps ahead with
        // the step's other inputs (pass 1a does not write them)
        auto ld_q = [&](const I4 &dc, float *qq) {
            const int o = max(dc.x, 0) * GF;
            qq[0] = s(o + F_Q);
            qq[1] = s(o + F_QD);
        };
        // chain form without branches (TG_1A_FLAT): every lane runs its step,
        // idle lanes on the root's inputs, and a lane that does not own its
        // group stores into the Delassus / row area, which the contact setup
        // rebuilds later in the substep -- straight-line code, so the
        // compiler can overlap a step's parent-independent work (sin / cos,
        // the joint rotation) with the previous step's chain
#ifndef TG_1A_FLAT
#define TG_1A_FLAT 1
#endif
        constexpr bool FLAT1 = CH && TG_1A_FLAT && PL::VFREE - PL::W >= F_V + 6;
// an idle lane (its chain ended) updates its chain registers too -- they
// are dead after the pass -- so the update is a register rename, not a
// divergent branch of 18 moves: on trees of at least TG_1A_IDLE_FREE groups
// (the humanoids: ThormangWalk 49.4 -> 48.1 us, bit-identical,
// profiles/r5/idle_free_ab.txt).  The scooters keep the branch: without it
// the compiler fuses some multiply-adds differently (fp-contract works per
// basic block), which changes their rounding (1e-4 after 100 steps).
#ifndef TG_1A_IDLE_FREE
#define TG_1A_IDLE_FREE 16
#endif
        constexpr bool IDLE_FREE = TG_1A_IDLE_FREE > 0 && M::NG >= TG_1A_IDLE_FREE;
        auto body1f = [&](const I4 &dc, const float *ck, const float *qq) {
            const int g = dc.x, jt = d_jt(dc);
            const float qg = qq[0], qdg = qq[1];
            M3 Rpc;
#pragma unroll
            for (int k = 0; k < 9; ++k) Rpc.a[k] = ck[k];
            V3 tr = v3(ck[9], ck[10], ck[11]);
            float sq, cq;
            tg_sincos(qg, &sq, &cq);
            if (all_revolute<M>() || jt == TG_JOINT_REVOLUTE) {   // Rpc * Rz(q), else a shifted origin
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const float c0 = Rpc.a[3 * r], c1 = Rpc.a[3 * r + 1];
                    Rpc.a[3 * r] = c0 * cq + c1 * sq;
                    Rpc.a[3 * r + 1] = c1 * cq - c0 * sq;
                }
            } else {
                tr = tr + qg * v3(Rpc.a[2], Rpc.a[5], Rpc.a[8]);
            }
            const M3 Rg = mul(pr_R, Rpc);
            const V3 Pg = pr_P + mul(pr_R, tr);
            const SV Sg = motion_Sm<M>(jt, v3(Rg.a[2], Rg.a[5], Rg.a[8]), Pg);
            const SV vg = pr_v + qdg * Sg;
            const int os = (g > 0 && d_own(dc)) ? g * GF : PL::W;
            stm3(s, os + F_RT, transpose(Rg));
            stv3(s, os + F_P, Pg);
            stsv(s, os + F_V, vg);
            if (IDLE_FREE || g > 0) {   // (see TG_1A_IDLE_FREE)
                pr_R = Rg;
                pr_P = Pg;
                pr_v = vg;
            }
        };
        auto body1 = [&](const I4 &dc, const float *ck, const float *qq) {
            if constexpr (FLAT1) {
                body1f(dc, ck, qq);
                return;
            }
            const int g = dc.x;
            if (g > 0) {
                const int o = g * GF, par = dc.y, jt = d_jt(dc);
                M3 Rp;
                V3 Pp;
                SV vp;
                if constexpr (CH1) {
                    Rp = pr_R;
                    Pp = pr_P;
                    vp = pr_v;
                } else {
                    Rp = ldR(s, par);
                    Pp = ldv3(s, par * GF + F_P);
                    vp = ldsv(s, par * GF + F_V);
                }
#if TG_Q_AHEAD
                const float qg = qq[0], qdg = qq[1];
#else
                (void)qq;
                const float qg = s(o + F_Q), qdg = s(o + F_QD);
#endif
                M3 Rpc;   // child -> parent rotation at q, then the root-frame pose
#pragma unroll
                for (int k = 0; k < 9; ++k) Rpc.a[k] = ck[k];
                V3 tr = v3(ck[9], ck[10], ck[11]);
                if (all_revolute<M>() || jt == TG_JOINT_REVOLUTE) {   // Rpc * Rz(q)
                    float sq, cq;
                    tg_sincos(qg, &sq, &cq);
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const float c0 = Rpc.a[3 * r], c1 = Rpc.a[3 * r + 1];
                        Rpc.a[3 * r] = c0 * cq + c1 * sq;
                        Rpc.a[3 * r + 1] = c1 * cq - c0 * sq;
                    }
                } else {
                    tr = tr + qg * v3(Rpc.a[2], Rpc.a[5], Rpc.a[8]);
                }
                const M3 Rg = mul(Rp, Rpc);
                const V3 Pg = Pp + mul(Rp, tr);
                const SV Sg = motion_Sm<M>(jt, v3(Rg.a[2], Rg.a[5], Rg.a[8]), Pg);
                const SV vg = vp + qdg * Sg;
                if (!CH || d_own(dc)) {   // (chain: the group's owner stores it)
                    stR(s, g, Rg);
                    stv3(s, o + F_P, Pg);
                    stsv(s, o + F_V, vg);
                }
                if constexpr (CH1) {
                    pr_R = Rg;
                    pr_P = Pg;
                    pr_v = vg;
                }
            }
            if constexpr (!CH || TG_CHAIN_SYNC) TG_SYNC();
        };
        static_assert(!FLAT1 || TG_Q_AHEAD, "the flat chain form takes q, qd from the prefetch ring");
        // fully unrolled, inputs two steps ahead in a 3-deep ring (renamed
        // registers, no copies: the wait for step t's inputs leaves steps
        // t + 1 and t + 2 in flight)
        float qr[3][2];
#ifndef TG_1A_REPS
#define TG_1A_REPS 1   // developer ablation: pass 1a run this many times (idempotent: its marginal cost)
#endif
#pragma unroll 1
        for (int rep1 = 0; rep1 < TG_1A_REPS; ++rep1) {
        if (rep1 > 0) {
            pr_R = eye3();
            pr_P = v3(0, 0, 0);
            pr_v = v0;
        }
        if constexpr (KIN1) {
            I4 dr[3];
            dr[0] = pdsc(0);
            if (TG_Q_AHEAD) ld_q(dr[0], qr[0]);
            if constexpr (M::NSTEP > 1) {
                dr[1] = pdsc(1);
                if (TG_Q_AHEAD) ld_q(dr[1], qr[1]);
            }
#pragma unroll
            for (int t = 0; t < M::NSTEP; ++t) {
                if (t + 2 < M::NSTEP) {
                    dr[(t + 2) % 3] = pdsc(t + 2);
                    if (TG_Q_AHEAD) ld_q(dr[(t + 2) % 3], qr[(t + 2) % 3]);
                }
                body1(dr[t % 3], kin1[t], qr[t % 3]);
            }
        } else {
#ifndef TG_KIN_AHEAD
#define TG_KIN_AHEAD 2   // pass 1a: the joint placements (composite cache) issued this many steps ahead
#endif
        constexpr int KA = TG_KIN_AHEAD, KR = KA + 1;
        float kr[KR][12], qk[KR][2];
        I4 dr[KR];
#pragma unroll
        for (int t = 0; t < KA && t < M::NSTEP; ++t) {
            dr[t] = pdsc(t);
            load_kin(dr[t].x, kr[t]);
            if (TG_Q_AHEAD) ld_q(dr[t], qk[t]);
        }
#pragma unroll
        for (int t = 0; t < M::NSTEP; ++t) {
            if (t + KA < M::NSTEP) {
                dr[(t + KA) % KR] = pdsc(t + KA);
                load_kin(dr[(t + KA) % KR].x, kr[(t + KA) % KR]);
                if (TG_Q_AHEAD) ld_q(dr[(t + KA) % KR], qk[(t + KA) % KR]);
            }
            body1(dr[t % KR], kr[t % KR], qk[t % KR]);
        }
        }
        }
        if constexpr (CH && (!TG_CHAIN_SYNC || FLAT1)) TG_SYNC();   // (pass 1b reads every group's pose)
#ifdef TG_DUMMY_STEPS
        // developer ablation: TG_DUMMY_STEPS dependent LDS round trips with no
        // arithmetic (kind 0: one float; kind 1: pass 1a's traffic, 18 floats
        // read from the next lane's slot, 18 written to the own slot) in the
        // (not yet used) Delassus / row area: the fixed cost of a schedule step
        {
            float *ds = s.b + PL::W;
            for (int t = 0; t < TG_DUMMY_STEPS; ++t) {
                const float *src = ds + 20 * ((sub + 1) % LPE);
                float *dst = ds + 20 * sub;
#if TG_DUMMY_KIND == 0
                float x = src[0];
                __asm__ volatile("" : "+v"(x));
                dst[0] = x;
#elif TG_DUMMY_KIND == 2   // 18 read, 1 written
                float x[18];
#pragma unroll
                for (int k = 0; k < 18; ++k) x[k] = src[k];
#pragma unroll
                for (int k = 0; k < 18; ++k) __asm__ volatile("" : "+v"(x[k]));
                dst[0] = x[0];
#elif TG_DUMMY_KIND == 3   // 1 read, 18 written
                float x = src[0];
                __asm__ volatile("" : "+v"(x));
#pragma unroll
                for (int k = 0; k < 18; ++k) dst[k] = x;
#elif TG_DUMMY_KIND == 4   // kind 1, stores by one lane of each pair only
                float x[18];
#pragma unroll
                for (int k = 0; k < 18; ++k) x[k] = src[k];
#pragma unroll
                for (int k = 0; k < 18; ++k) __asm__ volatile("" : "+v"(x[k]));
                if (sub < M::SL) {
#pragma unroll
                    for (int k = 0; k < 18; ++k) dst[k] = x[k];
                }
#else
                float x[18];
#pragma unroll
                for (int k = 0; k < 18; ++k) x[k] = src[k];
#pragma unroll
                for (int k = 0; k < 18; ++k) __asm__ volatile("" : "+v"(x[k]));
#pragma unroll
                for (int k = 0; k < 18; ++k) dst[k] = x[k];
#endif
                TG_SYNC();
            }
        }
#endif
#ifdef TG_PROF_SPLIT0   // developer: pass 1a of the first substep into its own slot (20)
        TG_PROF(sub_i == 0 ? 20 : 16)
#else
        TG_PROF(16)
#endif
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
            const int g = sub + r * LPE;
            if (g < M::NG) body_bias(g, ldsv(s, g * GF + F_V), ldR(s, g), ldv3(s, g * GF + F_P), gr, cin[r]);
            if constexpr (TG_LEAF_D0) {
                const int gl = min(g, M::NG - 1);
                const bool leaf = g > 0 && g < M::NG && gi[gl * GIW + GI_NCH] == 0;
                const bool rev = all_revolute<M>() || gi[gl * GIW + GI_JT] == TG_JOINT_REVOLUTE;
                const float *ci = cin[r];
                d0l[r] = leaf ? (rev ? ci[6] + ci[0] * (ci[1] * ci[1] + ci[2] * ci[2]) : ci[0]) : -1.f;
            }
        }
        TG_SYNC();
        }   // pass 1
        TG_PROF(1)
        // ---- pass 2a (every group at once, LPE lanes wide): the joint-space
        // terms that need no articulated inertia -- drive torque and implicit
        // gain (implicit, or clamped to +-effort on the rerun), effort torque,
        // limit spring/damper as multiples of D0 = S.I^A.S, velocity-product
        // acceleration cb -- parked in the group's own slots (F_V: cb, which
        // pass 3 reads too; F_DINV: c0, F_UU: tau, F_QDS: limit torque per D0, F_C1: 1 +
        // limit gain per D0)
        if constexpr (NR1 > 1) {
        // Every round's drive inputs are loaded first (clamped group index: the
        // loads are unconditional) and consumed by branch-free arithmetic with
        // only the stores predicated, so the compiler cannot sink a load into a
        // conditional block that uses it: the rounds share one memory latency.
        float cdr[NR1][10];
        if constexpr (EPI_TOUCH) {
            // the last substep: one line of the epilogue's inputs per lane
            // brought into the cache with this pass's own HBM loads, so the
            // epilogue's loads at the end of the kernel hit it
            if (sub_i == a.substeps - 1 && cp == 0) epi_touch = *P::template touch_addr<M, LPE>(pa, a, e, sub);
        }
#pragma unroll
        for (int r = 0; r < NR1; ++r) {
            const int gc = min(max(sub + r * LPE, 1), M::NG - 1);
            load_drv(bounded(gi[gc * GIW + GI_DOF], 0, 1 << 16), cdr[r]);
        }
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
            const int g0 = sub + r * LPE;
            const bool valid = g0 > 0 && g0 < M::NG;
            const int g = min(max(g0, 1), M::NG - 1);
            const int o = g * GF;
            const float *cd = cdr[r];
            const float q = s(o + F_Q), qd = s(o + F_QD), qdd0 = s(o + F_UU);
            const int mode = (int)rintf(cd[1]);
            const float kp = cd[2], kd = cd[3];
            const float eff = cd[4];
            const bool drv = mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL;
            const float te = kp * (cd[7] - q - h * qd) + kd * (cd[8] - qd);
            const float K = h * kd + h * h * kp;
            // implicit, or (rerun) clamped to +-effort when the implicit torque of the first solve exceeds it
            const float ti = te - K * qdd0;   // qdd0: qdd of the first solve
            const bool clampd = drv && cp == 1 && fabsf(ti) > eff;
            const bool implicit = drv && !clampd;
            const float ef = (mode == TG_DOF_MODE_EFFORT && a.act) ? fminf(fmaxf(cd[9], -eff), eff) : 0.f;
            const float tau = implicit ? te : (clampd ? (ti > 0.f ? eff : -eff) : ef);
            const float Dimp = implicit ? K : 0.f;
            const float cl0 = drv ? te : 0.f, cl1 = drv ? K : -1.f;   // clamp scratch (te, K) of the first solve
            // limit spring + damping (kl = lim_k D0 / h^2, cl = lim_c D0 / h),
            // damping/implicit terms ramped in past the limit
            const float lo = cd[5], hi = cd[6];
            const float qp = q + h * qd;
            const bool below = qp < lo && lo > -1e30f, above = !below && qp > hi && hi < 1e30f;
            const float lim = below ? lo : hi;
            const float rr = fminf(fabsf(lim - qp) * (1.0f / TG_LIMIT_RAMP), 1.0f);
            const bool on = below || above;
            const float al = on ? a.lim_k / (h * h) * (lim - qp) - rr * a.lim_c / h * qd : 0.f;
            const float be = on ? rr * (a.lim_c + a.lim_k) : 0.f;
            // with D0 = S.I^A.S + armature: D = (1 + be) D0 + Dimp, tau + al D0
            // cb replaces v (dead after pass 1b) in F_V; on a SEPC rerun pass 1
            // was not rerun and F_V already holds cb
            const SV cbv = crm(ldsv(s, o + F_V), qd * ldSm<M>(s, g, bounded(gi[g * GIW + GI_JT], 0, 4)));
            if (valid) {
                if (cp == 0) {
                    s(o + F_CL) = cl0;
                    s(o + F_CL + 1) = cl1;
                    s(o + F_CL + 2) = eff;
                }
                if (!SEPC || cp == 0) stsv(s, o + F_V, cbv);
                // (a leaf: D and u complete here from its local D0, pass 2b adds 0 x D0)
                const bool lf = TG_LEAF_D0 && d0l[r] >= 0.f;
                s(o + F_DINV) = (1.f + be) * cd[0] + Dimp + (lf ? (1.f + be) * d0l[r] : 0.f);
                s(o + F_UU) = tau + al * cd[0] + (lf ? al * d0l[r] : 0.f);
                s(o + F_QDS) = lf ? 0.f : al;
                s(o + F_C1) = lf ? 0.f : 1.f + be;
            }
        }
        } else {   // one round (small trees): loads consumed at once, branches kept
#pragma unroll
        for (int r = 0; r < NR1; ++r) {
            const int g = sub + r * LPE;
            if (g > 0 && g < M::NG) {
                const int o = g * GF;
                const float *cd = cd1;   // loaded once per launch (below the prologue)
                const float q = s(o + F_Q), qd = s(o + F_QD), qdd0 = s(o + F_UU);
                float Dimp = 0.f, tau = 0.f;
                const int mode = (int)rintf(cd[1]);
                const float kp = cd[2], kd = cd[3];
                const float eff = cd[4];
                float cl0 = 0.f, cl1 = -1.f;   // clamp scratch (te, K) of the first solve
                if (mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL) {
                    const float te = kp * (cd[7] - q - h * qd) + kd * (cd[8] - qd);
                    const float K = h * kd + h * h * kp;
                    bool implicit = true;
                    cl0 = te;
                    cl1 = K;
                    if (cp == 1) {
                        const float ti = te - K * qdd0;   // qdd0: qdd of the first solve
                        if (fabsf(ti) > eff) {
                            implicit = false;
                            tau += ti > 0.f ? eff : -eff;
                        }
                    }
                    if (implicit) { tau += te; Dimp += K; }
                } else {
                    if (mode == TG_DOF_MODE_EFFORT && a.act) tau += fminf(fmaxf(cd[9], -eff), eff);
                }
                // limit spring + damping (kl = lim_k D0 / h^2, cl = lim_c D0 / h),
                // damping/implicit terms ramped in past the limit
                const float lo = cd[5], hi = cd[6];
                const float qp = q + h * qd;
                float al = 0.f, be = 0.f;
                if (qp < lo && lo > -1e30f) {
                    const float rr = fminf((lo - qp) * (1.0f / TG_LIMIT_RAMP), 1.0f);
                    al = a.lim_k / (h * h) * (lo - qp) - rr * a.lim_c / h * qd;
                    be = rr * (a.lim_c + a.lim_k);
                } else if (qp > hi && hi < 1e30f) {
                    const float rr = fminf((qp - hi) * (1.0f / TG_LIMIT_RAMP), 1.0f);
                    al = a.lim_k / (h * h) * (hi - qp) - rr * a.lim_c / h * qd;
                    be = rr * (a.lim_c + a.lim_k);
                }
                if (cp == 0) {
                    s(o + F_CL) = cl0;
                    s(o + F_CL + 1) = cl1;
                    s(o + F_CL + 2) = eff;
                }
                // with D0 = S.I^A.S + armature: D = (1 + be) D0 + Dimp, tau + al D0
                // cb replaces v (dead after pass 1b) in F_V; on a SEPC rerun pass 1
                // was not rerun and F_V already holds cb
                if (!SEPC || cp == 0) stsv(s, o + F_V, crm(ldsv(s, o + F_V), qd * ldSm<M>(s, g, bounded(gi[g * GIW + GI_JT], 0, 4))));
                // (a leaf: D and u complete here from its local D0, pass 2b adds 0 x D0)
                const bool lf = TG_LEAF_D0 && d0l[r] >= 0.f;
                s(o + F_DINV) = (1.f + be) * cd[0] + Dimp + (lf ? (1.f + be) * d0l[r] : 0.f);
                s(o + F_UU) = tau + al * cd[0] + (lf ? al * d0l[r] : 0.f);
                s(o + F_QDS) = lf ? 0.f : al;
                s(o + F_C1) = lf ? 0.f : 1.f + be;
            }
        }
        }
        TG_SYNC();
        TG_PROF(17)
        // ---- pass 2b: schedule backward, children contributions gathered
        if constexpr (M::PAIR) {
        // Lane pairs split the group's update as the same instructions on
        // different data: with I = [A B; B^T C] acting on (w, v), lane half 0
        // computes the angular rows (X = A, Y = B, S1 = S.w, S2 = S.v), half 1
        // the linear rows (X = C, Y = B^T, S1 = S.v, S2 = S.w).  Dot products
        // over the 6-vector are completed with the partner's half (DPP swap);
        // B's update is formed so that both halves compute its entries from the
        // same two factors, and half 0 stores it.
        const int hh = sub >= M::SL ? 1 : 0;
        const bool hb = hh != 0;
        auto pswap3 = [](const float *v, float *o) {
#pragma unroll
            for (int k = 0; k < 3; ++k) o[k] = pair_swap(v[k]);
        };
        // unrolled (round 2: ThormangWalk kernel 56.8 -> 56.5 us, A/B twice),
        // the step index a compile-time constant (its gather width too)
        // (the children's descriptor read one step ahead, ahead of the step's own loads)
        I4 dnext = dsc(M::NSTEP - 1);
        float p2X[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, p2B[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f},
              p2p[3] = {0.f, 0.f, 0.f};
        (void)p2X; (void)p2B; (void)p2p;
        static_for<0, M::NSTEP>([&](auto TT) {
            constexpr int t = M::NSTEP - 1 - decltype(TT)::value;
            const I4 dc = dnext;   // (children for the gather)
            if constexpr (t > 0) dnext = dsc(t - 1);
            const I4 pc = pdsc2(t);  // own group from registers: its loads need not wait for dc
            const int g = pc.x;
            // (chain schedule: each group on its owner lane only; the first
            // child's contribution is in this lane's registers from the step
            // before, zeros for a leaf)
            constexpr bool CH2 = Chain<M>::ON && (TG_CHAIN_MASK & 2);
            if (g > 0 && (!CH2 || d_own(pc))) {
                const int o = g * GF;
                float X[6], Bm[9], ph[3], cb1[3], cb2[3];
#pragma unroll
                for (int k = 0; k < 6; ++k) X[k] = s(o + F_IA + 15 * hh + k);
#pragma unroll
                for (int k = 0; k < 9; ++k) Bm[k] = s(o + F_IA + 6 + k);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ph[k] = s(o + F_PA + 3 * hh + k);
                    cb1[k] = s(o + F_V + 3 * hh + k);
                    cb2[k] = s(o + F_V + 3 - 3 * hh + k);
                }
                const SV Sg = ldSm<M>(s, g, d_jt(pc));
                const float c0 = s(o + F_DINV), tau = s(o + F_UU), al = s(o + F_QDS), c1 = s(o + F_C1);
                // children: every load issued before the first add (absent children read the zero block)
                auto gather2 = [&](auto NCc, auto C0c) {
                    constexpr int n = decltype(NCc)::value, c0 = decltype(C0c)::value;
                    float cx[n][6], cbm[n][9], cp[n][3];
#pragma unroll
                    for (int c = c0; c < n; ++c) {
                        const bool has = c < d_nch(dc);
                        const int ch = d_child(dc, c);
                        const float *pi = has ? s.b + ia_c(ch) : zeros, *pp = has ? s.b + pa_c(ch) : zeros;
#pragma unroll
                        for (int k = 0; k < 6; ++k) cx[c][k] = pi[15 * hh + k];
#pragma unroll
                        for (int k = 0; k < 9; ++k) cbm[c][k] = pi[6 + k];
#pragma unroll
                        for (int k = 0; k < 3; ++k) cp[c][k] = pp[3 * hh + k];
                    }
#pragma unroll
                    for (int c = c0; c < n; ++c) {
#pragma unroll
                        for (int k = 0; k < 6; ++k) X[k] += cx[c][k];
#pragma unroll
                        for (int k = 0; k < 9; ++k) Bm[k] += cbm[c][k];
#pragma unroll
                        for (int k = 0; k < 3; ++k) ph[k] += cp[c][k];
                    }
                };
                constexpr int smax = step_smax<M>(t);
                if constexpr (CH2 || (TG_PROBE & 2)) {
                    // the first child from registers, then the children after it
                    // (other chains' heads) from LDS -- the list schedule's order;
                    // a leaf adds nothing (not even the zeros its registers hold:
                    // x + 0 is not x for x = -0 and denormals under the fast-math
                    // unit's flushing, and the chain form would then round apart
                    // from the list schedule's, measured)
                    if (d_nch(dc) > 0) {
#pragma unroll
                        for (int k = 0; k < 6; ++k) X[k] += p2X[k];
#pragma unroll
                        for (int k = 0; k < 9; ++k) Bm[k] += p2B[k];
#pragma unroll
                        for (int k = 0; k < 3; ++k) ph[k] += p2p[k];
                    }
                    if constexpr (CH2 && smax >= 2) gather2(IntC<(smax < 3 ? smax : 3)>{}, IntC<1>{});
                } else {
                    if constexpr (smax >= 1) gather2(IntC<(smax < 3 ? smax : 3)>{}, IntC<0>{});
                }
                // the half's orientation of B
                float Y[9];
                Y[0] = Bm[0]; Y[4] = Bm[4]; Y[8] = Bm[8];
                Y[1] = hb ? Bm[3] : Bm[1]; Y[3] = hb ? Bm[1] : Bm[3];
                Y[2] = hb ? Bm[6] : Bm[2]; Y[6] = hb ? Bm[2] : Bm[6];
                Y[5] = hb ? Bm[7] : Bm[5]; Y[7] = hb ? Bm[5] : Bm[7];
                const V3 S1 = hb ? Sg.v : Sg.w, S2 = hb ? Sg.w : Sg.v;
                const V3 Uv = symmul(X, S1) + bmul(Y, S2);
                const float Uh[3] = {Uv.x, Uv.y, Uv.z};
                const float d0 = dot(S1, Uv);
                const float D0 = d0 + pair_swap(d0);   // S.U, without the armature (folded into c0, tau)
                const float sp = dot(S1, v3(ph[0], ph[1], ph[2]));
                const float SpA = sp + pair_swap(sp);
                const float Dinv = 1.0f / (c1 * D0 + c0);
                const float u = tau + al * D0 - SpA;
                float Uo[3], DUh[3], DUo[3], Pf[3], Qf[3];
                pswap3(Uh, Uo);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    DUh[k] = Dinv * Uh[k];
                    DUo[k] = Dinv * Uo[k];
                    Pf[k] = hb ? Uh[k] : DUh[k];   // B entries from the same two factors on both halves
                    Qf[k] = hb ? DUo[k] : Uo[k];
                }
                const int ii[6] = {0, 1, 2, 0, 0, 1}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
                for (int k = 0; k < 6; ++k) X[k] -= DUh[ii[k]] * Uh[jj[k]];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 3; ++j) Y[3 * i + j] -= Pf[i] * Qf[j];
                const float ud = u * Dinv;
                const V3 pav = v3(ph[0], ph[1], ph[2]) + symmul(X, v3(cb1[0], cb1[1], cb1[2])) +
                               bmul(Y, v3(cb2[0], cb2[1], cb2[2])) + ud * Uv;
                stv3(s, o + F_U + 3 * hh, Uv);
                s(o + F_DINV) = Dinv;
                s(o + F_UU) = u;
                // contribution to the parent (same frame: no transform); chain
                // schedule: into this lane's registers for the parent (B in its
                // canonical orientation: half 1 holds its transpose, bitwise),
                // and to LDS only when the parent is another lane's or the root
                if constexpr (CH2 || (TG_PROBE & 2)) {
#pragma unroll
                    for (int k = 0; k < 6; ++k) p2X[k] = X[k];
#pragma unroll
                    for (int i = 0; i < 3; ++i)
#pragma unroll
                        for (int j = 0; j < 3; ++j) p2B[3 * i + j] = hb ? Y[3 * j + i] : Y[3 * i + j];
                    p2p[0] = pav.x; p2p[1] = pav.y; p2p[2] = pav.z;
                }
                if (!(CH2 || (TG_PROBE & 2)) || (CH2 && d_store(dc))) {
#pragma unroll
                    for (int k = 0; k < 6; ++k) s(ia_c(g) + 15 * hh + k) = X[k];
                    if (!hb) {
#pragma unroll
                        for (int k = 0; k < 9; ++k) s(ia_c(g) + 6 + k) = Y[k];
                    }
                    stv3(s, pa_c(g) + 3 * hh, pav);
                }
            }
            // (chain schedule: a sync where the next step gathers another chain's
            // head, and after the last step -- the root gathers its children)
            if constexpr (!CH2 || TG_CHAIN_SYNC || t == 0) TG_SYNC();
            else if constexpr (step_gathers<M>(t - 1)) TG_SYNC();
        });
        } else {
        // unrolled (round 2: Gogoro 8.27e7 -> 8.36e7, GogoroPaper 8.55e7 -> 8.64e7, A/B twice)
        // (the children's descriptor read one step ahead, ahead of the step's own loads)
        I4 dnext = dsc(M::NSTEP - 1);
        static_for<0, M::NSTEP>([&](auto TT) {
            constexpr int t = M::NSTEP - 1 - decltype(TT)::value;
            const I4 dc = dnext;   // (children for the gather)
            if constexpr (t > 0) dnext = dsc(t - 1);
            const I4 pc = pdsc2(t);
            const int g = pc.x;
            if (g > 0) {
                const int o = g * GF;
                SI IA = ldsi(s, o + F_IA);
                SV pA = ldsv(s, o + F_PA);
                const SV Sg = ldSm<M>(s, g, d_jt(pc));
                const SV cb = ldsv(s, o + F_V);
                const float c0 = s(o + F_DINV), tau = s(o + F_UU), al = s(o + F_QDS), c1 = s(o + F_C1);
                constexpr int smax = step_smax<M>(t);
                if constexpr (smax >= 1) gather(IntC<(smax < 3 ? smax : 3)>{}, dc, IA, pA);
                const SV U = mul(IA, Sg);
                const float D0 = dot(Sg, U);   // without the armature (folded into c0, tau)
                const float Dinv = 1.0f / (c1 * D0 + c0);
                const float u = tau + al * D0 - dot(Sg, pA);
                SI Ia = IA;
                si_sub_outer(Ia, U, Dinv);
                const SV pa = pA + mul(Ia, cb) + (u * Dinv) * U;
                stsv(s, o + F_U, U);
                s(o + F_DINV) = Dinv;
                s(o + F_UU) = u;
                stsi(s, ia_c(g), Ia);     // contribution to the parent (same frame: no transform)
                stsv(s, pa_c(g), pa);
            }
            TG_SYNC();
        });
        }
        TG_PROF(18)
        // root: every lane factors the root articulated inertia itself
        {
            SI IA0 = ldsi(s, F_IA);
            SV pA0 = ldsv(s, F_PA);
            SI ci[M::nchild[0] > 0 ? M::nchild[0] : 1];
            SV cv[M::nchild[0] > 0 ? M::nchild[0] : 1];
#pragma unroll
            for (int c = 0; c < M::nchild[0]; ++c) {
                ci[c] = ldsi(s, ia_c(M::child[0][c]));
                cv[c] = ldsv(s, pa_c(M::child[0][c]));
            }
#pragma unroll
            for (int c = 0; c < M::nchild[0]; ++c) {
                si_add(IA0, ci[c]);
                pA0 = pA0 + cv[c];
            }
            if (!fix_base) {
                rootf = ldl6(IA0);
                a0 = ldl6_solve(rootf, -1.0f * pA0);
            }
        }
        TG_SYNC();
        TG_PROF(2)
        // ---- pass 3: free accelerations (through the F_PA slots) and velocities
        if (lead) {
            stsv(s, ac_s(0), a0);
            s(PL::FLG) = 0.f;
        }
        TG_SYNC();
        {
        // fully unrolled; a step's own-group inputs (written by passes 2a/2b,
        // untouched by the earlier steps) are loaded one step ahead, so only
        // the parent's acceleration is waited on along the chain
        struct Own { SV cb, U, S; float qd, uu, dinv, te, K, eff; };
        auto ld_own = [&](const I4 &dc) {
            const int g = max(dc.x, 0), o = g * GF;
            return Own{ldsv(s, o + F_V), ldsv(s, o + F_U), ldSm<M>(s, g, d_jt(dc)),
                       s(o + F_QD), s(o + F_UU), s(o + F_DINV),
                       s(o + F_CL), s(o + F_CL + 1), s(o + F_CL + 2)};
        };
        I4 dr[2];
        Own ow[2];
        SV pr3 = a0;
        (void)pr3;
        dr[0] = pdsc3(0);
        ow[0] = ld_own(dr[0]);
#pragma unroll
        for (int t = 0; t < M::NSTEP; ++t) {
            const I4 dc = dr[t % 2];
            const Own &w = ow[t % 2];
            const int g = dc.x;
            // (chain schedule: the parent's acceleration is the lane's previous step's)
            constexpr bool CH3 = (Chain<M>::ON && (TG_CHAIN_MASK & 4)) || (TG_PROBE & 4);
            SV apar;
            if constexpr (CH3) apar = pr3;
            else apar = ldsv(s, ac_s(max(dc.y, 0)));
            if (t + 1 < M::NSTEP) {
                dr[(t + 1) % 2] = pdsc3(t + 1);
                ow[(t + 1) % 2] = ld_own(dr[(t + 1) % 2]);
            }
            if (g > 0) {
                const int o = g * GF;
                const SV ap = apar + w.cb;   // cb: pass 2a
                const float qdd = (w.uu - dot(w.U, ap)) * w.dinv;
                if constexpr (CH3) pr3 = ap + qdd * w.S;
                else stsv(s, ac_s(g), ap + qdd * w.S);
                if (!CH3 || d_own(dc)) {   // (chain: the group's owner stores it)
                    s(o + F_QDS) = w.qd + h * qdd;
                    if (cp == 0) {
                        s(o + F_UU) = qdd;
                        const float ti = w.te - w.K * qdd;
                        const bool sat = w.K >= 0.f && fabsf(ti) > w.eff;
                        if (sat) s(PL::FLG) = 1.f;
                        // (Woodbury: the drive's clamp side, F_C1 being dead after pass 2b)
                        if constexpr (PL::WOOD) s(o + F_C1) = sat ? (ti > 0.f ? 1.f : -1.f) : 0.f;
                    }
                }
            }
            if constexpr (!(Chain<M>::ON && (TG_CHAIN_MASK & 4)) || TG_CHAIN_SYNC) TG_SYNC();
        }
        if constexpr (Chain<M>::ON && (TG_CHAIN_MASK & 4) && !TG_CHAIN_SYNC) TG_SYNC();   // (the flag and F_QDS are read below)
        }
        if constexpr (PL::WOOD) {
            if (cp == 0 && s(PL::FLG) != 0.f && wood_update()) break;   // else the rerun below
        }
        if (cp == 0 && s(PL::FLG) == 0.f) break;
        }   // clamp pass
        SV v0s = v0 + h * a0;
        v0s.v = v0s.v + h * cross(v0.w, v0.v);
        if (fix_base) v0s = sv0();
        TG_PROF(3)

        // ---- contacts
        SV v0v = v0s;   // the stored root velocity (bias-free with velocity iterations)
        if constexpr (M::NS > 0) {
            // velocity iterations (sim.physx.num_velocity_iterations): the
            // positions integrate the biased sweeps' velocity (F_QDS, v0s),
            // the stored velocity is the bias-free one (F_QD, v0v).  TGS
            // (solver_type 1): the position iterations are sub-steps of
            // h / iters, the positions integrate the mean of their
            // multipliers, the stored velocity the last (or the velocity
            // iterations'); either way two multiplier sets (vit)
            const bool tgs = a.tgs != 0;
            const bool vit = a.viters > 0 || tgs;
            // contact-group world poses and free velocities (one lane per contact group)
            for (int c = sub; c < M::NCG; c += LPE) {
                // the group and its path (groups, joint types) selected from the
                // model's constant tables (no table load before the LDS reads),
                // every path term's LDS reads issued at once
                int cg = M::cgroup[0], lk = M::cpath_len[0], pk[M::MAXD], pj[M::MAXD];
#pragma unroll
                for (int i = 0; i < M::MAXD; ++i) {
                    pk[i] = M::cpath[0][i] > 0 ? M::cpath[0][i] : 0;
                    pj[i] = M::jtype[pk[i]];
                }
#pragma unroll
                for (int cc = 1; cc < M::NCG; ++cc) {
                    const bool on = c == cc;
                    cg = on ? M::cgroup[cc] : cg;
                    lk = on ? M::cpath_len[cc] : lk;
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i) {
                        const int gk = M::cpath[cc][i] > 0 ? M::cpath[cc][i] : 0;
                        pk[i] = on ? gk : pk[i];
                        pj[i] = on ? M::jtype[gk] : pj[i];
                    }
                }
                stm3(s, PL::CGP + 12 * c, mul(R, ldR(s, cg)));
                // (the position relative to the root origin, world-oriented: the
                // contact points and lever arms below never form world
                // coordinates, whose fp32 rounding at env origins ~100 m from
                // the world origin was 1.5e-5 m -- a lever-arm error that the
                // speculative contact bound amplified)
                stv3(s, PL::CGP + 12 * c + 9, mul(R, ldv3(s, cg * GF + F_P)));
                // root frame, at the contact group's own origin pc (round 6, see
                // at_group_origin): the root velocity shifted to pc plus the
                // path's joint terms, each about its own joint point
                const V3 pc = ldv3(s, cg * GF + F_P);
                float qv[M::MAXD];
                V3 ax[M::MAXD], Pj[M::MAXD];
#pragma unroll
                for (int i = 0; i < M::MAXD; ++i) {
                    qv[i] = i < lk ? s(pk[i] * GF + F_QDS) : 0.f;
                    ax[i] = ldv3(s, pk[i] * GF + F_AX);
                    Pj[i] = ldv3(s, pk[i] * GF + F_P);
                }
                SV v = shift_to(v0s, pc);
#pragma unroll
                for (int i = 0; i < M::MAXD; ++i) v = v + qv[i] * motion_at<M>(pj[i], ax[i], Pj[i], pc);
                stsv(s, PL::CGV + 6 * c, v);
            }
            TG_SYNC();
            if constexpr (ROWPAR) {
            // contact rows, one lane per ROW (K <= LPE): the lane forms its
            // row's shape geometry itself -- support points, separations,
            // patch centroid: the operations of the one-lane-per-shape form
            // below, in the same order, so every row is bit-identical -- and
            // stores only its own row.  The rows' Jacobians and stores then
            // spread over the env's lanes instead of running serially on one
            // lane per shape (a wave instruction costs its full width however
            // few lanes are active)
            if (sub < K) {
                const int i = sub;
                const int sh = row_shape_sel<M>(i);
                int cgi = M::shape_cg[0];   // (selected from the constant table, no load)
#pragma unroll
                for (int k = 1; k < M::NS; ++k) cgi = sh == k ? M::shape_cg[k] : cgi;
                const int kr = i - row_base<M>(sh);   // the row within its shape
                const M3 Rwg = ldm3(s, PL::CGP + 12 * cgi);
                const V3 pwg = ldv3(s, PL::CGP + 12 * cgi + 9);
                M3 Rsl;
                V3 cl;
                if constexpr (SHP1) {   // (the row's shape: loaded at kernel start)
#pragma unroll
                    for (int k = 0; k < 9; ++k) Rsl.a[k] = shp1[k];
                    cl = v3(shp1[9], shp1[10], shp1[11]);
                } else {
#pragma unroll
                    for (int k = 0; k < 9; ++k) Rsl.a[k] = CP(CL::shape(sh) + k);
                    cl = v3(CP(CL::shape(sh) + 9), CP(CL::shape(sh) + 10), CP(CL::shape(sh) + 11));
                }
                const M3 Rs = mul(Rwg, Rsl);
                const V3 cw = mul(Rwg, cl);   // (points about the contact group's origin pwg, world-oriented)
                V3 pts[4];
                const int nr = M::shape_nrows[sh];
                const int kind = M::shape_kind[sh];
                V3 n = v3(0, 0, 1);
                float gmu = a.ground_mu;
                auto support = [&](V3 nn) __attribute__((always_inline)) {
                    if (kind == TG_SHAPE_TORUS) {
                        const V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                        V3 dd = nn - dot(ax, nn) * ax;
                        float nd = sqrtf(dot(dd, dd));
                        if (nd < 1e-6f) { dd = v3(1, 0, 0); nd = 1.f; }
                        pts[0] = cw - (M::shape_params[sh][0] / nd) * dd - M::shape_params[sh][1] * nn;
                    } else if (kind == TG_SHAPE_SPHERE) {
                        pts[0] = cw - M::shape_params[sh][0] * nn;
                    } else {
                        const float hx = M::shape_params[sh][0], hy = M::shape_params[sh][1], hz = M::shape_params[sh][2];
                        const V3 ex = v3(Rs.a[0], Rs.a[3], Rs.a[6]), ey = v3(Rs.a[1], Rs.a[4], Rs.a[7]),
                                 ez = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                        const float zx = dot(ex, nn), zy = dot(ey, nn), zz = dot(ez, nn);
                        const float ax_ = fabsf(zx), ay_ = fabsf(zy), az_ = fabsf(zz);
                        V3 fn, u1, u2;
                        if (az_ >= ax_ && az_ >= ay_) { fn = (zz > 0 ? -hz : hz) * ez; u1 = hx * ex; u2 = hy * ey; }
                        else if (ay_ >= ax_) { fn = (zy > 0 ? -hy : hy) * ey; u1 = hx * ex; u2 = hz * ez; }
                        else { fn = (zx > 0 ? -hx : hx) * ex; u1 = hy * ey; u2 = hz * ez; }
                        pts[0] = cw + fn - u1 - u2;
                        pts[1] = cw + fn + u1 - u2;
                        pts[2] = cw + fn - u1 + u2;
                        pts[3] = cw + fn + u1 + u2;
                    }
                };
                if constexpr (HF) {
                    bool th;
                    ground_at(a, pos.x + (pwg.x + cw.x), pos.y + (pwg.y + cw.y), n, th);
                    support(n);
                    ground_at(a, pos.x + (pwg.x + pts[0].x), pos.y + (pwg.y + pts[0].y), n, th);
                    if (th) gmu = a.hf_mu;
                }
                support(n);
                const V3 dl = mulT(R, n);   // root frame
                V3 cen = v3(0, 0, 0), cen0 = v3(0, 0, 0), pk = pts[0];
                float wk[4], wsum = 0.f, phk = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= nr) continue;
                    // (pts: about the contact group's origin, world-oriented)
                    float phi = pos.z + (pwg.z + pts[k].z);
                    if constexpr (HF) {
                        V3 nk;
                        bool th;
                        const float gz = ground_at(a, pos.x + (pwg.x + pts[k].x), pos.y + (pwg.y + pts[k].y), nk, th);
                        phi = (pos.z + (pwg.z + pts[k].z) - gz) * nk.z;
                    }
                    phk = k == kr ? phi : phk;
                    // (component-wise: a select of whole V3s becomes a pointer
                    // select over the array, which then stays in scratch)
                    pk.x = k == kr ? pts[k].x : pk.x;
                    pk.y = k == kr ? pts[k].y : pk.y;
                    pk.z = k == kr ? pts[k].z : pk.z;
                    wk[k] = fminf(fmaxf((a.margin - phi) / a.margin, 0.f), 1.f);
                    wsum += wk[k];
                    cen = cen + wk[k] * pts[k];
                    cen0 = cen0 + pts[k];
                }
                const int ro = PL::ROW + i * 8;
                if (kr < nr) {   // normal row kr: Jacobian about the contact group's origin, separation
                    const SV J = SV{cross(mulT(R, pk), dl), dl};
                    stsv(s, ro, J);
                    // (contact_offset: no row beyond the pair's contact distance)
                    const float phr = contact_row_phi(a, phk);
                    s(ro + 6) = a.tgs ? phr : contact_target(a, phr, h);
                    s(ro + 7) = 1.f;
                } else {         // friction row t of the patch
                    const int t = kr - nr;
                    cen = wsum > 0.f ? (1.f / wsum) * cen : (1.f / nr) * cen0;
                    if (t == 0) {
                        float re = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (k >= nr) continue;
                            const V3 d = pts[k] - cen;
                            const V3 dt = d - dot(d, n) * n;   // in the contact plane
                            re += (wsum > 0.f ? wk[k] / wsum : 1.f / nr) * sqrtf(dot(dt, dt));
                        }
                        s(PL::SHP + 2 * sh) = 0.5f * ((SHP1 ? smu1 : a.shape_mu[(size_t)e * M::NS + sh]) + gmu);
                        s(PL::SHP + 2 * sh + 1) = re;
                    }
                    V3 t1 = v3(1, 0, 0);
                    {
                        const V3 x = kind == TG_SHAPE_TORUS ? cross(v3(Rs.a[2], Rs.a[5], Rs.a[8]), n)
                                                            : v3(1, 0, 0) - n.x * n;
                        const float nx = sqrtf(dot(x, x));
                        if (nx > 1e-6f) t1 = (1.f / nx) * x;
                    }
                    const V3 t2 = cross(n, t1);
                    const V3 rl = mulT(R, cen);
                    const V3 dt = mulT(R, t == 0 ? t1 : (t == 1 ? t2 : n));
                    stsv(s, ro, t == 2 ? SV{dt, v3(0, 0, 0)} : SV{cross(rl, dt), dt});   // torsion row: angular
                    s(ro + 6) = 0.f;
                    s(ro + 7) = 1.f;
                }
            }
            } else {
            // contact rows (one lane per shape)
            for (int sh = sub; sh < M::NS; sh += LPE) {
                int cgi = M::shape_cg[0];   // (selected from the constant table, no load)
#pragma unroll
                for (int k = 1; k < M::NS; ++k) cgi = sh == k ? M::shape_cg[k] : cgi;
                const int rb = row_base<M>(sh);
                const M3 Rwg = ldm3(s, PL::CGP + 12 * cgi);
                const V3 pwg = ldv3(s, PL::CGP + 12 * cgi + 9);
                M3 Rsl;
                V3 cl;
                if constexpr (SHP1) {   // (sh == sub: loaded at kernel start)
#pragma unroll
                    for (int k = 0; k < 9; ++k) Rsl.a[k] = shp1[k];
                    cl = v3(shp1[9], shp1[10], shp1[11]);
                } else {
#pragma unroll
                    for (int k = 0; k < 9; ++k) Rsl.a[k] = CP(CL::shape(sh) + k);
                    cl = v3(CP(CL::shape(sh) + 9), CP(CL::shape(sh) + 10), CP(CL::shape(sh) + 11));
                }
                const M3 Rs = mul(Rwg, Rsl);
                const V3 cw = mul(Rwg, cl);   // (points about the contact group's origin pwg, world-oriented)
                V3 pts[4];
                const int nr = M::shape_nrows[sh];
                const int kind = M::shape_kind[sh];
                // patch normal n: the ground normal under the shape's support
                // point (found from the normal under its centre, then refined
                // once); e_z on the plane
                V3 n = v3(0, 0, 1);
                float gmu = a.ground_mu;
                auto support = [&](V3 nn) {
                    if (kind == TG_SHAPE_TORUS) {
                        const V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                        V3 dd = nn - dot(ax, nn) * ax;
                        float nd = sqrtf(dot(dd, dd));
                        if (nd < 1e-6f) { dd = v3(1, 0, 0); nd = 1.f; }
                        pts[0] = cw - (M::shape_params[sh][0] / nd) * dd - M::shape_params[sh][1] * nn;
                    } else if (kind == TG_SHAPE_SPHERE) {
                        pts[0] = cw - M::shape_params[sh][0] * nn;
                    } else {
                        // the 4 corners of the face whose outward normal points most against nn
                        const float hx = M::shape_params[sh][0], hy = M::shape_params[sh][1], hz = M::shape_params[sh][2];
                        const V3 ex = v3(Rs.a[0], Rs.a[3], Rs.a[6]), ey = v3(Rs.a[1], Rs.a[4], Rs.a[7]),
                                 ez = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                        const float zx = dot(ex, nn), zy = dot(ey, nn), zz = dot(ez, nn);
                        const float ax_ = fabsf(zx), ay_ = fabsf(zy), az_ = fabsf(zz);
                        V3 fn, u1, u2;
                        if (az_ >= ax_ && az_ >= ay_) { fn = (zz > 0 ? -hz : hz) * ez; u1 = hx * ex; u2 = hy * ey; }
                        else if (ay_ >= ax_) { fn = (zy > 0 ? -hy : hy) * ey; u1 = hx * ex; u2 = hz * ez; }
                        else { fn = (zx > 0 ? -hx : hx) * ex; u1 = hy * ey; u2 = hz * ez; }
                        pts[0] = cw + fn - u1 - u2;
                        pts[1] = cw + fn + u1 - u2;
                        pts[2] = cw + fn - u1 + u2;
                        pts[3] = cw + fn + u1 + u2;
                    }
                };
                if constexpr (HF) {
                    bool th;
                    ground_at(a, pos.x + (pwg.x + cw.x), pos.y + (pwg.y + cw.y), n, th);
                    support(n);
                    ground_at(a, pos.x + (pwg.x + pts[0].x), pos.y + (pwg.y + pts[0].y), n, th);
                    if (th) gmu = a.hf_mu;
                }
                support(n);
                // every point carries a speculative normal row along n; the friction
                // patch is anchored at the centroid weighted by clamp((margin-phi)/margin)
                const V3 dl = mulT(R, n);   // root frame
                V3 cen = v3(0, 0, 0), cen0 = v3(0, 0, 0);
                float wk[4], wsum = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= nr) break;
                    const int ro = PL::ROW + (rb + k) * 8;
                    // (pts: about the contact group's origin, world-oriented)
                    float phi = pos.z + (pwg.z + pts[k].z);
                    if constexpr (HF) {   // separation along the normal of the point's own triangle
                        V3 nk;
                        bool th;
                        const float gz = ground_at(a, pos.x + (pwg.x + pts[k].x), pos.y + (pwg.y + pts[k].y), nk, th);
                        phi = (pos.z + (pwg.z + pts[k].z) - gz) * nk.z;
                    }
                    // row Jacobian in the root frame: (r x d, d), r = the point about the contact group's origin
                    const SV J = SV{cross(mulT(R, pts[k]), dl), dl};
                    stsv(s, ro, J);
                    // (TGS: the separation itself, the PGS forms the sub-step targets;
                    // contact_offset: no row beyond the pair's contact distance)
                    const float phr = contact_row_phi(a, phi);
                    s(ro + 6) = a.tgs ? phr : contact_target(a, phr, h);
                    s(ro + 7) = 1.f;
                    wk[k] = fminf(fmaxf((a.margin - phi) / a.margin, 0.f), 1.f);
                    wsum += wk[k];
                    cen = cen + wk[k] * pts[k];
                    cen0 = cen0 + pts[k];
                }
                cen = wsum > 0.f ? (1.f / wsum) * cen : (1.f / nr) * cen0;
                float re = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= nr) break;
                    const V3 d = pts[k] - cen;
                    const V3 dt = d - dot(d, n) * n;   // in the contact plane
                    re += (wsum > 0.f ? wk[k] / wsum : 1.f / nr) * sqrtf(dot(dt, dt));
                }
                s(PL::SHP + 2 * sh) = 0.5f * ((SHP1 ? smu1 : a.shape_mu[(size_t)e * M::NS + sh]) + gmu);
                s(PL::SHP + 2 * sh + 1) = re;
                // tangents: rolling direction (axis x n) for tori, else world x in the plane
                V3 t1 = v3(1, 0, 0);
                {
                    const V3 x = kind == TG_SHAPE_TORUS ? cross(v3(Rs.a[2], Rs.a[5], Rs.a[8]), n)
                                                        : v3(1, 0, 0) - n.x * n;
                    const float nx = sqrtf(dot(x, x));
                    if (nx > 1e-6f) t1 = (1.f / nx) * x;
                }
                const V3 t2 = cross(n, t1);
                const V3 rl = mulT(R, cen);
                const float fon = 1.f;
                const int nf = nr == 1 ? 2 : 3;   // (shape_nfric: no torsion row for a one-point patch)
                for (int t = 0; t < nf; ++t) {
                    const int ro = PL::ROW + (rb + nr + t) * 8;
                    const V3 dt = mulT(R, t == 0 ? t1 : (t == 1 ? t2 : n));
                    stsv(s, ro, t == 2 ? SV{dt, v3(0, 0, 0)} : SV{cross(rl, dt), dt});   // torsion row: angular
                    s(ro + 6) = 0.f;
                    s(ro + 7) = fon;
                }
            }
            }   // ROWPAR
            TG_SYNC();
            // row i: root-frame Jacobian J_i (6) about its contact group's origin
            // pc -> velocity J_i . v (v about pc), impulse about the root origin
            // lam (J.w + pc x J.v, J.v)
            auto rvel = [&](int i, const SV &vg) { return dot(ldsv(s, PL::ROW + i * 8), vg); };
            auto rforce = [&](int i, float lam) {
                const SV J = ldsv(s, PL::ROW + i * 8);
                const V3 pc = ldv3(s, row_group<M>(i) * GF + F_P);
                return lam * SV{J.w + cross(pc, J.v), J.v};
            };
            for (int i = sub; i < K; i += LPE) {
                s(PL::VFREE + i) = rvel(i, ldsv(s, PL::CGV + 6 * row_cg<M>(i)));
                s(PL::LAM + i) = 0.f;
            }
            TG_PROF(4)
            // Delassus columns, one per lane: unit row impulse on contact group k,
            // up-walk along k's path (du in registers), root solve, down-walk
            // along every contact group's path
#pragma unroll 1
            for (int j = sub; j < K; j += LPE) {
                const int ck = row_cg<M>(j);
                // the path of contact group ck (groups, joint types) selected from
                // the model's constant tables: no LDS round trip before the walk
                int lk = M::cpath_len[0], pk[M::MAXD], pj[M::MAXD];
#pragma unroll
                for (int i = 0; i < M::MAXD; ++i) {
                    pk[i] = M::cpath[0][i];
                    pj[i] = M::jtype[M::cpath[0][i] > 0 ? M::cpath[0][i] : 0];
                }
#pragma unroll
                for (int c = 1; c < M::NCG; ++c) {
                    const bool on = ck == c;
                    lk = on ? M::cpath_len[c] : lk;
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i) {
                        pk[i] = on ? M::cpath[c][i] : pk[i];
                        pj[i] = on ? M::jtype[M::cpath[c][i] > 0 ? M::cpath[c][i] : 0] : pj[i];
                    }
                }
                SV p = -1.0f * rforce(j, 1.0f);
                // the contact group's own joint (its axis through pc): S . J_root
                // = a . J.w exactly (revolute), a . J.v (prismatic) -- not a sum of
                // two ~|pc|-sized terms
                float uo;
                {
                    const SV Jl = ldsv(s, PL::ROW + j * 8);
                    const int go = row_group<M>(j);
                    const V3 axo = ldv3(s, go * GF + F_AX);
                    bool rev = true;
                    if constexpr (!all_revolute<M>()) {
#pragma unroll
                        for (int g = 1; g < M::NG; ++g) rev = go == g ? M::jtype[g] == TG_JOINT_REVOLUTE : rev;
                    }
                    uo = rev ? dot(axo, Jl.w) : dot(axo, Jl.v);
                }
                float du[M::MAXD];
#pragma unroll
                for (int i = M::MAXD - 1; i >= 0; --i) {
                    du[i] = 0.f;
                    if (i < lk) {
                        const int g = pk[i];
                        const float u = i == lk - 1 ? uo : -dot(ldSm<M>(s, g, pj[i]), p);
                        du[i] = u;
                        p = p + (u * s(g * GF + F_DINV)) * ldsv(s, g * GF + F_U);
                    }
                }
                const SV aj = fix_base ? sv0() : ldl6_solve(rootf, -1.0f * p);
                if constexpr (SUPER) {
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i)
                        if (i < lk) s(swa(j, i)) = du[i];
                    const float av[6] = {aj.w.x, aj.w.y, aj.w.z, aj.v.x, aj.v.y, aj.v.z};
#pragma unroll
                    for (int k = 0; k < 6; ++k) s(swa(j, M::MAXD + k)) = av[k];
                }
                if constexpr (M::NG <= 8) {
                    // small trees: the ABA's x from the walk about the root
                    // origin as before, the response about pcc accumulated
                    // beside it (A/B round 6: the form below cost the scooter
                    // +1.6 us, this one +0.3)
                    SV dvc[M::NCG];
#pragma unroll
                    for (int c = 0; c < M::NCG; ++c) {
                        SV av = aj;
                        const V3 pcc = ldv3(s, M::cgroup[c] * GF + F_P);
                        SV al = shift_to(aj, pcc);
#pragma unroll
                        for (int i = 0; i < M::MAXD; ++i) {
                            if (i < M::cpath_len[c]) {
                                const int hg = M::cpath[c][i];
                                const float dui = (i < lk && pk[i] == hg) ? du[i] : 0.0f;
                                const float x = (dui - dot(ldsv(s, hg * GF + F_U), av)) * s(hg * GF + F_DINV);
                                const V3 axh = ldv3(s, hg * GF + F_AX), Ph = ldv3(s, hg * GF + F_P);
                                av = av + x * motion_Sm<M>(M::jtype[hg], axh, Ph);
                                al = al + x * motion_at<M>(M::jtype[hg], axh, Ph, pcc);
                            }
                        }
                        dvc[c] = al;
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) s(PL::W + i * K + j) = rvel(i, dvc[M::shape_cg[row_shape<M>(i)]]);
                } else {
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) {
                    // large trees: one accumulator, the walk carried about the
                    // contact group's origin pcc (two per path cost the humanoid
                    // 60 more registers, spilled): U . a is invariant, so each U
                    // moves to pcc with it (moment - pcc x force)
                    const V3 pcc = ldv3(s, M::cgroup[c] * GF + F_P);
                    SV al = shift_to(aj, pcc);
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i) {
                        if (i < M::cpath_len[c]) {
                            const int hg = M::cpath[c][i];
                            const float dui = (i < lk && pk[i] == hg) ? du[i] : 0.0f;
                            const SV Uh = ldsv(s, hg * GF + F_U);
                            const float x = (dui - dot(SV{Uh.w - cross(pcc, Uh.v), Uh.v}, al)) * s(hg * GF + F_DINV);
                            al = al + x * motion_at<M>(M::jtype[hg], ldv3(s, hg * GF + F_AX), ldv3(s, hg * GF + F_P), pcc);
                        }
                    }
                    // column j's entries of the rows on contact group c (no
                    // per-group response array held across the groups)
#pragma unroll
                    for (int i = 0; i < K; ++i)
                        if (M::shape_cg[row_shape<M>(i)] == c) s(PL::W + i * K + j) = rvel(i, al);
                }
                }
                // a row with no response (W_jj ~ 0: a shape on a fixed base, a
                // normal row through a fixed-base scooter's wheel) gets a huge
                // diagonal, so the sweeps give it a multiplier ~1e-30 times its
                // target -- no impulse -- instead of 1/0 and then inf * 0 = NaN
                // (the oracle's OVERW gives it exactly 0).  Off the sweeps'
                // register peak: a guard there cost 1-5 %.
                if (!(s(PL::W + j * K + j) > TG_W_DEAD)) s(PL::W + j * K + j) = 1e30f;
            }
            TG_SYNC();
            if constexpr (PL::WOOD) {
                if (wn > 0) {
                    // clamped drives (Woodbury): W' = W + (J G) M^-1 (J G)^T, J G =
                    // each row's velocity response to the drives' unit torques
                    for (int j = sub; j < K; j += LPE) {
#pragma unroll
                        for (int i = 0; i < PL::WCM; ++i)
                            s(PL::WB_J + K * i + j) =
                                i < wn ? rvel(j, ldsv(s, PL::WB_A + 6 * (M::NCG * i + row_cg<M>(j)))) : 0.f;
                    }
                    TG_SYNC();
                    for (int j = sub; j < K; j += LPE) {
                        float t[PL::WCM];
#pragma unroll
                        for (int i = 0; i < PL::WCM; ++i) {
                            float x = 0.f;
#pragma unroll
                            for (int k = 0; k < PL::WCM; ++k) x += s(PL::WB_M + PL::WCM * i + k) * s(PL::WB_J + K * k + j);
                            t[i] = x;
                        }
#pragma unroll
                        for (int r = 0; r < K; ++r) {
                            float x = s(PL::W + r * K + j);
#pragma unroll
                            for (int i = 0; i < PL::WCM; ++i) x += s(PL::WB_J + K * i + r) * t[i];
                            s(PL::W + r * K + j) = x;
                        }
                    }
                    TG_SYNC();
                }
            }
            TG_PROF(5)
#ifdef TG_DUMP_ENV
            if (e == tg_dump_env && owner && lead && sub_i == tg_dump_sub) {
                tg_dump_buf[0] = (float)K;
                for (int i = 0; i < K * K; ++i) tg_dump_buf[16 + i] = s(PL::W + i);
                for (int i = 0; i < K; ++i) tg_dump_buf[2000 + i] = s(PL::VFREE + i);
                for (int i = 0; i < K * 8; ++i) tg_dump_buf[2100 + i] = s(PL::ROW + i);
                for (int k = 0; k < 6; ++k) tg_dump_buf[2700 + k] = k < 3 ? (&a0.w.x)[k] : (&a0.v.x)[k - 3];
                for (int g = 1; g < M::NG; ++g) tg_dump_buf[2800 + M::gdof[g]] = s(g * GF + F_UU);   // (no rerun: qdd)
                tg_dump_buf[2790] = s(PL::FLG);
                for (int k = 0; k < 6; ++k) tg_dump_buf[2710 + k] = k < 3 ? (&v0.w.x)[k] : (&v0.v.x)[k - 3];
            }
            TG_SYNC();
#endif
            if constexpr (!SUPER) {   // impulse accumulators (F_PA slots) cleared by all lanes
                for (int g = sub; g < M::NG; g += LPE) stsv(s, g * GF + F_PA, sv0());
                TG_SYNC();
            }
            if constexpr (LPE == 16) {
            // projected Gauss-Seidel with patch friction, all LPE lanes of the env:
            // lane sub owns rows k = sub + LPE*jj -- its W rows and its entries of
            // the row velocities r = vfree + W lambda, kept current incrementally
            // (a multiplier change d adds W[k][c] d, one FMA per lane); a row's
            // velocity reaches every lane of the env by one DPP row broadcast,
            // and every lane computes the same update (the full multiplier
            // vector in registers, no LDS traffic in the sweeps)
            // (instantiated per solver: the PGS build carries none of the TGS
            // state -- one more live array in this section cost the walk 1 us)
            auto pgs16 = [&](auto TC) {
                constexpr bool T = decltype(TC)::value != 0;
                constexpr int JL = (K + LPE - 1) / LPE;
                constexpr int JT = T ? JL : 1, KT = T ? K : 1;
                // (the lane's own rows: W rows, velocities, targets; TGS: their
                // separations and displacements)
                // PGS: every lane holds every row's target (tg), as before TGS;
                // TGS: the owner lane holds its rows' moving targets (tgo)
                float wr[JL][K], rv[JL], tgo[JT], tg[T ? 1 : K], phio[JT], dsp[JT], rvs[JT], wd[K], lam[K], lbar[KT];
                bool nrm[JT];
                const float hs = T ? h / (float)a.iters : h;   // (TGS sub-step)
#pragma unroll
                for (int jj = 0; jj < JL; ++jj) {
                    const int k = sub + LPE * jj;
#pragma unroll
                    for (int c = 0; c < K; ++c) wr[jj][c] = k < K ? s(PL::W + k * K + c) : 0.f;
                    rv[jj] = k < K ? s(PL::VFREE + k) : 0.f;
                    if constexpr (T) {   // slot 6: the separation (TGS; 0 on friction rows)
                        const float t6 = k < K ? s(PL::ROW + k * 8 + 6) : 0.f;
                        nrm[jj] = k < K && row_normal<M>(k);
                        phio[jj] = t6;
                        dsp[jj] = 0.f;
                        rvs[jj] = 0.f;
                        tgo[jj] = nrm[jj] ? contact_target(a, t6, hs) : t6;
                    }
                }
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    if constexpr (!T) tg[i] = s(PL::ROW + i * 8 + 6);   // the target (0 on friction rows)
                    wd[i] = 1.0f / s(PL::W + i * K + i);   // (the inverse diagonal, formed once)
                    lam[i] = 0.f;
                    if constexpr (T) lbar[i] = 0.f;
                }
                // the shapes' patch friction and torsion radius, in registers for
                // all the sweeps (read from LDS inside the sweep, each was a
                // round trip on the Gauss-Seidel chain)
                float smu[M::NS], sre[M::NS];
#pragma unroll
                for (int sh = 0; sh < M::NS; ++sh) {
                    smu[sh] = s(PL::SHP + 2 * sh);
                    sre[sh] = s(PL::SHP + 2 * sh + 1);
                }
                // row i's velocity vfree_i + (W lambda)_i, from its owner lane
                auto row_v = [&](int i) { return env_bcast<LPE>(rv[i / LPE], i % LPE, sub); };
                // a normal row's target (TGS: the owner's moving target, broadcast
                // off the Gauss-Seidel chain: it changes once per sweep)
                auto row_t = [&](int i) {
                    if constexpr (T) return env_bcast<LPE>(tgo[i / LPE], i % LPE, sub);
                    else return tg[i];
                };
                auto set_lam = [&](int i, float v) {
                    const float d = v - lam[i];
                    lam[i] = v;
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) rv[jj] += wr[jj][i] * d;
                };
#ifdef TG_PGS_REFRESH   // developer build (drift study): row velocities re-formed at every sweep
                float vfr[JL];
#pragma unroll
                for (int jj = 0; jj < JL; ++jj) vfr[jj] = rv[jj];
#endif
                auto sweeps = [&](int n_it, auto SUBC) {
#pragma unroll 1
                for (int it = 0; it < n_it; ++it) {
#ifdef TG_PGS_REFRESH
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) {
                        float r = vfr[jj];
#pragma unroll
                        for (int c = 0; c < K; ++c) r += wr[jj][c] * lam[c];
                        rv[jj] = r;
                    }
#endif
#pragma unroll
                    for (int sh = 0; sh < M::NS; ++sh) {
                        const int rb = row_base<M>(sh), nr = M::shape_nrows[sh];
                        float Nsum = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (k >= nr) break;
                            const int i = rb + k;
                            // lam + (target - v) / W_ii with the target term formed
                            // first: one dependent FMA after the row velocity
                            // arrives (every row slot 7, the on flag, is 1)
                            const float ci = lam[i] + row_t(i) * wd[i];
                            const float li = fmaxf(ci - row_v(i) * wd[i], 0.f);
                            set_lam(i, li);
                            Nsum += li;
                        }
                        const int f = rb + nr;
                        const float mu = smu[sh], reff = sre[sh];
                        // tangent 1, then tangent 2 with the cone projection of the
                        // pair, then the torsional row clamped (friction targets 0)
                        set_lam(f, lam[f] - row_v(f) * wd[f]);
                        {
                            // the cone scale lim / |l| by one reciprocal square root
                            // (|l| > lim >= 0 makes |l|^2 > 0)
                            const float l0 = lam[f], l1 = lam[f + 1] - row_v(f + 1) * wd[f + 1];
                            const float n2 = l0 * l0 + l1 * l1, lim = mu * Nsum;
                            const float sc = n2 > lim * lim ? lim * rsqrtf(n2) : 1.f;
                            set_lam(f, l0 * sc);
                            set_lam(f + 1, l1 * sc);
                        }
                        if (shape_nfric<M>(sh) == 3) {   // torsion (several-point patches)
                            const float lim3 = mu * Nsum * reff;
                            set_lam(f + 2, fminf(fmaxf(lam[f + 2] - row_v(f + 2) * wd[f + 2], -lim3), lim3));
                        }
                    }
                    if constexpr (T && decltype(SUBC)::value != 0) {
                        // TGS: each normal row advances by hs times its velocity after
                        // the sweep, its next target is re-formed from that
                        // separation; the multipliers accumulate for their mean
#pragma unroll
                        for (int jj = 0; jj < JL; ++jj) {
                            rvs[jj] += rv[jj];   // (the row velocity of the mean multipliers, rv being affine in them)
                            dsp[jj] += hs * rv[jj];
                            tgo[jj] = nrm[jj] ? contact_target(a, phio[jj] + dsp[jj], hs) : tgo[jj];
                        }
#pragma unroll
                        for (int i = 0; i < K; ++i) lbar[i] += lam[i];
                    }
                }
                };
                sweeps(a.iters, IntC<1>{});   // position iterations: push-out bias in the normal targets
                if (vit) {
                    // two multiplier sets: the positions' (the biased multipliers,
                    // TGS their mean over the sub-steps) park in the dead Delassus
                    // slots (W is in registers now); the velocity iterations lose
                    // the push-out (min(target, 0)) and continue from the last sweep
                    if (lead) {
                        const float inv = 1.0f / (float)(a.iters > 0 ? a.iters : 1);
#pragma unroll
                        for (int i = 0; i < K; ++i) {
                            if constexpr (T) s(PL::W + i) = lbar[i] * inv;
                            else s(PL::W + i) = lam[i];
                        }
                    }
                    if constexpr (T) {
                        // TGS: a normal row's bias-free target is re-formed from its
                        // final separation over the whole substep h, not the sub-step
                        // hs, and the velocity iterations start from the sub-steps'
                        // mean multipliers, not the last sub-step's: the velocity
                        // stored here is the one the next substep starts from, and
                        // either sub-step form gave it a gain of N/h on a contact's
                        // residual gap (DESIGN.md §2 "TGS conditioning")
                        // (no velocity iterations: the last sub-step's velocity is stored)
                        const float inv = 1.0f / (float)a.iters;
                        const bool mean = a.viters > 0;
#pragma unroll
                        for (int jj = 0; jj < JL; ++jj) {
                            tgo[jj] = nrm[jj] ? fminf(-(phio[jj] + dsp[jj] - a.rest) / h, 0.f) : fminf(tgo[jj], 0.f);
                            rv[jj] = mean ? rvs[jj] * inv : rv[jj];
                        }
#pragma unroll
                        for (int i = 0; i < K; ++i) lam[i] = mean ? lbar[i] * inv : lam[i];
                    } else {
#pragma unroll
                        for (int i = 0; i < K; ++i) tg[i] = fminf(tg[i], 0.f);
                    }
                    if (a.viters > 0) sweeps(a.viters, IntC<0>{});
                }
                if (lead) {
#pragma unroll
                    for (int i = 0; i < K; ++i) s(PL::LAM + i) = lam[i];
                }
            };
            if (tgs) pgs16(IntC<1>{});
            else pgs16(IntC<0>{});
            } else {   // 8-lane envs: the row velocity by an 8-lane reduction (two broadcasts
                       // and a select measured slower than the three DPP levels; W and the
                       // row velocities in every lane, kept incrementally as for 16 lanes:
                       // Gogoro +2.7 %, GogoroPaper +10 %, round 3)
            // projected Gauss-Seidel with patch friction, all LPE lanes of the env:
            // each lane holds W's columns j = sub + LPE*jj and the full multiplier
            // vector in registers; a row's W*lambda is an 8-lane reduction, so
            // every lane computes the same update (no LDS traffic in the sweeps)
            {
                constexpr int JL = (K + LPE - 1) / LPE;
                float wc[K][JL], vf[K], tg[K], onr[K], wd[K], lam[K], my[JL], phi[K], dsp[K], lbar[K];
                const float hs = tgs ? h / (float)a.iters : h;   // (TGS sub-step)
#pragma unroll
                for (int i = 0; i < K; ++i) {
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) {
                        const int j = sub + LPE * jj;
                        wc[i][jj] = j < K ? s(PL::W + i * K + j) : 0.f;
                    }
                    vf[i] = s(PL::VFREE + i);
                    phi[i] = s(PL::ROW + i * 8 + 6);   // the target (PGS) or the separation (TGS)
                    dsp[i] = 0.f;
                    lbar[i] = 0.f;
                    tg[i] = (tgs && row_normal<M>(i)) ? contact_target(a, phi[i], hs) : phi[i];
                    onr[i] = s(PL::ROW + i * 8 + 7);
                    wd[i] = inv_diag(s(PL::W + i * K + i));   // (the inverse diagonal, formed once)
                    lam[i] = 0.f;
                }
#pragma unroll
                for (int jj = 0; jj < JL; ++jj) my[jj] = 0.f;
                // the shapes' patch friction and torsion radius, in registers for
                // all the sweeps (read from LDS inside the sweep, each was a
                // round trip on the Gauss-Seidel chain)
                float smu[M::NS], sre[M::NS];
#pragma unroll
                for (int sh = 0; sh < M::NS; ++sh) {
                    smu[sh] = s(PL::SHP + 2 * sh);
                    sre[sh] = s(PL::SHP + 2 * sh + 1);
                }
                auto row_v = [&](int i) {   // vfree_i + (W lambda)_i
                    float part = 0.f;
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) part += wc[i][jj] * my[jj];
                    return vf[i] + sum_lanes<LPE>(part);
                };
                auto set_lam = [&](int i, float v) {
                    lam[i] = v;
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj)
                        if (sub + LPE * jj == i) my[jj] = v;
                };
                auto sweeps = [&](int n_it, bool sub_steps) {
#pragma unroll 1
                for (int it = 0; it < n_it; ++it) {
#pragma unroll
                    for (int sh = 0; sh < M::NS; ++sh) {
                        const int rb = row_base<M>(sh), nr = M::shape_nrows[sh];
                        float Nsum = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (k >= nr) break;
                            const int i = rb + k;
                            const float vi = row_v(i);
                            const float l = lam[i] + (tg[i] - vi) * wd[i];
                            const float li = onr[i] * fmaxf(l, 0.f);
                            set_lam(i, li);
                            Nsum += li;
                        }
                        const int f = rb + nr;
                        const float mu = smu[sh], reff = sre[sh];
#pragma unroll
                        for (int t = 0; t < shape_nfric<M>(sh); ++t) {
                            const int i = f + t;
                            const float vi = row_v(i);
                            set_lam(i, lam[i] - vi * wd[i]);
                            if (t == 1) {
                                const float l0 = lam[f], l1 = lam[f + 1];
                                const float lt = sqrtf(l0 * l0 + l1 * l1), lim = mu * Nsum;
                                const float sc = lt > lim ? (lt > 0.f ? lim / lt : 0.f) : 1.f;
                                set_lam(f, l0 * sc);
                                set_lam(f + 1, l1 * sc);
                            }
                        }
                        if (shape_nfric<M>(sh) == 3) {
                            const float lim3 = mu * Nsum * reff;
                            set_lam(f + 2, fminf(fmaxf(lam[f + 2], -lim3), lim3));
                        }
                    }
                    if (sub_steps) {   // TGS (as the 16-lane sweeps)
#pragma unroll
                        for (int i = 0; i < K; ++i) {
                            if (row_normal<M>(i)) {
                                dsp[i] += hs * row_v(i);
                                tg[i] = contact_target(a, phi[i] + dsp[i], hs);
                            }
                            lbar[i] += lam[i];
                        }
                    }
                }
                };
                sweeps(a.iters, tgs);   // position iterations (biased), then the bias-free velocity iterations
                if (vit) {
                    if (lead) {   // the positions' multipliers (TGS: the sub-steps' mean)
                        const float inv = 1.0f / (float)(a.iters > 0 ? a.iters : 1);
#pragma unroll
                        for (int i = 0; i < K; ++i) s(PL::W + i) = tgs ? lbar[i] * inv : lam[i];
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) {   // (TGS: over h, from the mean multipliers, as the 16-lane sweeps)
                        tg[i] = (tgs && row_normal<M>(i)) ? fminf(-(phi[i] + dsp[i] - a.rest) / h, 0.f)
                                                          : fminf(tg[i], 0.f);
                        if (tgs && a.viters > 0) set_lam(i, lbar[i] * (1.0f / (float)a.iters));
                    }
                    if (a.viters > 0) sweeps(a.viters, false);
                }
                if (lead) {
#pragma unroll
                    for (int i = 0; i < K; ++i) s(PL::LAM + i) = lam[i];
                }
            }
            }
            TG_SYNC();
#ifdef TG_DUMP_ENV
            if (e == tg_dump_env && owner && lead && sub_i == tg_dump_sub) {
                for (int i = 0; i < K; ++i) {
                    tg_dump_buf[2500 + i] = s(PL::LAM + i);                 // stored-velocity multipliers
                    tg_dump_buf[2600 + i] = vit ? s(PL::W + i) : s(PL::LAM + i);   // the positions'
                }
            }
            TG_SYNC();
#endif
            SV da0 = sv0(), da0v = sv0();
            if constexpr (SUPER) {
                TG_PROF(6)
                // joint impulses u_g = sum_j lam_j du_j on the contact paths (0 elsewhere),
                // one contact group at a time (paths may share ancestors); with
                // velocity iterations also u_v (F_C1, dead after pass 2b) from
                // the bias-free multipliers, the biased ones parked at PL::W
                const int LP = vit ? PL::W : PL::LAM;
                for (int g = sub; g < M::NG; g += LPE) {
                    s(g * GF + F_UU) = 0.f;
                    if (vit) s(g * GF + F_C1) = 0.f;
                }
                TG_SYNC();
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) {
                    for (int i = sub; i < M::cpath_len[c]; i += LPE) {
                        float acc = 0.f, accv = 0.f;
#pragma unroll
                        for (int j = 0; j < K; ++j)
                            if (M::shape_cg[row_shape<M>(j)] == c) {
                                const float du = s(swa(j, i));
                                acc += s(LP + j) * du;
                                accv += s(PL::LAM + j) * du;
                            }
                        const int o = bounded(cpath[c * M::MAXD + i], -1, M::NG) * GF;
                        s(o + F_UU) += acc;
                        if (vit) s(o + F_C1) += accv;
                    }
                    TG_SYNC();
                }
                if (!fix_base) {
                    // (every lane forms the root response from all columns:
                    // broadcast LDS reads; an LPE-lane DPP sum of per-column
                    // terms measured slower, ThormangWalk 55.5 -> 56.9 us)
                    float d6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const float l = s(LP + j), lv = s(PL::LAM + j);
#pragma unroll
                        for (int k = 0; k < 6; ++k) {
                            const float aj = s(swa(j, M::MAXD + k));
                            d6[k] += l * aj;
                            v6[k] += lv * aj;
                        }
                    }
                    da0 = SV{v3(d6[0], d6[1], d6[2]), v3(d6[3], d6[4], d6[5])};
                    da0v = SV{v3(v6[0], v6[1], v6[2]), v3(v6[3], v6[4], v6[5])};
                }
                TG_SYNC();
                if (lead) {
                    stsv(s, F_PA, da0);
                    stsv(s, F_V, da0v);   // (the root's F_V: dead after pass 1)
                }
                TG_SYNC();
                // top-down, fully unrolled, own-group inputs one step ahead (as in
                // pass 3); with velocity iterations the bias-free response rides
                // along (F_V accelerations, F_QD the stored velocity)
                struct OwnI { SV U, S; float uu, uv, dinv, qds; };
                auto ld_own = [&](const I4 &dc) {
                    const int g = max(dc.x, 0), o = g * GF;
                    return OwnI{ldsv(s, o + F_U), ldSm<M>(s, g, d_jt(dc)), s(o + F_UU), s(o + F_C1), s(o + F_DINV),
                                s(o + F_QDS)};
                };
                I4 dr[2];
                OwnI ow[2];
                SV pri = da0, priv = da0v;
                (void)pri; (void)priv;
                dr[0] = pdsc4(0);
                ow[0] = ld_own(dr[0]);
#pragma unroll
                for (int t = 0; t < M::NSTEP; ++t) {
                    const I4 dc = dr[t % 2];
                    const OwnI &w = ow[t % 2];
                    const int g = dc.x;
                    const int op = max(dc.y, 0) * GF;
                    // (chain schedule: the parent's responses are the lane's previous step's)
                    constexpr bool CHI = (Chain<M>::ON && (TG_CHAIN_MASK & 8)) || (TG_PROBE & 8);
                    SV ap, av;
                    if constexpr (CHI) {
                        ap = pri;
                        av = priv;
                        (void)op;
                    } else {
                        ap = ldsv(s, op + F_PA);
                        av = vit ? ldsv(s, op + F_V) : sv0();
                    }
                    if (t + 1 < M::NSTEP) {
                        dr[(t + 1) % 2] = pdsc4(t + 1);
                        ow[(t + 1) % 2] = ld_own(dr[(t + 1) % 2]);
                    }
                    if (g > 0) {
                        const int o = g * GF;
                        const float x = (w.uu - dot(w.U, ap)) * w.dinv;
                        if constexpr (CHI) {
                            pri = ap + x * w.S;
                        }
                        if constexpr (!CHI) stsv(s, o + F_PA, ap + x * w.S);
                        // (every lane of the group stores, duplicates too: the same
                        // value, and the same contraction as the list form's)
                        s(o + F_QDS) = w.qds + x;
                        if (vit) {
                            const float xv = (w.uv - dot(w.U, av)) * w.dinv;
                            if constexpr (CHI) {
                                priv = av + xv * w.S;
                            }
                            if constexpr (!CHI) stsv(s, o + F_V, av + xv * w.S);
                            s(o + F_QD) = w.qds + xv;
                        }
                    }
                    if constexpr (!(Chain<M>::ON && (TG_CHAIN_MASK & 8)) || TG_CHAIN_SYNC) TG_SYNC();
                }
                if constexpr (Chain<M>::ON && (TG_CHAIN_MASK & 8) && !TG_CHAIN_SYNC) TG_SYNC();
            } else {
                // bottom-up gather, root solve, top-down -- once per multiplier
                // set: with velocity iterations first the bias-free one (its
                // joint velocities to F_QD, F_QDS untouched), then the biased one
                for (int pass = vit ? 0 : 1; pass < 2; ++pass) {
                    const int LS = (pass == 1 && vit) ? PL::W : PL::LAM;
                    if (pass == 1 && vit) {   // the accumulators again
                        for (int g = sub; g < M::NG; g += LPE) stsv(s, g * GF + F_PA, sv0());
                        TG_SYNC();
                    }
                    if (lead) {
                        // impulses into the contact groups' F_PA slots (p = -f convention)
                        for (int i = 0; i < K; ++i) {
                            const int g = M::shape_group[row_shape<M>(i)];
                            stsv(s, g * GF + F_PA, ldsv(s, g * GF + F_PA) + (-1.0f) * rforce(i, s(LS + i)));
                        }
                    }
                    TG_SYNC();
                    TG_PROF(6)
#pragma unroll 1
                    for (int t = M::NSTEP - 1; t >= 0; --t) {
                        const I4 dc = dsc(t);
                        const int g = dc.x;
                        if (g > 0) {
                            const int o = g * GF;
                            SV p = ldsv(s, o + F_PA);
                            for (int c = 0; c < d_nch(dc); ++c) p = p + ldsv(s, d_child(dc, c) * GF + F_PA);
                            const float u = -dot(ldSm<M>(s, g, d_jt(dc)), p);
                            s(o + F_UU) = u;
                            stsv(s, o + F_PA, p + (u * s(o + F_DINV)) * ldsv(s, o + F_U));
                        }
                        TG_SYNC();
                    }
                    SV p0 = ldsv(s, F_PA);
                    for (int c = 0; c < M::nchild[0]; ++c) p0 = p0 + ldsv(s, M::child[0][c] * GF + F_PA);
                    SV d0 = sv0();
                    if (!fix_base) d0 = ldl6_solve(rootf, -1.0f * p0);
                    TG_SYNC();
                    if (lead) stsv(s, F_PA, d0);
                    TG_SYNC();
#pragma unroll 1
                    for (int t = 0; t < M::NSTEP; ++t) {
                        const I4 dc = dsc(t);
                        const int g = dc.x;
                        const SV ap = ldsv(s, max(dc.y, 0) * GF + F_PA);
                        if (g > 0) {
                            const int o = g * GF;
                            const float x = (s(o + F_UU) - dot(ldsv(s, o + F_U), ap)) * s(o + F_DINV);
                            stsv(s, o + F_PA, ap + x * ldSm<M>(s, g, d_jt(dc)));
                            s(o + (pass == 0 ? F_QD : F_QDS)) = s(o + F_QDS) + x;
                        }
                        TG_SYNC();
                    }
                    if (pass == 0) da0v = d0;
                    else da0 = d0;
                }
            }
            if constexpr (PL::WOOD) {
                if (wn > 0) {
                    // clamped drives (Woodbury): the impulse response A'^-1 J^T lam =
                    // A^-1 J^T lam (above) + G M^-1 (J G)^T lam, for both multiplier sets
                    const int LPW = vit ? PL::W : PL::LAM;
                    float jl[PL::WCM], jlv[PL::WCM];
#pragma unroll
                    for (int i = 0; i < PL::WCM; ++i) {
                        float x = 0.f, xv = 0.f;
#pragma unroll
                        for (int r = 0; r < K; ++r) {
                            const float jg = s(PL::WB_J + K * i + r);
                            x += jg * s(LPW + r);
                            xv += jg * s(PL::LAM + r);
                        }
                        jl[i] = x;
                        jlv[i] = xv;
                    }
                    float y[PL::WCM], yv[PL::WCM];
#pragma unroll
                    for (int i = 0; i < PL::WCM; ++i) {
                        float x = 0.f, xv = 0.f;
#pragma unroll
                        for (int k = 0; k < PL::WCM; ++k) {
                            const float mi = s(PL::WB_M + PL::WCM * i + k);
                            x += mi * jl[k];
                            xv += mi * jlv[k];
                        }
                        y[i] = x;
                        yv[i] = xv;
                    }
                    const int gl = 1 + sub;
                    if (gl < M::NG) {
                        float dq = 0.f, dqv = 0.f;
#pragma unroll
                        for (int i = 0; i < PL::WCM; ++i) {
                            const float gi = s(PL::WB_G + 8 * i + gl);
                            dq += gi * y[i];
                            dqv += gi * yv[i];
                        }
                        s(gl * GF + F_QDS) += dq;
                        if (vit) s(gl * GF + F_QD) += dqv;
                    }
#pragma unroll
                    for (int i = 0; i < PL::WCM; ++i) {
                        const SV ri = ldsv(s, PL::WB_R + 6 * i);
                        da0 = da0 + y[i] * ri;
                        da0v = da0v + yv[i] * ri;
                    }
                }
            }
            if (!fix_base) {
                v0v = v0s + (vit ? da0v : da0);
                v0s = v0s + da0;
            }
            TG_PROF(7)
        }
        // ---- velocity limits + integration: the positions with the biased
        // sweeps' velocity (F_QDS, v0s), the stored velocity the bias-free one
        // (F_QD, v0v) when velocity iterations ran
        const bool vst = M::NS > 0 && (a.viters > 0 || a.tgs);
#pragma unroll
        for (int r = 0; r < NRX; ++r) {
            const int g = 1 + sub + r * LPE;
            if (g >= M::NG) break;
            const int o = g * GF;
            const float vl = vlim[r];
            float x = s(o + F_QDS), xv = vst ? s(o + F_QD) : x;
            if (vl > 0.f) {
                x = fminf(fmaxf(x, -vl), vl);
                xv = fminf(fmaxf(xv, -vl), vl);
            }
            s(o + F_QD) = xv;
            s(o + F_Q) += h * x;
        }
        if (!fix_base) {
            v0 = v0s;
            pos = pos + h * mul(R, v0.v);
            const float wn = sqrtf(dot(v0.w, v0.w));
            const float an = wn * h;
            float dx = 0.f, dy = 0.f, dz = 0.f, dw = 1.f;
            if (an > 1e-12f) {
                float sa, ca;
                // the libm half-angle sine / cosine, not the hardware v_sin / v_cos
                // (__sincosf): at these small angles the approximation's absolute
                // error is a large relative error in the orientation increment,
                // the largest GPU-specific term of the Gogoro drift study
                // (profiles/r3/drift_gogoro.txt); once per substep
#ifdef TG_FAST_QUAT   // developer build: the hardware approximation (drift study control)
                __sincosf(0.5f * an, &sa, &ca);
#else
                sincosf(0.5f * an, &sa, &ca);
#endif
                const float kk = sa / wn;
                dx = v0.w.x * kk; dy = v0.w.y * kk; dz = v0.w.z * kk; dw = ca;
            }
            v0 = v0v;
            const float nx = qw * dx + qx * dw + qy * dz - qz * dy;
            const float ny = qw * dy - qx * dz + qy * dw + qz * dx;
            const float nz = qw * dz + qx * dy - qy * dx + qz * dw;
            const float nw = qw * dw - qx * dx - qy * dy - qz * dz;
            const float in = rsqrtf(nx * nx + ny * ny + nz * nz + nw * nw);
            qx = nx * in; qy = ny * in; qz = nz * in; qw = nw * in;
            R = quat_to_m3(qx, qy, qz, qw);
            const M3 Rd = quat_to_m3(dx, dy, dz, dw);
            v0.w = mulT(Rd, v0.w);
            v0.v = mulT(Rd, v0.v);
        }
        TG_SYNC();
        TG_PROF(8)
    }
    if constexpr (EPI_TOUCH) __asm__ volatile("" ::"v"(epi_touch));   // (keeps the touch load)
    if constexpr (P::on) {
        // final root state in the world frame (every lane of the env holds it)
        const V3 wwo = mul(R, v0.w);
        const V3 vco = mul(R, v0.v) + cross(wwo, mul(R, c0));
        const float rt[13] = {pos.x, pos.y, pos.z, qx, qy, qz, qw, vco.x, vco.y, vco.z, wwo.x, wwo.y, wwo.z};
        P::template epilogue<M, LPE>(pa, a, s, e, owner, sub, rt, root, dofs, xpre);
    } else if (owner) {
        if (lead) {
            const V3 wwo = mul(R, v0.w);
            const V3 vco = mul(R, v0.v) + cross(wwo, mul(R, c0));
            root[0] = pos.x; root[1] = pos.y; root[2] = pos.z;
            root[3] = qx; root[4] = qy; root[5] = qz; root[6] = qw;
            root[7] = vco.x; root[8] = vco.y; root[9] = vco.z;
            root[10] = wwo.x; root[11] = wwo.y; root[12] = wwo.z;
        }
        for (int g = 1 + sub; g < M::NG; g += LPE) {
            const int d = bounded(gi[g * GIW + GI_DOF], 0, 1 << 16);
            dofs[2 * d] = s(g * GF + F_Q);
            dofs[2 * d + 1] = s(g * GF + F_QD);
        }
        for (int d = sub; d < M::ND; d += LPE) {
            if (M::dof_locked[d]) {
                dofs[2 * d] = 0.5f * (PR(TG_PROP_LOWER, d) + PR(TG_PROP_UPPER, d));
                dofs[2 * d + 1] = 0.f;
            }
        }
    }
    TG_PROF(9)
    TG_PROF_FLUSH
}

#undef TG_SYNC

}  // namespace tg
