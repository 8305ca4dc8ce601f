// step_par.h -- tree-parallel, LDS-resident articulation step (included by
// articulation.hip after the shared helpers; the algorithm of
// oracle/physics_ref.c, operation for operation per group).
//
// Layout: EPB envs per workgroup, LPE lanes per env (LPE consecutive lanes of
// one wavefront).  Each env's articulated state (per group: X, v, I^A, p^A, U,
// D^-1, u, q, qd, qds, gravity-in-frame) lives in LDS at
// lds[env * ES + group * GF + field] with 16-byte aligned field blocks.  At 16 envs x 2370 floats the
// Thormang block uses 148 KB of the 160 KB LDS of a CU; 4096 envs = 256
// workgroups = one per CU.
//
// Parallelism inside an env: model/codegen.py list-schedules the non-root
// groups onto the LPE lanes (M::sched[step][lane], parents at earlier steps).
//   pass 1 (kinematics, velocities, bias)      -- schedule forward
//   pass 2 (articulated inertias)               -- schedule backward; a group
//          gathers its children's contributions (each child leaves
//          X^T I^a X and X^T p^a in its own I^A / p^A slots), so lanes never
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
__device__ unsigned long long tg_prof_acc[16];
#define TG_PROF_INIT unsigned long long tg_t0 = clock64();
#define TG_PROF(k)                                                              \
    {                                                                           \
        const unsigned long long t1 = clock64();                               \
        if (threadIdx.x == 0) atomicAdd(&tg_prof_acc[k], t1 - tg_t0);           \
        tg_t0 = t1;                                                             \
    }
#else
#define TG_PROF_INIT
#define TG_PROF(k)
#endif

// one env's LDS state
struct LE {
    float *b;
    __device__ __forceinline__ float &operator()(int i) const { return b[i]; }
};

// per-group field offsets (GF floats per group)
// (16-byte aligned blocks: X = E,r [0,12), v [12,18), I^A [20,41), p^A [44,50),
// so the compiler can move them with ds_read/write_b128)
enum : int {
    F_E = 0, F_R = 9, F_V = 12, F_Q = 18, F_QD = 19, F_IA = 20, F_DINV = 41, F_UU = 42, F_QDS = 43, F_PA = 44,
    F_U = 50, F_GL = 56, GF = 60
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
__device__ __forceinline__ Xf ldx(const LE &s, int g) { return Xf{ldm3(s, g * GF + F_E), ldv3(s, g * GF + F_R)}; }

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
    static constexpr int CGP = SHP + 2 * M::NSA;     // per contact group: world R (9), p (3)
    static constexpr int CGV = CGP + 12 * M::NCG;    // per contact group: free velocity (6)
    static constexpr int FLG = CGV + 6 * M::NCG;     // a drive exceeded its effort limit
    // per-block ints after the env area
    static constexpr int T_GI = 0;
    static constexpr int T_SCHED = M::NG * GIW;
    static constexpr int T_CPATH = T_SCHED + M::NSTEP * M::LPE;   // [NCG][MAXD]
    static constexpr int T_TOTAL = T_CPATH + M::NCG * M::MAXD;
    // SEPC (when the LDS has room): pass 2 writes each group's contribution to
    // its parent (I^a 21 at +0, p^a 6 at +24) and pass 3 its acceleration (+0)
    // into a separate 32-float block, so pass 1's rigid inertias and bias
    // forces survive and the drive-clamp rerun starts at pass 2
    static constexpr int CB = (FLG + 1 + 3) & ~3;
    static constexpr bool SEPC = ((size_t)M::EPB * (CB + 32 * M::NG) + T_TOTAL) * 4 <= 160 * 1024;
    static constexpr int TOTAL = SEPC ? CB + 32 * M::NG : FLG + 1;
    static constexpr int ES = (TOTAL + 3) & ~3;      // env stride (16-byte aligned)
    template <int EPB> static constexpr size_t bytes() { return ((size_t)EPB * ES + T_TOTAL) * 4; }
};

// Group frames are joint-aligned (model/codegen.py gq, applied by
// compose_kernel): every motion subspace is S = (e_z, 0) (revolute) or
// (0, e_z) (prismatic), so S-products are component selects.
struct GInfo {
    int parent, dof, jt;
};

template <class M> __device__ __forceinline__ GInfo ginfo(const int *gi, int g) {
    const int *p = gi + g * ParLayout<M>::GIW;
    return GInfo{p[GI_PARENT], p[GI_DOF], p[GI_JT]};
}

__device__ __forceinline__ float dotS(int jt, const SV &x) { return jt == TG_JOINT_REVOLUTE ? x.w.z : x.v.z; }
__device__ __forceinline__ SV addS(int jt, SV x, float a) {   // x + a S
    if (jt == TG_JOINT_REVOLUTE) x.w.z += a;
    else x.v.z += a;
    return x;
}
__device__ __forceinline__ SV colS(int jt, const SI &I) {   // I S
    return jt == TG_JOINT_REVOLUTE ? SV{v3(I.A[4], I.A[5], I.A[2]), v3(I.B[6], I.B[7], I.B[8])}
                                   : SV{v3(I.B[2], I.B[5], I.B[8]), v3(I.C[4], I.C[5], I.C[2])};
}
__device__ __forceinline__ SV crmS(int jt, const SV &v, float qd) {   // v x (qd S)
    const V3 wz = v3(v.w.y * qd, -v.w.x * qd, 0.f);
    return jt == TG_JOINT_REVOLUTE ? SV{wz, v3(v.v.y * qd, -v.v.x * qd, 0.f)} : SV{v3(0, 0, 0), wz};
}

// world pose of group g by walking up to the root: R_g = R_0 E_a1^T ... E_g^T
__device__ __forceinline__ void world_pose(const LE &s, const int *gi, int giw, int g, const M3 &R0, V3 p0, M3 &Rg,
                                           V3 &pg) {
    M3 Mr = eye3();
    V3 t = v3(0, 0, 0);
    while (g > 0) {
        const M3 Et = transpose(ldm3(s, g * GF + F_E));
        t = ldv3(s, g * GF + F_R) + mul(Et, t);
        Mr = mul(Et, Mr);
        g = gi[g * giw + GI_PARENT];
    }
    Rg = mul(R0, Mr);
    pg = p0 + mul(R0, t);
}

// The LPE lanes of an env are consecutive lanes of one wavefront, whose LDS
// operations execute in program order: an env-level "barrier" only has to stop
// the compiler from moving LDS accesses across it (no s_barrier, and no
// s_waitcnt on the prefetched global loads still in flight).
// sum over the 8 lanes of an env with DPP moves (row half-mirror, then quad
// swaps): every lane ends with the total, no LDS round trip
template <int CTRL> __device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8(float v) {
    v += dpp<0x141>(v);   // row_half_mirror: lane i <-> 7 - i
    v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
    return v;
}

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

template <class M, int EPB, bool HF> __global__ __launch_bounds__(EPB * M::LPE) void step_par_kernel(StepArgs a) {
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
    constexpr bool SUPER = K > 0 && K * SW <= M::NG * 21;
    constexpr bool SEPC = PL::SEPC;
    auto ia_c = [](int g) { return SEPC ? PL::CB + 32 * g : g * GF + F_IA; };        // pass-2 contribution I^a
    auto pa_c = [](int g) { return SEPC ? PL::CB + 32 * g + 24 : g * GF + F_PA; };   // pass-2 contribution p^a
    auto ac_s = [](int g) { return SEPC ? PL::CB + 32 * g : g * GF + F_PA; };        // pass-3 acceleration
    extern __shared__ __attribute__((aligned(16))) float lds_raw[];
    int *tab = reinterpret_cast<int *>(lds_raw + EPB * PL::ES);
    const int *gi = tab + PL::T_GI;
    const int *sched = tab + PL::T_SCHED;
    const int *cpath = tab + PL::T_CPATH;
    const int tid = threadIdx.x;
    const int le = tid / LPE, sub = tid % LPE;
    // XCD-aware chunk order: workgroups are dispatched round-robin over the 8
    // XCDs, so workgroup b takes env chunk (b % 8) * (nb / 8) + b / 8 and each
    // XCD's L2 sees a contiguous env range (the [KC][N] composite cache rows
    // of neighbouring chunks share 128-B lines)
    const int nb = gridDim.x;
    const int chunk = (nb % 8 == 0) ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
    const int e = min(chunk * EPB + le, a.N - 1);   // tail lanes redo the last env, never store
    const bool owner = chunk * EPB + le < a.N;
    TG_PROF_INIT

    for (int i = tid; i < M::NG; i += EPB * LPE) {
        int *p = tab + PL::T_GI + i * GIW;
        p[GI_PARENT] = M::parent[i];
        p[GI_DOF] = M::gdof[i];
        p[GI_JT] = M::jtype[i];
        p[GI_NCH] = M::nchild[i];
        for (int c = 0; c < M::MAXC; ++c) p[GI_CH + c] = M::child[i][c];
    }
    for (int i = tid; i < M::NSTEP * LPE; i += EPB * LPE) tab[PL::T_SCHED + i] = M::sched[i / LPE][i % LPE];
    for (int i = tid; i < M::NCG * M::MAXD; i += EPB * LPE) tab[PL::T_CPATH + i] = M::cpath[i / M::MAXD][i % M::MAXD];

    const LE s{lds_raw + le * PL::ES};
    const size_t N = a.N;
    const int D = a.D;
    const float h = a.h;
    const bool fix_base = a.fix_base != 0;
    const float *comp = a.comp;
    auto CP = [&](int k) { return comp[(size_t)k * N + e]; };
    auto PR = [&](int f, int d) { return a.props[((size_t)f * N + e) * D + d]; };
    const bool lead = sub == 0;

    float *root = a.root + (size_t)e * 13;
    float *dofs = a.dof + (size_t)e * D * 2;
    __syncthreads();   // group tables (shared by both wavefronts)
    for (int g = 1 + sub; g < M::NG; g += LPE) {
        const int d = gi[g * GIW + GI_DOF];
        s(g * GF + F_Q) = dofs[2 * d];
        s(g * GF + F_QD) = dofs[2 * d + 1];
    }
    V3 pos = v3(root[0], root[1], root[2]);
    float qx = root[3], qy = root[4], qz = root[5], qw = root[6];
    {
        const float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
        qx *= in; qy *= in; qz *= in; qw *= in;
    }
    M3 R = quat_to_m3(qx, qy, qz, qw);
    const V3 c0 = v3(M::root_com[0], M::root_com[1], M::root_com[2]);
    const V3 ww = v3(root[10], root[11], root[12]);
    const V3 vo = v3(root[7], root[8], root[9]) - cross(ww, mul(R, c0));
    SV v0 = fix_base ? sv0() : SV{mulT(R, ww), mulT(R, vo)};
    const V3 grav = v3(a.gx, a.gy, a.gz);

    // rigid inertia + bias force of group g (pass 1 body), v and gl already known
    // cin: the group's composite inertia (m, c, Ic) from the per-env cache
    auto body_bias = [&](int g, const SV &vg, V3 gl, const float *cin) {
        const int o = g * GF;
        const float m = cin[0];
        const V3 cg = v3(cin[1], cin[2], cin[3]);
        float Ic[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) Ic[k] = cin[4 + k];
        const SI I = rb_inertia(m, cg, Ic);
        stsi(s, o + F_IA, I);
        const SV b = crf(vg, mul(I, vg));
        V3 F = m * gl;
        F = F - (a.lin_damp * m) * (vg.v + cross(vg.w, cg));
        V3 n = cross(cg, F) - a.ang_damp * symmul(Ic, vg.w);
        if (a.force) {
            const float *fw = a.force + ((size_t)e * M::NG + g) * 6;
            M3 Rw;
            V3 pw;
            world_pose(s, gi, GIW, g, R, pos, Rw, pw);
            const V3 fl = mulT(Rw, v3(fw[0], fw[1], fw[2])), tl = mulT(Rw, v3(fw[3], fw[4], fw[5]));
            F = F + fl;
            n = n + tl + cross(cg, fl);
        }
        stsv(s, o + F_PA, SV{b.w - n, b.v - F});
    };
    // per-group per-env inputs, prefetched one schedule step ahead
    auto load_kin = [&](int g, float *x) {   // joint placement (12) + inertia (10)
#pragma unroll
        for (int k = 0; k < 12; ++k) x[k] = CP(CL::xtree(g) + k);
#pragma unroll
        for (int k = 0; k < 10; ++k) x[12 + k] = CP(CL::inertia(g) + k);
    };
    auto load_drv = [&](int g, float *x) {   // drive / limit inputs of the group's dof
        const int d = gi[g * GIW + GI_DOF];
        x[0] = PR(TG_PROP_ARMATURE, d);
        x[1] = PR(TG_PROP_DRIVE_MODE, d);
        x[2] = PR(TG_PROP_STIFFNESS, d);
        x[3] = PR(TG_PROP_DAMPING, d);
        x[4] = PR(TG_PROP_EFFORT, d);
        x[5] = PR(TG_PROP_LOWER, d);
        x[6] = PR(TG_PROP_UPPER, d);
        x[7] = a.pos_tgt[(size_t)e * D + d];
        x[8] = a.vel_tgt[(size_t)e * D + d];
        x[9] = a.act ? a.act[(size_t)e * D + d] : 0.f;
    };
    float rin[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) rin[k] = CP(CL::inertia(0) + k);
    TG_SYNC();
    TG_PROF(0)

    for (int sub_i = 0; sub_i < a.substeps; ++sub_i) {
        // Passes 1-3 run with every position/velocity drive implicit and
        // unclamped; if some drive's implicit end-of-substep torque te - K*qdd
        // exceeds its effort, they run once more with those drives as the
        // explicit torque +-effort ("implicit, then clamp", as
        // oracle/physics_ref.c aba()).  Between the two runs the F_GL slots of
        // a drive group hold (te, K, effort) and F_UU holds qdd.
        LDL6 rootf{};
        SV a0 = sv0();
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
        // results are intact)
        int gn;
        if (!SEPC || cp == 0) {
        if (lead) {
            const V3 gl = mulT(R, grav);
            stsv(s, F_V, v0);
            stv3(s, F_GL, gl);
            body_bias(0, v0, gl, rin);
        }
        TG_SYNC();
        float nk[22];
        gn = sched[sub];
        if (gn > 0) load_kin(gn, nk);
#pragma unroll 1
        for (int t = 0; t < M::NSTEP; ++t) {
            const int g = gn;
            float ck[22];
#pragma unroll
            for (int k = 0; k < 22; ++k) ck[k] = nk[k];
            gn = t + 1 < M::NSTEP ? sched[(t + 1) * LPE + sub] : -1;
            if (gn > 0) load_kin(gn, nk);
            if (g > 0) {
                const int o = g * GF;
                const GInfo G = ginfo<M>(gi, g);
                M3 Rpc;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rpc.a[k] = ck[k];
                V3 tr = v3(ck[9], ck[10], ck[11]);
                const float qg = s(o + F_Q);
                if (G.jt == TG_JOINT_REVOLUTE) {   // Rpc * Rz(q)
                    float sq, cq;
                    __sincosf(qg, &sq, &cq);
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const float c0 = Rpc.a[3 * r], c1 = Rpc.a[3 * r + 1];
                        Rpc.a[3 * r] = c0 * cq + c1 * sq;
                        Rpc.a[3 * r + 1] = c1 * cq - c0 * sq;
                    }
                } else {
                    tr = tr + qg * v3(Rpc.a[2], Rpc.a[5], Rpc.a[8]);
                }
                const Xf X{transpose(Rpc), tr};
                stm3(s, o + F_E, X.E);
                stv3(s, o + F_R, tr);
                const SV vg = addS(G.jt, xmotion(X, ldsv(s, G.parent * GF + F_V)), s(o + F_QD));
                const V3 gl = mul(X.E, ldv3(s, G.parent * GF + F_GL));
                stsv(s, o + F_V, vg);
                stv3(s, o + F_GL, gl);
                body_bias(g, vg, gl, ck + 12);
            }
            TG_SYNC();
        }
        }   // pass 1
        TG_PROF(1)
        // ---- pass 2: schedule backward, children contributions gathered
        float nd[10];
        gn = sched[(M::NSTEP - 1) * LPE + sub];
        if (gn > 0) load_drv(gn, nd);
#pragma unroll 1
        for (int t = M::NSTEP - 1; t >= 0; --t) {
            const int g = gn;
            float cd[10];
#pragma unroll
            for (int k = 0; k < 10; ++k) cd[k] = nd[k];
            gn = t > 0 ? sched[(t - 1) * LPE + sub] : -1;
            if (gn > 0) load_drv(gn, nd);
            if (g > 0) {
                const int o = g * GF;
                const GInfo G = ginfo<M>(gi, g);
                SI IA = ldsi(s, o + F_IA);
                SV pA = ldsv(s, o + F_PA);
                const int nch = gi[g * GIW + GI_NCH];
                for (int c = 0; c < nch; ++c) {
                    const int ch = gi[g * GIW + GI_CH + c];
                    si_add(IA, ldsi(s, ia_c(ch)));
                    pA = pA + ldsv(s, pa_c(ch));
                }
                const SV U = colS(G.jt, IA);
                const float q = s(o + F_Q), qd = s(o + F_QD);
                const float D0 = dotS(G.jt, U) + cd[0];
                float Dimp = 0.f, tau = 0.f;
                const int mode = (int)rintf(cd[1]);
                const float kp = cd[2], kd = cd[3];
                const float eff = cd[4];
                if (mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL) {
                    const float te = kp * (cd[7] - q - h * qd) + kd * (cd[8] - qd);
                    const float K = h * kd + h * h * kp;
                    bool implicit = true;
                    if (cp == 0) {
                        s(o + F_GL) = te;
                        s(o + F_GL + 1) = K;
                        s(o + F_GL + 2) = eff;
                    } else {
                        const float ti = te - K * s(o + F_UU);   // F_UU: qdd of the first solve
                        if (fabsf(ti) > eff) {
                            implicit = false;
                            tau += ti > 0.f ? eff : -eff;
                        }
                    }
                    if (implicit) { tau += te; Dimp += K; }
                } else {
                    if (cp == 0) s(o + F_GL + 1) = -1.f;
                    if (mode == TG_DOF_MODE_EFFORT && a.act) tau += fminf(fmaxf(cd[9], -eff), eff);
                }
                const float lo = cd[5], hi = cd[6];
                const float qp = q + h * qd;
                const float kl = a.lim_k * D0 / (h * h), cl = a.lim_c * D0 / h;
                // limit spring + damping, damping/implicit terms ramped in past the limit
                if (qp < lo && lo > -1e30f) {
                    const float r = fminf((lo - qp) * (1.0f / TG_LIMIT_RAMP), 1.0f);
                    tau += kl * (lo - qp) - r * cl * qd;
                    Dimp += r * (h * cl + h * h * kl);
                } else if (qp > hi && hi < 1e30f) {
                    const float r = fminf((qp - hi) * (1.0f / TG_LIMIT_RAMP), 1.0f);
                    tau += kl * (hi - qp) - r * cl * qd;
                    Dimp += r * (h * cl + h * h * kl);
                }
                const float Dinv = 1.0f / (D0 + Dimp);
                const float u = tau - dotS(G.jt, pA);
                stsv(s, o + F_U, U);
                s(o + F_DINV) = Dinv;
                s(o + F_UU) = u;
                SI Ia = IA;
                si_sub_outer(Ia, U, Dinv);
                const SV cb = crmS(G.jt, ldsv(s, o + F_V), qd);
                const SV pa = pA + mul(Ia, cb) + (u * Dinv) * U;
                const Xf X = ldx(s, g);
                stsi(s, ia_c(g), si_to_parent(Ia, X));     // contribution to the parent
                stsv(s, pa_c(g), xTforce(X, pa));
            }
            TG_SYNC();
        }
        // root: every lane factors the root articulated inertia itself
        {
            SI IA0 = ldsi(s, F_IA);
            SV pA0 = ldsv(s, F_PA);
            for (int c = 0; c < M::nchild[0]; ++c) {
                si_add(IA0, ldsi(s, ia_c(M::child[0][c])));
                pA0 = pA0 + ldsv(s, pa_c(M::child[0][c]));
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
#pragma unroll 1
        for (int t = 0; t < M::NSTEP; ++t) {
            const int g = sched[t * LPE + sub];
            if (g > 0) {
                const int o = g * GF;
                const GInfo G = ginfo<M>(gi, g);
                const float qd = s(o + F_QD);
                const SV cb = crmS(G.jt, ldsv(s, o + F_V), qd);
                const SV ap = xmotion(ldx(s, g), ldsv(s, ac_s(G.parent))) + cb;
                const float qdd = (s(o + F_UU) - dot(ldsv(s, o + F_U), ap)) * s(o + F_DINV);
                stsv(s, ac_s(g), addS(G.jt, ap, qdd));
                s(o + F_QDS) = qd + h * qdd;
                if (cp == 0) {
                    s(o + F_UU) = qdd;
                    const float K = s(o + F_GL + 1);
                    if (K >= 0.f && fabsf(s(o + F_GL) - K * qdd) > s(o + F_GL + 2)) s(PL::FLG) = 1.f;
                }
            }
            TG_SYNC();
        }
        if (cp == 0 && s(PL::FLG) == 0.f) break;
        }   // clamp pass
        SV v0s = v0 + h * a0;
        v0s.v = v0s.v + h * cross(v0.w, v0.v);
        if (fix_base) v0s = sv0();
        TG_PROF(3)

        // ---- contacts
        if constexpr (M::NS > 0) {
            // contact-group world poses and free velocities (one lane per contact group)
            for (int c = sub; c < M::NCG; c += LPE) {
                M3 Rc;
                V3 pc;
                world_pose(s, gi, GIW, M::cgroup[c], R, pos, Rc, pc);
                stm3(s, PL::CGP + 12 * c, Rc);
                stv3(s, PL::CGP + 12 * c + 9, pc);
                SV v = v0s;
                for (int i = 0; i < M::cpath_len[c]; ++i) {
                    const int hg = cpath[c * M::MAXD + i];
                    v = addS(ginfo<M>(gi, hg).jt, xmotion(ldx(s, hg), v), s(hg * GF + F_QDS));
                }
                stsv(s, PL::CGV + 6 * c, v);
            }
            TG_SYNC();
            // contact rows (one lane per shape)
            for (int sh = sub; sh < M::NS; sh += LPE) {
                const int cgi = M::shape_cg[sh];
                const int rb = row_base<M>(sh);
                const M3 Rwg = ldm3(s, PL::CGP + 12 * cgi);
                const V3 pwg = ldv3(s, PL::CGP + 12 * cgi + 9);
                M3 Rsl;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rsl.a[k] = CP(CL::shape(sh) + k);
                const M3 Rs = mul(Rwg, Rsl);
                const V3 cl = v3(CP(CL::shape(sh) + 9), CP(CL::shape(sh) + 10), CP(CL::shape(sh) + 11));
                const V3 cw = pwg + mul(Rwg, cl);
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
                    ground_at(a, cw.x, cw.y, n, th);
                    support(n);
                    ground_at(a, pts[0].x, pts[0].y, n, th);
                    if (th) gmu = a.hf_mu;
                }
                support(n);
                // every point carries a speculative normal row along n; the friction
                // patch is anchored at the centroid weighted by clamp((margin-phi)/margin)
                const V3 dl = mulT(Rwg, n);
                V3 cen = v3(0, 0, 0), cen0 = v3(0, 0, 0);
                float wk[4], wsum = 0.f;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k >= nr) break;
                    const int ro = PL::ROW + (rb + k) * 8;
                    float phi = pts[k].z;
                    if constexpr (HF) {   // separation along the normal of the point's own triangle
                        V3 nk;
                        bool th;
                        const float gz = ground_at(a, pts[k].x, pts[k].y, nk, th);
                        phi = (pts[k].z - gz) * nk.z;
                    }
                    // row Jacobian in the group frame: (r x d, d), d = Rwg^T n
                    stsv(s, ro, SV{cross(mulT(Rwg, pts[k] - pwg), dl), dl});
                    s(ro + 6) = phi > a.rest ? -(phi - a.rest) / h : fminf(a.baumgarte * (a.rest - phi) / h, a.max_depen);
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
                s(PL::SHP + 2 * sh) = 0.5f * (a.shape_mu[(size_t)e * M::NS + sh] + gmu);
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
                const V3 rl = mulT(Rwg, cen - pwg);
                const float fon = 1.f;
                for (int t = 0; t < 3; ++t) {
                    const int ro = PL::ROW + (rb + nr + t) * 8;
                    const V3 dt = mulT(Rwg, t == 0 ? t1 : (t == 1 ? t2 : n));
                    stsv(s, ro, t == 2 ? SV{dt, v3(0, 0, 0)} : SV{cross(rl, dt), dt});   // torsion row: angular
                    s(ro + 6) = 0.f;
                    s(ro + 7) = fon;
                }
            }
            TG_SYNC();
            // row i: group-frame Jacobian J_i (6) -> velocity J_i . v, impulse lam J_i
            auto rvel = [&](int i, const SV &vg) { return dot(ldsv(s, PL::ROW + i * 8), vg); };
            auto rforce = [&](int i, float lam) { return lam * ldsv(s, PL::ROW + i * 8); };
            for (int i = sub; i < K; i += LPE) {
                s(PL::VFREE + i) = rvel(i, ldsv(s, PL::CGV + 6 * M::shape_cg[row_shape<M>(i)]));
                s(PL::LAM + i) = 0.f;
            }
            TG_PROF(4)
            // Delassus columns, one per lane: unit row impulse on contact group k,
            // up-walk along k's path (du in registers), root solve, down-walk
            // along every contact group's path
#pragma unroll 1
            for (int j = sub; j < K; j += LPE) {
                const int ck = M::shape_cg[row_shape<M>(j)];
                const int lk = M::cpath_len[ck];
                const int *pk = cpath + ck * M::MAXD;
                SV p = -1.0f * rforce(j, 1.0f);
                float du[M::MAXD];
#pragma unroll
                for (int i = M::MAXD - 1; i >= 0; --i) {
                    du[i] = 0.f;
                    if (i < lk) {
                        const int g = pk[i];
                        const float u = -dotS(ginfo<M>(gi, g).jt, p);
                        du[i] = u;
                        const SV pa = p + (u * s(g * GF + F_DINV)) * ldsv(s, g * GF + F_U);
                        p = xTforce(ldx(s, g), pa);
                    }
                }
                const SV aj = fix_base ? sv0() : ldl6_solve(rootf, -1.0f * p);
                if constexpr (SUPER) {
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i)
                        if (i < lk) s(scr(j * SW + i)) = du[i];
                    const float av[6] = {aj.w.x, aj.w.y, aj.w.z, aj.v.x, aj.v.y, aj.v.z};
#pragma unroll
                    for (int k = 0; k < 6; ++k) s(scr(j * SW + M::MAXD + k)) = av[k];
                }
                SV dvc[M::NCG];
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) {
                    SV av = aj;
#pragma unroll
                    for (int i = 0; i < M::MAXD; ++i) {
                        if (i < M::cpath_len[c]) {
                            const int hg = M::cpath[c][i];
                            const SV ap = xmotion(ldx(s, hg), av);
                            const float dui = (i < lk && pk[i] == hg) ? du[i] : 0.0f;
                            const float x = (dui - dot(ldsv(s, hg * GF + F_U), ap)) * s(hg * GF + F_DINV);
                            av = addS(M::jtype[hg], ap, x);
                        }
                    }
                    dvc[c] = av;
                }
#pragma unroll
                for (int i = 0; i < K; ++i) s(PL::W + i * K + j) = rvel(i, dvc[M::shape_cg[row_shape<M>(i)]]);
            }
            TG_SYNC();
            TG_PROF(5)
            if constexpr (!SUPER) {   // impulse accumulators (F_PA slots) cleared by all lanes
                for (int g = sub; g < M::NG; g += LPE) stsv(s, g * GF + F_PA, sv0());
                TG_SYNC();
            }
            // projected Gauss-Seidel with patch friction, all LPE lanes of the env:
            // each lane holds W's columns j = sub + LPE*jj and the full multiplier
            // vector in registers; a row's W*lambda is an 8-lane reduction, so
            // every lane computes the same update (no LDS traffic in the sweeps)
            {
                static_assert(LPE == 8, "sum8 reduces over 8 lanes");
                constexpr int JL = (K + LPE - 1) / LPE;
                float wc[K][JL], vf[K], tg[K], onr[K], wd[K], lam[K], my[JL];
#pragma unroll
                for (int i = 0; i < K; ++i) {
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) {
                        const int j = sub + LPE * jj;
                        wc[i][jj] = j < K ? s(PL::W + i * K + j) : 0.f;
                    }
                    vf[i] = s(PL::VFREE + i);
                    tg[i] = s(PL::ROW + i * 8 + 6);
                    onr[i] = s(PL::ROW + i * 8 + 7);
                    wd[i] = s(PL::W + i * K + i);
                    lam[i] = 0.f;
                }
#pragma unroll
                for (int jj = 0; jj < JL; ++jj) my[jj] = 0.f;
                auto row_v = [&](int i) {   // vfree_i + (W lambda)_i
                    float part = 0.f;
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj) part += wc[i][jj] * my[jj];
                    return vf[i] + sum8(part);
                };
                auto set_lam = [&](int i, float v) {
                    lam[i] = v;
#pragma unroll
                    for (int jj = 0; jj < JL; ++jj)
                        if (sub + LPE * jj == i) my[jj] = v;
                };
#pragma unroll 1
                for (int it = 0; it < a.iters; ++it) {
#pragma unroll
                    for (int sh = 0; sh < M::NS; ++sh) {
                        const int rb = row_base<M>(sh), nr = M::shape_nrows[sh];
                        float Nsum = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (k >= nr) break;
                            const int i = rb + k;
                            const float vi = row_v(i);
                            const float l = lam[i] + (tg[i] - vi) / wd[i];
                            const float li = onr[i] * fmaxf(l, 0.f);
                            set_lam(i, li);
                            Nsum += li;
                        }
                        const int f = rb + nr;
                        const float mu = s(PL::SHP + 2 * sh), reff = s(PL::SHP + 2 * sh + 1);
#pragma unroll
                        for (int t = 0; t < 3; ++t) {
                            const int i = f + t;
                            const float vi = row_v(i);
                            set_lam(i, lam[i] - vi / wd[i]);
                            if (t == 1) {
                                const float l0 = lam[f], l1 = lam[f + 1];
                                const float lt = sqrtf(l0 * l0 + l1 * l1), lim = mu * Nsum;
                                const float sc = lt > lim ? (lt > 0.f ? lim / lt : 0.f) : 1.f;
                                set_lam(f, l0 * sc);
                                set_lam(f + 1, l1 * sc);
                            }
                        }
                        const float lim3 = mu * Nsum * reff;
                        set_lam(f + 2, fminf(fmaxf(lam[f + 2], -lim3), lim3));
                    }
                }
                if (lead) {
#pragma unroll
                    for (int i = 0; i < K; ++i) s(PL::LAM + i) = lam[i];
                }
            }
            TG_SYNC();
            SV da0 = sv0();
            if constexpr (SUPER) {
                TG_PROF(6)
                // joint impulses u_g = sum_j lam_j du_j on the contact paths (0 elsewhere),
                // one contact group at a time (paths may share ancestors)
                for (int g = sub; g < M::NG; g += LPE) s(g * GF + F_UU) = 0.f;
                TG_SYNC();
#pragma unroll
                for (int c = 0; c < M::NCG; ++c) {
                    for (int i = sub; i < M::cpath_len[c]; i += LPE) {
                        float acc = 0.f;
#pragma unroll
                        for (int j = 0; j < K; ++j)
                            if (M::shape_cg[row_shape<M>(j)] == c) acc += s(PL::LAM + j) * s(scr(j * SW + i));
                        s(cpath[c * M::MAXD + i] * GF + F_UU) += acc;
                    }
                    TG_SYNC();
                }
                if (!fix_base) {
                    float d6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const float l = s(PL::LAM + j);
#pragma unroll
                        for (int k = 0; k < 6; ++k) d6[k] += l * s(scr(j * SW + M::MAXD + k));
                    }
                    da0 = SV{v3(d6[0], d6[1], d6[2]), v3(d6[3], d6[4], d6[5])};
                }
            } else {
                if (lead) {
                    // impulses into the contact groups' F_PA slots (p = -f convention)
                    for (int i = 0; i < K; ++i) {
                        const int g = M::shape_group[row_shape<M>(i)];
                        stsv(s, g * GF + F_PA, ldsv(s, g * GF + F_PA) + (-1.0f) * rforce(i, s(PL::LAM + i)));
                    }
                }
                TG_SYNC();
                TG_PROF(6)
                // impulse application: bottom-up gather, root solve, top-down
#pragma unroll 1
                for (int t = M::NSTEP - 1; t >= 0; --t) {
                    const int g = sched[t * LPE + sub];
                    if (g > 0) {
                        const int o = g * GF;
                        SV p = ldsv(s, o + F_PA);
                        const int nch = gi[g * GIW + GI_NCH];
                        for (int c = 0; c < nch; ++c) p = p + ldsv(s, gi[g * GIW + GI_CH + c] * GF + F_PA);
                        const float u = -dotS(ginfo<M>(gi, g).jt, p);
                        s(o + F_UU) = u;
                        const SV pa = p + (u * s(o + F_DINV)) * ldsv(s, o + F_U);
                        stsv(s, o + F_PA, xTforce(ldx(s, g), pa));
                    }
                    TG_SYNC();
                }
                SV p0 = ldsv(s, F_PA);
                for (int c = 0; c < M::nchild[0]; ++c) p0 = p0 + ldsv(s, M::child[0][c] * GF + F_PA);
                if (!fix_base) da0 = ldl6_solve(rootf, -1.0f * p0);
            }
            TG_SYNC();
            if (lead) stsv(s, F_PA, da0);
            TG_SYNC();
#pragma unroll 1
            for (int t = 0; t < M::NSTEP; ++t) {
                const int g = sched[t * LPE + sub];
                if (g > 0) {
                    const int o = g * GF;
                    const GInfo G = ginfo<M>(gi, g);
                    const SV ap = xmotion(ldx(s, g), ldsv(s, G.parent * GF + F_PA));
                    const float x = (s(o + F_UU) - dot(ldsv(s, o + F_U), ap)) * s(o + F_DINV);
                    stsv(s, o + F_PA, addS(G.jt, ap, x));
                    s(o + F_QDS) += x;
                }
                TG_SYNC();
            }
            if (!fix_base) v0s = v0s + da0;
            TG_PROF(7)
        }
        // ---- velocity limits + integration
        for (int g = 1 + sub; g < M::NG; g += LPE) {
            const int o = g * GF;
            const float vl = PR(TG_PROP_VELOCITY, gi[g * GIW + GI_DOF]);
            float x = s(o + F_QDS);
            if (vl > 0.f) x = fminf(fmaxf(x, -vl), vl);
            s(o + F_QD) = x;
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
                __sincosf(0.5f * an, &sa, &ca);
                const float kk = sa / wn;
                dx = v0.w.x * kk; dy = v0.w.y * kk; dz = v0.w.z * kk; dw = ca;
            }
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
    if (owner) {
        if (lead) {
            const V3 wwo = mul(R, v0.w);
            const V3 vco = mul(R, v0.v) + cross(wwo, mul(R, c0));
            root[0] = pos.x; root[1] = pos.y; root[2] = pos.z;
            root[3] = qx; root[4] = qy; root[5] = qz; root[6] = qw;
            root[7] = vco.x; root[8] = vco.y; root[9] = vco.z;
            root[10] = wwo.x; root[11] = wwo.y; root[12] = wwo.z;
        }
        for (int g = 1 + sub; g < M::NG; g += LPE) {
            const int d = gi[g * GIW + GI_DOF];
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
}

#undef TG_SYNC

}  // namespace tg
