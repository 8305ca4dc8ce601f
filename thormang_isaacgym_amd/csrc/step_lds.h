// step_lds.h -- LDS-resident variant of the articulation step for large joint
// trees (included by articulation.hip; same algorithm as step_kernel<M> and
// oracle/physics_ref.c).
//
// One env per lane, EPB envs per workgroup (EPB = 16 for Thormang: 256
// workgroups fill all 256 CUs at 4096 envs).  Per-group articulated state
// (X, v, I^A, p^A, U, D^-1, u, q, qd, world pose) lives in LDS at
// [field][lane] (lane-contiguous, conflict-free); the per-group loops are
// rolled and the joint-tree tables are wave-uniform scalar loads, so register
// pressure is bounded by one group's working set instead of the whole tree.
// The Delassus matrix is built with path-restricted impulse responses: a unit
// impulse on contact group k only changes p^A on k's ancestor path, and only
// the accelerations along the root->contact-group paths are propagated down.
#pragma once

namespace tg {

template <int EPB> struct LV {
    float *b;
    int lane;
    __device__ __forceinline__ float &operator()(int i) const { return b[i * EPB + lane]; }
};

// per-group field offsets (GF floats per group)
enum : int {
    F_E = 0, F_R = 9, F_V = 12, F_IA = 18, F_PA = 39, F_U = 45, F_DINV = 51, F_UU = 52, F_Q = 53, F_QD = 54,
    F_QDS = 55, F_GL = 56, GF = 59
};

template <int EPB> __device__ __forceinline__ V3 ldv3(const LV<EPB> &s, int o) { return v3(s(o), s(o + 1), s(o + 2)); }
template <int EPB> __device__ __forceinline__ void stv3(const LV<EPB> &s, int o, V3 v) {
    s(o) = v.x; s(o + 1) = v.y; s(o + 2) = v.z;
}
template <int EPB> __device__ __forceinline__ SV ldsv(const LV<EPB> &s, int o) { return SV{ldv3(s, o), ldv3(s, o + 3)}; }
template <int EPB> __device__ __forceinline__ void stsv(const LV<EPB> &s, int o, const SV &v) {
    stv3(s, o, v.w);
    stv3(s, o + 3, v.v);
}
template <int EPB> __device__ __forceinline__ M3 ldm3(const LV<EPB> &s, int o) {
    M3 m;
#pragma unroll
    for (int k = 0; k < 9; ++k) m.a[k] = s(o + k);
    return m;
}
template <int EPB> __device__ __forceinline__ void stm3(const LV<EPB> &s, int o, const M3 &m) {
#pragma unroll
    for (int k = 0; k < 9; ++k) s(o + k) = m.a[k];
}
template <int EPB> __device__ __forceinline__ SI ldsi(const LV<EPB> &s, int o) {
    SI I;
#pragma unroll
    for (int k = 0; k < 6; ++k) { I.A[k] = s(o + k); I.C[k] = s(o + 15 + k); }
#pragma unroll
    for (int k = 0; k < 9; ++k) I.B[k] = s(o + 6 + k);
    return I;
}
template <int EPB> __device__ __forceinline__ void stsi(const LV<EPB> &s, int o, const SI &I) {
#pragma unroll
    for (int k = 0; k < 6; ++k) { s(o + k) = I.A[k]; s(o + 15 + k) = I.C[k]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) s(o + 6 + k) = I.B[k];
}
template <int EPB> __device__ __forceinline__ Xf ldx(const LV<EPB> &s, int g) {
    return Xf{ldm3(s, g * GF + F_E), ldv3(s, g * GF + F_R)};
}

template <class M> __device__ __forceinline__ SV motion_S(int g) {
    const V3 ax = v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]);
    return M::jtype[g] == TG_JOINT_REVOLUTE ? SV{ax, v3(0, 0, 0)} : SV{v3(0, 0, 0), ax};
}

// world pose of group g by walking up to the root: R_g = R_0 E_a1^T ... E_g^T
template <class M, int EPB>
__device__ __forceinline__ void world_pose(const LV<EPB> &s, int g, const M3 &R0, V3 p0, M3 &Rg, V3 &pg) {
    M3 Mr = eye3();
    V3 t = v3(0, 0, 0);
    while (g != 0) {
        const M3 Et = transpose(ldm3(s, g * GF + F_E));
        t = ldv3(s, g * GF + F_R) + mul(Et, t);
        Mr = mul(Et, Mr);
        g = M::parent[g];
    }
    Rg = mul(R0, Mr);
    pg = p0 + mul(R0, t);
}

template <class M> struct LdsLayout {
    static constexpr int K = M::NROWS;
    static constexpr int groups = M::NG * GF;
    static constexpr int W = groups;                 // K*K
    static constexpr int ROW = W + K * K;            // K * 8: r(3) d(3) target on
    static constexpr int VFREE = ROW + K * 8;
    static constexpr int LAM = VFREE + K;
    static constexpr int SHP = LAM + K;              // per shape: mu, reff
    static constexpr int CGP = SHP + 2 * M::NSA;     // per contact group: world R (9), p (3)
    static constexpr int TOTAL = CGP + 12 * M::NCG;
};

// velocity change at every contact group for impulse fk (group frame) applied to group k.
// du[g] for g on k's ancestor path is left in LDS field F_UU; a0 returned.
template <class M, int EPB>
__device__ __forceinline__ void impulse_contact_groups(const LV<EPB> &s, const LDL6 &root, bool fix_base, int k,
                                                       SV p, SV *dvc) {
    // up the path k -> root
    int g = k;
    while (g != 0) {
        const SV S = motion_S<M>(g);
        const float u = -dot(S, p);
        s(g * GF + F_UU) = u;
        const SV pa = p + (u * s(g * GF + F_DINV)) * ldsv(s, g * GF + F_U);
        p = xTforce(ldx(s, g), pa);
        g = M::parent[g];
    }
    const SV a0 = fix_base ? sv0() : ldl6_solve(root, -1.0f * p);
    for (int c = 0; c < M::NCG; ++c) {
        SV a = a0;
        for (int i = 0; i < M::cpath_len[c]; ++i) {
            const int h = M::cpath[c][i];
            const SV ap = xmotion(ldx(s, h), a);
            const float du = M::anc[k][h] ? s(h * GF + F_UU) : 0.0f;
            const float x = (du - dot(ldsv(s, h * GF + F_U), ap)) * s(h * GF + F_DINV);
            a = ap + x * motion_S<M>(h);
        }
        dvc[c] = a;
    }
}

template <class M, int EPB> __global__ __launch_bounds__(EPB) void step_lds_kernel(StepArgs a) {
    extern __shared__ float lds_raw[];
    const int lane = threadIdx.x;
    const int e = blockIdx.x * EPB + lane;
    if (e >= a.N) return;
    using CL = CompLayout<M>;
    using LL = LdsLayout<M>;
    const LV<EPB> s{lds_raw, lane};
    const size_t N = a.N;
    const int D = a.D;
    const float h = a.h;
    const bool fix_base = a.fix_base != 0;
    const float *comp = a.comp;
    auto CP = [&](int k) { return comp[(size_t)k * N + e]; };

    float *root = a.root + (size_t)e * 13;
    float *dofs = a.dof + (size_t)e * D * 2;
#pragma unroll 1
    for (int g = 1; g < M::NG; ++g) {
        s(g * GF + F_Q) = dofs[2 * M::gdof[g]];
        s(g * GF + F_QD) = dofs[2 * M::gdof[g] + 1];
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

    for (int sub = 0; sub < a.substeps; ++sub) {
        // ---- pass 1
#pragma unroll 1
        for (int g = 0; g < M::NG; ++g) {
            const int o = g * GF;
            SV vg;
            V3 gl;
            if (g == 0) {
                vg = v0;
                gl = mulT(R, grav);
            } else {
                const int p = M::parent[g];
                M3 Rpc;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rpc.a[k] = CP(CL::xtree(g) + k);
                V3 t = v3(CP(CL::xtree(g) + 9), CP(CL::xtree(g) + 10), CP(CL::xtree(g) + 11));
                const float qg = s(o + F_Q);
                if (M::jtype[g] == TG_JOINT_REVOLUTE) Rpc = mul(Rpc, rot_axis(M::axis[g][0], M::axis[g][1], M::axis[g][2], qg));
                else t = t + qg * mul(Rpc, v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]));
                const Xf X{transpose(Rpc), t};
                stm3(s, o + F_E, X.E);
                stv3(s, o + F_R, t);
                vg = xmotion(X, ldsv(s, p * GF + F_V)) + s(o + F_QD) * motion_S<M>(g);
                gl = mul(X.E, ldv3(s, p * GF + F_GL));
            }
            stsv(s, o + F_V, vg);
            stv3(s, o + F_GL, gl);
            const float m = CP(CL::inertia(g));
            const V3 cg = v3(CP(CL::inertia(g) + 1), CP(CL::inertia(g) + 2), CP(CL::inertia(g) + 3));
            float Ic[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) Ic[k] = CP(CL::inertia(g) + 4 + k);
            const SI I = rb_inertia(m, cg, Ic);
            stsi(s, o + F_IA, I);
            const SV b = crf(vg, mul(I, vg));
            V3 F = m * gl;
            F = F - (a.lin_damp * m) * (vg.v + cross(vg.w, cg));
            V3 n = cross(cg, F) - a.ang_damp * symmul(Ic, vg.w);
            if (a.force) {
                const float *fw = a.force + ((size_t)e * M::NG + g) * 6;
                M3 Rw;
                V3 pw_;
                world_pose<M, EPB>(s, g, R, pos, Rw, pw_);
                const V3 fl = mulT(Rw, v3(fw[0], fw[1], fw[2])), tl = mulT(Rw, v3(fw[3], fw[4], fw[5]));
                F = F + fl;
                n = n + tl + cross(cg, fl);
            }
            stsv(s, o + F_PA, SV{b.w - n, b.v - F});
        }
        // ---- pass 2
#pragma unroll 1
        for (int g = M::NG - 1; g >= 1; --g) {
            const int o = g * GF, p = M::parent[g], d = M::gdof[g];
            const SV S = motion_S<M>(g);
            const SI IA = ldsi(s, o + F_IA);
            const SV U = mul(IA, S);
            const float q = s(o + F_Q), qd = s(o + F_QD);
            const float D0 = dot(S, U) + prop(a, TG_PROP_ARMATURE, e, d);
            float Dimp = 0.f, tau = 0.f;
            const int mode = (int)rintf(prop(a, TG_PROP_DRIVE_MODE, e, d));
            const float kp = prop(a, TG_PROP_STIFFNESS, e, d), kd = prop(a, TG_PROP_DAMPING, e, d);
            const float eff = prop(a, TG_PROP_EFFORT, e, d);
            if (mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL) {
                const float te = kp * (a.pos_tgt[(size_t)e * D + d] - q - h * qd) + kd * (a.vel_tgt[(size_t)e * D + d] - qd);
                if (fabsf(te) <= eff) { tau += te; Dimp += h * kd + h * h * kp; }
                else tau += te > 0.f ? eff : -eff;
            } else if (mode == TG_DOF_MODE_EFFORT && a.act) {
                tau += fminf(fmaxf(a.act[(size_t)e * D + d], -eff), eff);
            }
            const float lo = prop(a, TG_PROP_LOWER, e, d), hi = prop(a, TG_PROP_UPPER, e, d);
            const float qp = q + h * qd;
            const float kl = a.lim_k * D0 / (h * h), cl = a.lim_c * D0 / h;
            if (qp < lo && lo > -1e30f) { tau += kl * (lo - qp) - cl * qd; Dimp += h * cl + h * h * kl; }
            else if (qp > hi && hi < 1e30f) { tau += kl * (hi - qp) - cl * qd; Dimp += h * cl + h * h * kl; }
            const float Dinv = 1.0f / (D0 + Dimp);
            const SV pA = ldsv(s, o + F_PA);
            const float u = tau - dot(S, pA);
            stsv(s, o + F_U, U);
            s(o + F_DINV) = Dinv;
            s(o + F_UU) = u;
            SI Ia = IA;
            si_sub_outer(Ia, U, Dinv);
            const SV vg = ldsv(s, o + F_V);
            const SV c = crm(vg, qd * S);
            const SV pa = pA + mul(Ia, c) + (u * Dinv) * U;
            const Xf X = ldx(s, g);
            SI IAp = ldsi(s, p * GF + F_IA);
            si_add(IAp, si_to_parent(Ia, X));
            stsi(s, p * GF + F_IA, IAp);
            stsv(s, p * GF + F_PA, ldsv(s, p * GF + F_PA) + xTforce(X, pa));
        }
        // ---- pass 3: free accelerations / velocities
        const LDL6 rootf = fix_base ? LDL6{} : ldl6(ldsi(s, F_IA));
        SV a0 = fix_base ? sv0() : ldl6_solve(rootf, -1.0f * ldsv(s, F_PA));
        // accelerations are propagated through the F_PA slots (p^A no longer needed)
        stsv(s, F_PA, a0);
#pragma unroll 1
        for (int g = 1; g < M::NG; ++g) {
            const int o = g * GF;
            const SV S = motion_S<M>(g);
            const float qd = s(o + F_QD);
            const SV c = crm(ldsv(s, o + F_V), qd * S);
            const SV ap = xmotion(ldx(s, g), ldsv(s, M::parent[g] * GF + F_PA)) + c;
            const float qdd = (s(o + F_UU) - dot(ldsv(s, o + F_U), ap)) * s(o + F_DINV);
            stsv(s, o + F_PA, ap + qdd * S);
            s(o + F_QDS) = qd + h * qdd;
        }
        SV v0s = v0 + h * a0;
        v0s.v = v0s.v + h * cross(v0.w, v0.v);
        if (fix_base) v0s = sv0();

        // ---- contacts
        if constexpr (M::NS > 0) {
            constexpr int K = M::NROWS;
            // free velocities of the contact groups (propagate v with qds along their paths)
            SV vcs[M::NCG];
            for (int c = 0; c < M::NCG; ++c) {
                M3 Rc;
                V3 pc;
                world_pose<M, EPB>(s, M::cgroup[c], R, pos, Rc, pc);
                stm3(s, LL::CGP + 12 * c, Rc);
                stv3(s, LL::CGP + 12 * c + 9, pc);
            }
            for (int c = 0; c < M::NCG; ++c) {
                SV v = v0s;
                for (int i = 0; i < M::cpath_len[c]; ++i) {
                    const int hg = M::cpath[c][i];
                    v = xmotion(ldx(s, hg), v) + s(hg * GF + F_QDS) * motion_S<M>(hg);
                }
                vcs[c] = v;
            }
#pragma unroll 1
            for (int sh = 0; sh < M::NS; ++sh) {
                const int cgi = M::shape_cg[sh];
                const int rb = row_base<M>(sh);
                const M3 Rwg = ldm3(s, LL::CGP + 12 * cgi);
                const V3 pwg = ldv3(s, LL::CGP + 12 * cgi + 9);
                M3 Rsl;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rsl.a[k] = CP(CL::shape(sh) + k);
                const M3 Rs = mul(Rwg, Rsl);
                const V3 cl = v3(CP(CL::shape(sh) + 9), CP(CL::shape(sh) + 10), CP(CL::shape(sh) + 11));
                const V3 cw = pwg + mul(Rwg, cl);
                V3 pts[4];
                const int nr = M::shape_nrows[sh];
                if (M::shape_kind[sh] == TG_SHAPE_TORUS) {
                    const V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                    V3 dd = v3(-ax.z * ax.x, -ax.z * ax.y, 1.f - ax.z * ax.z);
                    float nd = sqrtf(dot(dd, dd));
                    if (nd < 1e-6f) { dd = v3(1, 0, 0); nd = 1.f; }
                    pts[0] = cw - (M::shape_params[sh][0] / nd) * dd - v3(0, 0, M::shape_params[sh][1]);
                } else if (M::shape_kind[sh] == TG_SHAPE_SPHERE) {
                    pts[0] = cw - v3(0, 0, M::shape_params[sh][0]);
                } else {
                    const float hx = M::shape_params[sh][0], hy = M::shape_params[sh][1], hz = M::shape_params[sh][2];
                    const float zx = Rs.a[6], zy = Rs.a[7], zz = Rs.a[8];
                    const float ax_ = fabsf(zx), ay_ = fabsf(zy), az_ = fabsf(zz);
                    const V3 ex = v3(Rs.a[0], Rs.a[3], Rs.a[6]), ey = v3(Rs.a[1], Rs.a[4], Rs.a[7]),
                             ez = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                    V3 fn, u1, u2;
                    if (az_ >= ax_ && az_ >= ay_) { fn = (zz > 0 ? -hz : hz) * ez; u1 = hx * ex; u2 = hy * ey; }
                    else if (ay_ >= ax_) { fn = (zy > 0 ? -hy : hy) * ey; u1 = hx * ex; u2 = hz * ez; }
                    else { fn = (zx > 0 ? -hx : hx) * ex; u1 = hy * ey; u2 = hz * ez; }
                    pts[0] = cw + fn - u1 - u2;
                    pts[1] = cw + fn + u1 - u2;
                    pts[2] = cw + fn - u1 + u2;
                    pts[3] = cw + fn + u1 + u2;
                }
                V3 cen = v3(0, 0, 0);
                float nact = 0.f;
                for (int k = 0; k < nr; ++k) {
                    const int ro = LL::ROW + (rb + k) * 8;
                    const float phi = pts[k].z;
                    const float on = phi <= a.margin ? 1.f : 0.f;
                    stv3(s, ro, mulT(Rwg, pts[k] - pwg));
                    stv3(s, ro + 3, v3(0, 0, 1));
                    s(ro + 6) = phi > a.rest ? -(phi - a.rest) / h : fminf(a.baumgarte * (a.rest - phi) / h, a.max_depen);
                    s(ro + 7) = on;
                    cen = cen + on * pts[k];
                    nact += on;
                }
                cen = (nact > 0.f ? 1.f / nact : 0.f) * cen;
                float re = 0.f;
                for (int k = 0; k < nr; ++k) {
                    const float dx = pts[k].x - cen.x, dy = pts[k].y - cen.y;
                    re += s(LL::ROW + (rb + k) * 8 + 7) * sqrtf(dx * dx + dy * dy);
                }
                s(LL::SHP + 2 * sh) = 0.5f * (a.shape_mu[(size_t)e * M::NS + sh] + a.ground_mu);
                s(LL::SHP + 2 * sh + 1) = nact > 0.f ? re / nact : 0.f;
                V3 t1 = v3(1, 0, 0);
                if (M::shape_kind[sh] == TG_SHAPE_TORUS) {
                    const V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                    const V3 x = cross(ax, v3(0, 0, 1));
                    const float nx = sqrtf(dot(x, x));
                    if (nx > 1e-6f) t1 = (1.f / nx) * x;
                }
                const V3 t2 = cross(v3(0, 0, 1), t1);
                const V3 rl = mulT(Rwg, cen - pwg);
                const float fon = nact > 0.f ? 1.f : 0.f;
                for (int t = 0; t < 3; ++t) {
                    const int ro = LL::ROW + (rb + nr + t) * 8;
                    stv3(s, ro, rl);
                    stv3(s, ro + 3, t == 0 ? t1 : (t == 1 ? t2 : v3(0, 0, 1)));
                    s(ro + 6) = 0.f;
                    s(ro + 7) = fon;
                }
            }
            // row helpers
            auto row_is_ang = [&](int i) {
                const int sh = row_shape<M>(i);
                return i == row_base<M>(sh) + M::shape_nrows[sh] + 2;
            };
            auto rvel = [&](int i, const SV &vg) {
                const int ro = LL::ROW + i * 8;
                const M3 Rwg = ldm3(s, LL::CGP + 12 * M::shape_cg[row_shape<M>(i)]);
                const V3 o = row_is_ang(i) ? mul(Rwg, vg.w) : mul(Rwg, vg.v + cross(vg.w, ldv3(s, ro)));
                return dot(o, ldv3(s, ro + 3));
            };
            auto rforce = [&](int i, float lam) {
                const int ro = LL::ROW + i * 8;
                const V3 dl = mulT(ldm3(s, LL::CGP + 12 * M::shape_cg[row_shape<M>(i)]), ldv3(s, ro + 3));
                return row_is_ang(i) ? SV{lam * dl, v3(0, 0, 0)} : SV{lam * cross(ldv3(s, ro), dl), lam * dl};
            };
#pragma unroll 1
            for (int i = 0; i < K; ++i) {
                s(LL::VFREE + i) = rvel(i, vcs[M::shape_cg[row_shape<M>(i)]]);
                s(LL::LAM + i) = 0.f;
            }
            // Delassus columns
#pragma unroll 1
            for (int j = 0; j < K; ++j) {
                const int gj = M::shape_group[row_shape<M>(j)];
                SV dvc[M::NCG];
                impulse_contact_groups<M, EPB>(s, rootf, fix_base, gj, -1.0f * rforce(j, 1.0f), dvc);
                for (int i = 0; i < K; ++i) s(LL::W + i * K + j) = rvel(i, dvc[M::shape_cg[row_shape<M>(i)]]);
            }
            // projected Gauss-Seidel with patch friction
#pragma unroll 1
            for (int it = 0; it < a.iters; ++it) {
                for (int sh = 0; sh < M::NS; ++sh) {
                    const int rb = row_base<M>(sh), nr = M::shape_nrows[sh];
                    float Nsum = 0.f;
                    for (int k = 0; k < nr; ++k) {
                        const int i = rb + k;
                        float vi = s(LL::VFREE + i);
                        for (int j = 0; j < K; ++j) vi += s(LL::W + i * K + j) * s(LL::LAM + j);
                        const float l = s(LL::LAM + i) + (s(LL::ROW + i * 8 + 6) - vi) / s(LL::W + i * K + i);
                        const float li = s(LL::ROW + i * 8 + 7) * fmaxf(l, 0.f);
                        s(LL::LAM + i) = li;
                        Nsum += li;
                    }
                    const int f = rb + nr;
                    const float mu = s(LL::SHP + 2 * sh), reff = s(LL::SHP + 2 * sh + 1);
                    for (int t = 0; t < 3; ++t) {
                        const int i = f + t;
                        float vi = s(LL::VFREE + i);
                        for (int j = 0; j < K; ++j) vi += s(LL::W + i * K + j) * s(LL::LAM + j);
                        s(LL::LAM + i) = s(LL::LAM + i) - vi / s(LL::W + i * K + i);
                        if (t == 1) {
                            const float l0 = s(LL::LAM + f), l1 = s(LL::LAM + f + 1);
                            const float lt = sqrtf(l0 * l0 + l1 * l1), lim = mu * Nsum;
                            const float sc = lt > lim ? (lt > 0.f ? lim / lt : 0.f) : 1.f;
                            s(LL::LAM + f) = l0 * sc;
                            s(LL::LAM + f + 1) = l1 * sc;
                        }
                    }
                    const float lim3 = mu * Nsum * reff;
                    s(LL::LAM + f + 2) = fminf(fmaxf(s(LL::LAM + f + 2), -lim3), lim3);
                }
            }
            // apply: accumulate impulses per group in the F_PA slots (reset), full tree sweep
#pragma unroll 1
            for (int g = 0; g < M::NG; ++g) stsv(s, g * GF + F_PA, sv0());
#pragma unroll 1
            for (int i = 0; i < K; ++i) {
                const int g = M::shape_group[row_shape<M>(i)];
                stsv(s, g * GF + F_PA, ldsv(s, g * GF + F_PA) + (-1.0f) * rforce(i, s(LL::LAM + i)));
            }
#pragma unroll 1
            for (int g = M::NG - 1; g >= 1; --g) {
                const int o = g * GF;
                const SV p = ldsv(s, o + F_PA);
                const float u = -dot(motion_S<M>(g), p);
                s(o + F_UU) = u;
                const SV pa = p + (u * s(o + F_DINV)) * ldsv(s, o + F_U);
                const int pg = M::parent[g];
                stsv(s, pg * GF + F_PA, ldsv(s, pg * GF + F_PA) + xTforce(ldx(s, g), pa));
            }
            const SV da0 = fix_base ? sv0() : ldl6_solve(rootf, -1.0f * ldsv(s, F_PA));
            stsv(s, F_PA, da0);
#pragma unroll 1
            for (int g = 1; g < M::NG; ++g) {
                const int o = g * GF;
                const SV ap = xmotion(ldx(s, g), ldsv(s, M::parent[g] * GF + F_PA));
                const float x = (s(o + F_UU) - dot(ldsv(s, o + F_U), ap)) * s(o + F_DINV);
                stsv(s, o + F_PA, ap + x * motion_S<M>(g));
                s(o + F_QDS) += x;
            }
            if (!fix_base) v0s = v0s + da0;
        }
        // ---- velocity limits + integration
#pragma unroll 1
        for (int g = 1; g < M::NG; ++g) {
            const int o = g * GF;
            const float vl = prop(a, TG_PROP_VELOCITY, e, M::gdof[g]);
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
    }
    const V3 wwo = mul(R, v0.w);
    const V3 vco = mul(R, v0.v) + cross(wwo, mul(R, c0));
    root[0] = pos.x; root[1] = pos.y; root[2] = pos.z;
    root[3] = qx; root[4] = qy; root[5] = qz; root[6] = qw;
    root[7] = vco.x; root[8] = vco.y; root[9] = vco.z;
    root[10] = wwo.x; root[11] = wwo.y; root[12] = wwo.z;
#pragma unroll 1
    for (int g = 1; g < M::NG; ++g) {
        dofs[2 * M::gdof[g]] = s(g * GF + F_Q);
        dofs[2 * M::gdof[g] + 1] = s(g * GF + F_QD);
    }
#pragma unroll 1
    for (int d = 0; d < M::ND; ++d) {
        if (M::dof_locked[d]) {
            dofs[2 * d] = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
            dofs[2 * d + 1] = 0.f;
        }
    }
}

}  // namespace tg
