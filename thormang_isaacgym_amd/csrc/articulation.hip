// articulation.hip -- the per-env articulated-body step that replaces PhysX's
// gym.simulate (reference: isaacgymenvs/tasks/base/vec_task.py:332-335; model
// and drive set-up tasks/gogoro_new.py:196-294, cfg/task/Gogoro.yaml:9-31).
//
// One env per lane.  The kernel template is specialised per compiled model
// (generated/Model_*.inc): every per-group loop is fully unrolled over the
// joint tree, so tree indices, joint axes and shape parameters are
// instruction immediates and the per-group state lives in registers.
//
// Per substep (h = dt / substeps), mirroring oracle/physics_ref.c:
//   1. kinematics + velocities + bias forces (gravity, damping, applied wrench)
//   2. articulated-body inertias with implicit PD drive / limit terms folded
//      into the joint-space diagonal D (h*kd + h^2*kp), effort saturation
//   3. accelerations -> free velocities (semi-implicit Euler, world-fixed root velocity)
//   4. ground contact: static row set per model (normals per shape point,
//      patch friction t1/t2 + torsion), Delassus matrix from impulse
//      responses through the same articulated inertias, projected
//      Gauss-Seidel, one impulse application
//   5. velocity limits, integration of joint positions and the floating base.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tgsim.h"
#include "generated/models.inc"
#include "tg_math.h"
#include "tg_kernels.h"

namespace tg {

// per-env composite cache layout (SoA, [KC][N])
template <class M> struct CompLayout {
    static constexpr int inertia(int g) { return 10 * g; }
    static constexpr int xtree(int g) { return 10 * M::NG + 12 * (g - 1); }
    static constexpr int shape(int s) { return 10 * M::NG + 12 * (M::NG - 1) + 12 * s; }
};

__device__ __forceinline__ float prop(const StepArgs &a, int f, int e, int d) {
    return a.props[((size_t)f * a.N + e) * a.D + d];
}

// ---------------------------------------------------------------- compose
// Per-env group composites from the locked joint positions (centre of each
// lock window) and the per-link mass scale (domain randomisation).
template <class M> __global__ __launch_bounds__(64) void compose_kernel(StepArgs a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.N || !a.dirty[e]) return;
    using CL = CompLayout<M>;
    M3 TR[M::NL];
    V3 TP[M::NL];
    float gm[M::NG];
    V3 gc[M::NG];
#pragma unroll
    for (int g = 0; g < M::NG; ++g) { gm[g] = 0.f; gc[g] = v3(0, 0, 0); }
#pragma unroll
    for (int l = 0; l < M::NL; ++l) {
        if (M::link_is_group_root[l]) {
            TR[l] = eye3();
            TP[l] = v3(0, 0, 0);
        } else {
            const int p = M::link_parent[l];
            const float *o = M::link_origin[l];
            M3 Ro{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}};
            V3 to = v3(o[9], o[10], o[11]);
            const int d = M::link_dof[l];
            if (d >= 0) {
                const float q = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
                const float *ax = M::link_axis[l];
                if (M::link_jtype[l] == TG_JOINT_REVOLUTE) Ro = mul(Ro, rot_axis(ax[0], ax[1], ax[2], q));
                else if (M::link_jtype[l] == TG_JOINT_PRISMATIC) to = to + q * mul(Ro, v3(ax[0], ax[1], ax[2]));
            }
            TR[l] = mul(TR[p], Ro);
            TP[l] = TP[p] + mul(TR[p], to);
        }
        const float s = a.mass_scale ? a.mass_scale[(size_t)e * M::NL + l] : 1.0f;
        const float ml = M::link_inertia[l][0] * s;
        const V3 cg = mul(TR[l], v3(M::link_inertia[l][1], M::link_inertia[l][2], M::link_inertia[l][3])) + TP[l];
        gm[M::link_group[l]] += ml;
        gc[M::link_group[l]] = gc[M::link_group[l]] + ml * cg;
    }
    float gI[M::NG][6];
#pragma unroll
    for (int g = 0; g < M::NG; ++g) {
        gc[g] = (gm[g] > 0.f ? 1.0f / gm[g] : 0.f) * gc[g];
#pragma unroll
        for (int k = 0; k < 6; ++k) gI[g][k] = 0.f;
    }
#pragma unroll
    for (int l = 0; l < M::NL; ++l) {
        const int g = M::link_group[l];
        const float s = a.mass_scale ? a.mass_scale[(size_t)e * M::NL + l] : 1.0f;
        const float *in = M::link_inertia[l];
        const float ml = in[0] * s;
        M3 Il{{in[4] * s, in[7] * s, in[8] * s, in[7] * s, in[5] * s, in[9] * s, in[8] * s, in[9] * s, in[6] * s}};
        M3 RI = mul(mul(TR[l], Il), transpose(TR[l]));
        V3 dd = mul(TR[l], v3(in[1], in[2], in[3])) + TP[l] - gc[g];
        float d2 = dot(dd, dd);
        gI[g][0] += RI.a[0] + ml * (d2 - dd.x * dd.x);
        gI[g][1] += RI.a[4] + ml * (d2 - dd.y * dd.y);
        gI[g][2] += RI.a[8] + ml * (d2 - dd.z * dd.z);
        gI[g][3] += RI.a[1] - ml * dd.x * dd.y;
        gI[g][4] += RI.a[2] - ml * dd.x * dd.z;
        gI[g][5] += RI.a[5] - ml * dd.y * dd.z;
    }
    float *c = a.comp;
    const size_t N = a.N;
#pragma unroll
    for (int g = 0; g < M::NG; ++g) {
        float *ci = c + CL::inertia(g) * N + e;
        ci[0] = gm[g];
        ci[N] = gc[g].x; ci[2 * N] = gc[g].y; ci[3 * N] = gc[g].z;
#pragma unroll
        for (int k = 0; k < 6; ++k) ci[(4 + k) * N] = gI[g][k];
        if (g > 0) {
            const int r = M::group_root[g], p = M::link_parent[r];
            const float *o = M::link_origin[r];
            M3 Ro{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}};
            M3 R = mul(TR[p], Ro);
            V3 t = TP[p] + mul(TR[p], v3(o[9], o[10], o[11]));
            float *cx = c + CL::xtree(g) * N + e;
#pragma unroll
            for (int k = 0; k < 9; ++k) cx[k * N] = R.a[k];
            cx[9 * N] = t.x; cx[10 * N] = t.y; cx[11 * N] = t.z;
        }
    }
#pragma unroll
    for (int s = 0; s < M::NS; ++s) {
        const int l = M::shape_link[s];
        const float *o = M::shape_pose[s];
        M3 Ro{{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]}};
        M3 R = mul(TR[l], Ro);
        V3 t = TP[l] + mul(TR[l], v3(o[9], o[10], o[11]));
        float *cs = c + CL::shape(s) * N + e;
#pragma unroll
        for (int k = 0; k < 9; ++k) cs[k * N] = R.a[k];
        cs[9 * N] = t.x; cs[10 * N] = t.y; cs[11 * N] = t.z;
    }
    a.dirty[e] = 0;
}

// ---------------------------------------------------------------- step
struct Row {
    V3 r;        // application point in group frame (linear rows)
    V3 d;        // world direction / axis
    float target;
    float on;    // 1 active, 0 inactive
};

template <class M> struct Work {
    Xf X[M::NG];
    M3 Rw[M::NG];
    V3 pw[M::NG];
    SV c[M::NG];
    SI IA[M::NG];
    SV pA[M::NG];
    SV U[M::NG];
    float Dinv[M::NG];
    float u[M::NG];
    LDL6 root;
};

template <class M>
__device__ __forceinline__ void group_vels(const Work<M> &w, const float *qd, const SV &v0, SV *vg) {
    vg[0] = v0;
#pragma unroll
    for (int g = 1; g < M::NG; ++g) {
        SV S = M::jtype[g] == TG_JOINT_REVOLUTE ? SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)}
                                               : SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
        vg[g] = xmotion(w.X[g], vg[M::parent[g]]) + qd[g] * S;
    }
}

// impulse response: spatial impulses fi (group frames) -> dqd (per group), dv0
template <class M>
__device__ __forceinline__ void impulse_response(const Work<M> &w, bool fix_base, const SV *fi, float *dqd, SV &dv0) {
    SV p[M::NG];
#pragma unroll
    for (int g = 0; g < M::NG; ++g) p[g] = -1.0f * fi[g];
    float u[M::NG];
#pragma unroll
    for (int g = M::NG - 1; g >= 1; --g) {
        SV S = M::jtype[g] == TG_JOINT_REVOLUTE ? SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)}
                                               : SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
        u[g] = -dot(S, p[g]);
        SV pa = p[g] + (u[g] * w.Dinv[g]) * w.U[g];
        p[M::parent[g]] = p[M::parent[g]] + xTforce(w.X[g], pa);
    }
    SV a[M::NG];
    a[0] = fix_base ? sv0() : ldl6_solve(w.root, -1.0f * p[0]);
    dv0 = a[0];
    dqd[0] = 0.f;
#pragma unroll
    for (int g = 1; g < M::NG; ++g) {
        SV S = M::jtype[g] == TG_JOINT_REVOLUTE ? SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)}
                                               : SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
        SV ap = xmotion(w.X[g], a[M::parent[g]]);
        float x = (u[g] - dot(w.U[g], ap)) * w.Dinv[g];
        dqd[g] = x;
        a[g] = ap + x * S;
    }
}

template <class M> __device__ __forceinline__ constexpr int row_shape(int i) {
    int base = 0;
    for (int s = 0; s < M::NS; ++s) {
        if (i < base + M::shape_nrows[s] + 3) return s;
        base += M::shape_nrows[s] + 3;
    }
    return 0;
}
template <class M> __device__ __forceinline__ constexpr int row_base(int s) {
    int base = 0;
    for (int k = 0; k < s; ++k) base += M::shape_nrows[k] + 3;
    return base;
}

template <class M>
__device__ __forceinline__ float row_vel(const Work<M> &w, int g, bool angular, const Row &r, const SV &vg) {
    V3 o = angular ? mul(w.Rw[g], vg.w) : mul(w.Rw[g], vg.v + cross(vg.w, r.r));
    return dot(o, r.d);
}
template <class M>
__device__ __forceinline__ SV row_force(const Work<M> &w, int g, bool angular, const Row &r, float lam) {
    V3 dl = mulT(w.Rw[g], r.d);
    return angular ? SV{lam * dl, v3(0, 0, 0)} : SV{lam * cross(r.r, dl), lam * dl};
}

template <class M> __global__ __launch_bounds__(64) void step_kernel(StepArgs a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.N) return;
    using CL = CompLayout<M>;
    const size_t N = a.N;
    const int D = a.D;
    const float h = a.h;
    const bool fix_base = a.fix_base != 0;
    const float *comp = a.comp;
    auto CP = [&](int k) { return comp[(size_t)k * N + e]; };

    // ---- load state
    float *root = a.root + (size_t)e * 13;
    float *dofs = a.dof + (size_t)e * D * 2;
    float q[M::NG], qd[M::NG];
    q[0] = qd[0] = 0.f;
#pragma unroll
    for (int g = 1; g < M::NG; ++g) {
        q[g] = dofs[2 * M::gdof[g]];
        qd[g] = dofs[2 * M::gdof[g] + 1];
    }
    V3 pos = v3(root[0], root[1], root[2]);
    float qx = root[3], qy = root[4], qz = root[5], qw = root[6];
    {
        float in = rsqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
        qx *= in; qy *= in; qz *= in; qw *= in;
    }
    M3 R = quat_to_m3(qx, qy, qz, qw);
    const V3 c0 = v3(M::root_com[0], M::root_com[1], M::root_com[2]);
    V3 ww = v3(root[10], root[11], root[12]);
    V3 vo = v3(root[7], root[8], root[9]) - cross(ww, mul(R, c0));
    SV v0 = fix_base ? sv0() : SV{mulT(R, ww), mulT(R, vo)};
    const V3 grav = v3(a.gx, a.gy, a.gz);

    Work<M> w;
    for (int sub = 0; sub < a.substeps; ++sub) {
        // ---- pass 1: kinematics, velocities, bias forces
        w.Rw[0] = R;
        w.pw[0] = pos;
        SV v[M::NG];
        v[0] = v0;
        w.c[0] = sv0();
#pragma unroll
        for (int g = 0; g < M::NG; ++g) {
            if (g > 0) {
                const int p = M::parent[g];
                M3 Rpc;
                V3 t;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rpc.a[k] = CP(CL::xtree(g) + k);
                t = v3(CP(CL::xtree(g) + 9), CP(CL::xtree(g) + 10), CP(CL::xtree(g) + 11));
                SV S;
                if (M::jtype[g] == TG_JOINT_REVOLUTE) {
                    Rpc = mul(Rpc, rot_axis(M::axis[g][0], M::axis[g][1], M::axis[g][2], q[g]));
                    S = SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)};
                } else {
                    t = t + q[g] * mul(Rpc, v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]));
                    S = SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
                }
                w.X[g].E = transpose(Rpc);
                w.X[g].r = t;
                SV vJ = qd[g] * S;
                v[g] = xmotion(w.X[g], v[p]) + vJ;
                w.c[g] = crm(v[g], vJ);
                w.Rw[g] = mul(w.Rw[p], Rpc);
                w.pw[g] = w.pw[p] + mul(w.Rw[p], t);
            }
            const float m = CP(CL::inertia(g));
            const V3 cg = v3(CP(CL::inertia(g) + 1), CP(CL::inertia(g) + 2), CP(CL::inertia(g) + 3));
            float Ic[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) Ic[k] = CP(CL::inertia(g) + 4 + k);
            w.IA[g] = rb_inertia(m, cg, Ic);
            SV b = crf(v[g], mul(w.IA[g], v[g]));
            V3 F = m * mulT(w.Rw[g], grav);
            F = F - (a.lin_damp * m) * (v[g].v + cross(v[g].w, cg));
            V3 n = cross(cg, F) - a.ang_damp * symmul(Ic, v[g].w);
            if (a.force) {
                const float *fw = a.force + ((size_t)e * M::NG + g) * 6;
                V3 fl = mulT(w.Rw[g], v3(fw[0], fw[1], fw[2])), tl = mulT(w.Rw[g], v3(fw[3], fw[4], fw[5]));
                F = F + fl;
                n = n + tl + cross(cg, fl);
            }
            w.pA[g] = SV{b.w - n, b.v - F};
        }
        // ---- pass 2: articulated inertias, implicit drives / limits
#pragma unroll
        for (int g = M::NG - 1; g >= 1; --g) {
            const int p = M::parent[g], d = M::gdof[g];
            SV S = M::jtype[g] == TG_JOINT_REVOLUTE ? SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)}
                                                   : SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
            w.U[g] = mul(w.IA[g], S);
            const float D0 = dot(S, w.U[g]) + prop(a, TG_PROP_ARMATURE, e, d);
            float Dimp = 0.f, tau = 0.f;
            const int mode = (int)rintf(prop(a, TG_PROP_DRIVE_MODE, e, d));
            const float kp = prop(a, TG_PROP_STIFFNESS, e, d), kd = prop(a, TG_PROP_DAMPING, e, d);
            const float eff = prop(a, TG_PROP_EFFORT, e, d);
            if (mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL) {
                const float te = kp * (a.pos_tgt[(size_t)e * D + d] - q[g] - h * qd[g]) + kd * (a.vel_tgt[(size_t)e * D + d] - qd[g]);
                if (fabsf(te) <= eff) { tau += te; Dimp += h * kd + h * h * kp; }
                else tau += te > 0.f ? eff : -eff;
            } else if (mode == TG_DOF_MODE_EFFORT && a.act) {
                tau += fminf(fmaxf(a.act[(size_t)e * D + d], -eff), eff);
            }
            const float lo = prop(a, TG_PROP_LOWER, e, d), hi = prop(a, TG_PROP_UPPER, e, d);
            const float qp = q[g] + h * qd[g];
            const float kl = a.lim_k * D0 / (h * h), cl = a.lim_c * D0 / h;
            if (qp < lo && lo > -1e30f) { tau += kl * (lo - qp) - cl * qd[g]; Dimp += h * cl + h * h * kl; }
            else if (qp > hi && hi < 1e30f) { tau += kl * (hi - qp) - cl * qd[g]; Dimp += h * cl + h * h * kl; }
            const float Dt = D0 + Dimp;
            w.Dinv[g] = 1.0f / Dt;
            w.u[g] = tau - dot(S, w.pA[g]);
            SI Ia = w.IA[g];
            si_sub_outer(Ia, w.U[g], w.Dinv[g]);
            SV pa = w.pA[g] + mul(Ia, w.c[g]) + (w.u[g] * w.Dinv[g]) * w.U[g];
            si_add(w.IA[p], si_to_parent(Ia, w.X[g]));
            w.pA[p] = w.pA[p] + xTforce(w.X[g], pa);
        }
        // ---- pass 3: accelerations -> free velocities
        SV acc[M::NG];
        if (!fix_base) w.root = ldl6(w.IA[0]);
        acc[0] = fix_base ? sv0() : ldl6_solve(w.root, -1.0f * w.pA[0]);
        float qds[M::NG];
        qds[0] = 0.f;
#pragma unroll
        for (int g = 1; g < M::NG; ++g) {
            SV S = M::jtype[g] == TG_JOINT_REVOLUTE ? SV{v3(M::axis[g][0], M::axis[g][1], M::axis[g][2]), v3(0, 0, 0)}
                                                   : SV{v3(0, 0, 0), v3(M::axis[g][0], M::axis[g][1], M::axis[g][2])};
            SV ap = xmotion(w.X[g], acc[M::parent[g]]) + w.c[g];
            float qdd = (w.u[g] - dot(w.U[g], ap)) * w.Dinv[g];
            acc[g] = ap + qdd * S;
            qds[g] = qd[g] + h * qdd;
        }
        SV v0s = v0 + h * acc[0];
        v0s.v = v0s.v + h * cross(v0.w, v0.v);
        if (fix_base) v0s = sv0();

        // ---- 4. contacts
        if constexpr (M::NS > 0) {
            constexpr int K = M::NROWS;
            Row rows[K];
            float mu_p[M::NSA], reff[M::NSA];
#pragma unroll
            for (int s = 0; s < M::NS; ++s) {
                const int g = M::shape_group[s];
                const int rb = row_base<M>(s);
                M3 Rs, Rsl;
#pragma unroll
                for (int k = 0; k < 9; ++k) Rsl.a[k] = CP(CL::shape(s) + k);
                Rs = mul(w.Rw[g], Rsl);
                V3 cl = v3(CP(CL::shape(s) + 9), CP(CL::shape(s) + 10), CP(CL::shape(s) + 11));
                V3 cw = w.pw[g] + mul(w.Rw[g], cl);
                V3 pts[4];
                if (M::shape_kind[s] == TG_SHAPE_TORUS) {
                    V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                    V3 dd = v3(-ax.z * ax.x, -ax.z * ax.y, 1.f - ax.z * ax.z);
                    float nd = sqrtf(dot(dd, dd));
                    if (nd < 1e-6f) { dd = v3(1, 0, 0); nd = 1.f; }
                    pts[0] = cw - (M::shape_params[s][0] / nd) * dd - v3(0, 0, M::shape_params[s][1]);
                } else if (M::shape_kind[s] == TG_SHAPE_SPHERE) {
                    pts[0] = cw - v3(0, 0, M::shape_params[s][0]);
                } else {
                    // box: the 4 corners of the face whose outward normal points most downward
                    const float hx = M::shape_params[s][0], hy = M::shape_params[s][1], hz = M::shape_params[s][2];
                    const float zx = Rs.a[6], zy = Rs.a[7], zz = Rs.a[8];
                    const float ax_ = fabsf(zx), ay_ = fabsf(zy), az_ = fabsf(zz);
                    V3 ex = v3(Rs.a[0], Rs.a[3], Rs.a[6]), ey = v3(Rs.a[1], Rs.a[4], Rs.a[7]), ez = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
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
#pragma unroll
                for (int k = 0; k < M::shape_nrows[s]; ++k) {
                    Row &r = rows[rb + k];
                    const float phi = pts[k].z;
                    r.on = phi <= a.margin ? 1.f : 0.f;
                    r.r = mulT(w.Rw[g], pts[k] - w.pw[g]);
                    r.d = v3(0, 0, 1);
                    const float rest = a.rest;
                    r.target = phi > rest ? -(phi - rest) / h : fminf(a.baumgarte * (rest - phi) / h, a.max_depen);
                    cen = cen + r.on * pts[k];
                    nact += r.on;
                }
                cen = (nact > 0.f ? 1.f / nact : 0.f) * cen;
                float re = 0.f;
#pragma unroll
                for (int k = 0; k < M::shape_nrows[s]; ++k) {
                    float dx = pts[k].x - cen.x, dy = pts[k].y - cen.y;
                    re += rows[rb + k].on * sqrtf(dx * dx + dy * dy);
                }
                reff[s] = nact > 0.f ? re / nact : 0.f;
                mu_p[s] = 0.5f * (a.shape_mu[(size_t)e * M::NS + s] + a.ground_mu);
                V3 t1 = v3(1, 0, 0);
                if (M::shape_kind[s] == TG_SHAPE_TORUS) {
                    V3 ax = v3(Rs.a[2], Rs.a[5], Rs.a[8]);
                    V3 x = cross(ax, v3(0, 0, 1));
                    float nx = sqrtf(dot(x, x));
                    if (nx > 1e-6f) t1 = (1.f / nx) * x;
                }
                V3 t2 = cross(v3(0, 0, 1), t1);
                V3 rl = mulT(w.Rw[g], cen - w.pw[g]);
                const int f0 = rb + M::shape_nrows[s];
                rows[f0] = Row{rl, t1, 0.f, nact > 0.f ? 1.f : 0.f};
                rows[f0 + 1] = Row{rl, t2, 0.f, nact > 0.f ? 1.f : 0.f};
                rows[f0 + 2] = Row{rl, v3(0, 0, 1), 0.f, nact > 0.f ? 1.f : 0.f};
            }
            // free row velocities
            float vfree[K], lam[K], W[K][K];
            {
                SV vg[M::NG];
                group_vels<M>(w, qds, v0s, vg);
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const int s = row_shape<M>(i);
                    const bool ang = (i == row_base<M>(s) + M::shape_nrows[s] + 2);
                    vfree[i] = row_vel<M>(w, M::shape_group[s], ang, rows[i], vg[M::shape_group[s]]);
                    lam[i] = 0.f;
                }
            }
            // Delassus columns by impulse response
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const int sj = row_shape<M>(j);
                const int gj = M::shape_group[sj];
                const bool angj = (j == row_base<M>(sj) + M::shape_nrows[sj] + 2);
                SV fi[M::NG];
#pragma unroll
                for (int g = 0; g < M::NG; ++g) fi[g] = sv0();
                fi[gj] = row_force<M>(w, gj, angj, rows[j], 1.0f);
                float dqd[M::NG];
                SV dv0, dvg[M::NG];
                impulse_response<M>(w, fix_base, fi, dqd, dv0);
                group_vels<M>(w, dqd, dv0, dvg);
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    const int si = row_shape<M>(i);
                    const bool angi = (i == row_base<M>(si) + M::shape_nrows[si] + 2);
                    W[i][j] = row_vel<M>(w, M::shape_group[si], angi, rows[i], dvg[M::shape_group[si]]);
                }
            }
            // projected Gauss-Seidel, patch friction
            for (int it = 0; it < a.iters; ++it) {
#pragma unroll
                for (int s = 0; s < M::NS; ++s) {
                    const int rb = row_base<M>(s);
                    float Nsum = 0.f;
#pragma unroll
                    for (int k = 0; k < M::shape_nrows[s]; ++k) {
                        const int i = rb + k;
                        float vi = vfree[i];
#pragma unroll
                        for (int j = 0; j < K; ++j) vi += W[i][j] * lam[j];
                        float l = lam[i] + (rows[i].target - vi) / W[i][i];
                        lam[i] = rows[i].on * fmaxf(l, 0.f);
                        Nsum += lam[i];
                    }
                    const int f = rb + M::shape_nrows[s];
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
                        float vi = vfree[f + t];
#pragma unroll
                        for (int j = 0; j < K; ++j) vi += W[f + t][j] * lam[j];
                        lam[f + t] -= vi / W[f + t][f + t];
                        if (t == 1) {
                            float lt = sqrtf(lam[f] * lam[f] + lam[f + 1] * lam[f + 1]), lim = mu_p[s] * Nsum;
                            float sc = lt > lim ? (lt > 0.f ? lim / lt : 0.f) : 1.f;
                            lam[f] *= sc;
                            lam[f + 1] *= sc;
                        }
                    }
                    const float lim3 = mu_p[s] * Nsum * reff[s];
                    lam[f + 2] = fminf(fmaxf(lam[f + 2], -lim3), lim3);
                }
            }
            // apply the impulses
            SV fi[M::NG];
#pragma unroll
            for (int g = 0; g < M::NG; ++g) fi[g] = sv0();
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const int s = row_shape<M>(i);
                const int g = M::shape_group[s];
                const bool ang = (i == row_base<M>(s) + M::shape_nrows[s] + 2);
                fi[g] = fi[g] + row_force<M>(w, g, ang, rows[i], lam[i]);
            }
            float dqd[M::NG];
            SV dv0;
            impulse_response<M>(w, fix_base, fi, dqd, dv0);
#pragma unroll
            for (int g = 1; g < M::NG; ++g) qds[g] += dqd[g];
            if (!fix_base) v0s = v0s + dv0;
        }
        // ---- 5. velocity limits + integration
#pragma unroll
        for (int g = 1; g < M::NG; ++g) {
            const float vl = prop(a, TG_PROP_VELOCITY, e, M::gdof[g]);
            float x = qds[g];
            if (vl > 0.f) x = fminf(fmaxf(x, -vl), vl);
            qd[g] = x;
            q[g] += h * x;
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
                float k = sa / wn;
                dx = v0.w.x * k; dy = v0.w.y * k; dz = v0.w.z * k; dw = ca;
            }
            float nx = qw * dx + qx * dw + qy * dz - qz * dy;
            float ny = qw * dy - qx * dz + qy * dw + qz * dx;
            float nz = qw * dz + qx * dy - qy * dx + qz * dw;
            float nw = qw * dw - qx * dx - qy * dy - qz * dz;
            float in = rsqrtf(nx * nx + ny * ny + nz * nz + nw * nw);
            qx = nx * in; qy = ny * in; qz = nz * in; qw = nw * in;
            R = quat_to_m3(qx, qy, qz, qw);
            M3 Rd = quat_to_m3(dx, dy, dz, dw);
            v0.w = mulT(Rd, v0.w);
            v0.v = mulT(Rd, v0.v);
        }
    }
    // ---- write back
    V3 wwo = mul(R, v0.w);
    V3 vco = mul(R, v0.v) + cross(wwo, mul(R, c0));
    root[0] = pos.x; root[1] = pos.y; root[2] = pos.z;
    root[3] = qx; root[4] = qy; root[5] = qz; root[6] = qw;
    root[7] = vco.x; root[8] = vco.y; root[9] = vco.z;
    root[10] = wwo.x; root[11] = wwo.y; root[12] = wwo.z;
#pragma unroll
    for (int g = 1; g < M::NG; ++g) {
        dofs[2 * M::gdof[g]] = q[g];
        dofs[2 * M::gdof[g] + 1] = qd[g];
    }
#pragma unroll
    for (int d = 0; d < M::ND; ++d) {
        if (M::dof_locked[d]) {
            dofs[2 * d] = 0.5f * (prop(a, TG_PROP_LOWER, e, d) + prop(a, TG_PROP_UPPER, e, d));
            dofs[2 * d + 1] = 0.f;
        }
    }
}

}  // namespace tg

#include "step_par.h"

namespace tg {

// ---------------------------------------------------------------- dispatch
// Small trees: fully unrolled register-resident step_kernel, 64 envs/block.
// Large trees (M::use_lds): tree-parallel LDS-resident step_par_kernel,
// LDS_EPB envs x M::LPE lanes per block (Thormang: 16 envs, 151 KB of LDS).
constexpr int LDS_EPB = 16;

template <class M> int launch_model(const StepArgs &a, hipStream_t stream) {
    const dim3 cgrid((a.N + 63) / 64), cblock(64);
    hipLaunchKernelGGL(compose_kernel<M>, cgrid, cblock, 0, stream, a);
    if constexpr (M::use_lds) {
        constexpr size_t bytes = ParLayout<M>::template bytes<LDS_EPB>();
        static_assert(bytes <= 160 * 1024, "LDS budget");
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute((const void *)step_par_kernel<M, LDS_EPB>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
                return TG_ERR_HIP;
            attr = true;
        }
        hipLaunchKernelGGL((step_par_kernel<M, LDS_EPB>), dim3((a.N + LDS_EPB - 1) / LDS_EPB), dim3(LDS_EPB * M::LPE),
                           bytes, stream, a);
    } else {
        hipLaunchKernelGGL(step_kernel<M>, cgrid, cblock, 0, stream, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

#define TG_LAUNCH(MODEL) \
    if (hash == MODEL::hash) return launch_model<MODEL>(a, stream);

int launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream) {
    TG_FOR_EACH_MODEL(TG_LAUNCH)
    return TG_ERR_MODEL;
}

#define TG_COMPOSE(MODEL)                                                                     \
    if (hash == MODEL::hash) {                                                                \
        dim3 grid((a.N + 63) / 64), block(64);                                                \
        hipLaunchKernelGGL(compose_kernel<MODEL>, grid, block, 0, stream, a);                 \
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;                              \
    }

int launch_compose(uint64_t hash, const StepArgs &a, hipStream_t stream) {
    TG_FOR_EACH_MODEL(TG_COMPOSE)
    return TG_ERR_MODEL;
}

#ifdef TG_SECTION_PROF
extern "C" int tg_prof_read(unsigned long long *out, int n) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_prof_acc), sizeof(unsigned long long) * (n < 16 ? n : 16)) != hipSuccess)
        return -1;
    return 0;
}
#endif

#define TG_HASH(MODEL) if (n < cap) out[n] = MODEL::hash; ++n;
#define TG_KC(MODEL) if (hash == MODEL::hash) return MODEL::KC;

int compiled_hashes(uint64_t *out, int cap) {
    int n = 0;
    TG_FOR_EACH_MODEL(TG_HASH)
    return n;
}
int model_kc(uint64_t hash) {
    TG_FOR_EACH_MODEL(TG_KC)
    return -1;
}

}  // namespace tg
