/*
 * oracle/physics_ref.c -- fp64 CPU restatement of the articulated-body step.
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for the HIP step kernel
 * (thormang_isaacgym_amd/csrc/articulation.hip) and the cpu_baseline leg of
 * bench.py.  The product path never loads it.
 *
 * PARITY STATUS.  The reference's physics is the closed IsaacGym/PhysX binary
 * (gym.simulate, isaacgymenvs/tasks/base/vec_task.py:335), absent from
 * /root/reference and unavailable offline: physics parity with
 * PhysX is UNPINNED.  This file restates the algorithm the build implements
 * (Featherstone articulated-body algorithm over the URDF joint tree, implicit
 * joint-space PD drives, implicit limit springs, speculative velocity-level
 * ground contact solved by projected Gauss-Seidel, semi-implicit Euler) from
 * the published algorithm (Featherstone, "Rigid Body Dynamics Algorithms",
 * 2008, ch. 2, 7, 9) with the reference's parameters.  It
 * is pinned by analytic known-answer tests in tests/test_physics_oracle.py
 * (free fall, pendulum period, torque-free momentum/energy, drive steady
 * state, resting contact).  It deliberately uses a different data layout from
 * the HIP kernel: dense 6x6 double matrices, table-driven loops, no
 * specialisation.
 *
 * Spatial conventions: motion [w; v], force [n; f]; X = child-from-parent.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/tgsim.h"

#define MAXG 64
#define MAXL 96
#define MAXD 64
#define MAXC 32

#ifdef ORACLE_REAL_F32
/* fp32 build (oracle/_build/liboracle_f32.so, drift study scripts/parity_drift.py):
 * every quantity stored and evaluated in float (with -fsingle-precision-constant
 * and the float math functions), the same operation order */
#define sqrt sqrtf
#define sin sinf
#define cos cosf
#define fabs fabsf
#define exp expf
typedef float real;
#else
typedef double real;
#endif
typedef real V3[3];
typedef real M3[9];
typedef real V6[6];
typedef real M6[36];

static void m3_mul(const M3 a, const M3 b, M3 o) {
    M3 t;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
    memcpy(o, t, sizeof t);
}
static void m3_T(const M3 a, M3 o) {
    M3 t;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = a[3 * j + i];
    memcpy(o, t, sizeof t);
}
static void m3_v(const M3 a, const V3 v, V3 o) {
    V3 t = {a[0] * v[0] + a[1] * v[1] + a[2] * v[2], a[3] * v[0] + a[4] * v[1] + a[5] * v[2],
            a[6] * v[0] + a[7] * v[1] + a[8] * v[2]};
    memcpy(o, t, sizeof t);
}
static void m3T_v(const M3 a, const V3 v, V3 o) {
    V3 t = {a[0] * v[0] + a[3] * v[1] + a[6] * v[2], a[1] * v[0] + a[4] * v[1] + a[7] * v[2],
            a[2] * v[0] + a[5] * v[1] + a[8] * v[2]};
    memcpy(o, t, sizeof t);
}
static void cross3(const V3 a, const V3 b, V3 o) {
    V3 t = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    memcpy(o, t, sizeof t);
}
static real dot3(const V3 a, const V3 b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void axis_angle(const V3 a, real q, M3 R) {
    real c = cos(q), s = sin(q), t = 1 - c, x = a[0], y = a[1], z = a[2];
    R[0] = t * x * x + c; R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
    R[3] = t * x * y + s * z; R[4] = t * y * y + c; R[5] = t * y * z - s * x;
    R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}
static void quat_to_m3(const real *q, M3 R) {   /* xyzw, body->world */
    real x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}

/* ---------------------------------------------------------------- spatial */
typedef struct { M3 E; V3 r; } Xform;   /* child-from-parent: E parent->child coords, r child origin in parent */

static void X_motion(const Xform *X, const V6 v, V6 o) {   /* o = X v */
    V3 w = {v[0], v[1], v[2]}, lin = {v[3], v[4], v[5]}, rxw, t;
    cross3(X->r, w, rxw);
    for (int k = 0; k < 3; ++k) t[k] = lin[k] - rxw[k];
    V3 ow, ol;
    m3_v(X->E, w, ow);
    m3_v(X->E, t, ol);
    o[0] = ow[0]; o[1] = ow[1]; o[2] = ow[2]; o[3] = ol[0]; o[4] = ol[1]; o[5] = ol[2];
}
static void XT_force(const Xform *X, const V6 f, V6 o) {   /* o = X^T f  (child force -> parent) */
    V3 n = {f[0], f[1], f[2]}, fl = {f[3], f[4], f[5]}, En, Ef, rxf;
    m3T_v(X->E, n, En);
    m3T_v(X->E, fl, Ef);
    cross3(X->r, Ef, rxf);
    o[0] = En[0] + rxf[0]; o[1] = En[1] + rxf[1]; o[2] = En[2] + rxf[2];
    o[3] = Ef[0]; o[4] = Ef[1]; o[5] = Ef[2];
}
static void X_dense(const Xform *X, M6 M) {   /* dense motion transform */
    memset(M, 0, sizeof(M6));
    real rx[9] = {0, -X->r[2], X->r[1], X->r[2], 0, -X->r[0], -X->r[1], X->r[0], 0};
    M3 Erx;
    m3_mul(X->E, rx, Erx);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            M[6 * i + j] = X->E[3 * i + j];
            M[6 * (i + 3) + j + 3] = X->E[3 * i + j];
            M[6 * (i + 3) + j] = -Erx[3 * i + j];
        }
}
static void m6_v(const M6 A, const V6 v, V6 o) {
    V6 t;
    for (int i = 0; i < 6; ++i) {
        real s = 0;
        for (int j = 0; j < 6; ++j) s += A[6 * i + j] * v[j];
        t[i] = s;
    }
    memcpy(o, t, sizeof t);
}
static void crm(const V6 v, const V6 m, V6 o) {   /* v x m */
    V3 w = {v[0], v[1], v[2]}, vl = {v[3], v[4], v[5]}, mw = {m[0], m[1], m[2]}, ml = {m[3], m[4], m[5]}, a, b, c;
    cross3(w, mw, a);
    cross3(w, ml, b);
    cross3(vl, mw, c);
    o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = b[0] + c[0]; o[4] = b[1] + c[1]; o[5] = b[2] + c[2];
}
static void crf(const V6 v, const V6 f, V6 o) {   /* v x* f */
    V3 w = {v[0], v[1], v[2]}, vl = {v[3], v[4], v[5]}, fn = {f[0], f[1], f[2]}, ff = {f[3], f[4], f[5]}, a, b, c;
    cross3(w, fn, a);
    cross3(vl, ff, b);
    cross3(w, ff, c);
    o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2]; o[3] = c[0]; o[4] = c[1]; o[5] = c[2];
}
/* rigid-body spatial inertia at frame origin from mass, com, rotational inertia about com (3x3) */
static void rb_inertia(real m, const V3 c, const M3 Ic, M6 I) {
    memset(I, 0, sizeof(M6));
    real cx[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    M3 cxcxT;
    real cxT[9];
    m3_T(cx, cxT);
    m3_mul(cx, cxT, cxcxT);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            I[6 * i + j] = Ic[3 * i + j] + m * cxcxT[3 * i + j];
            I[6 * i + j + 3] = m * cx[3 * i + j];
            I[6 * (i + 3) + j] = m * cxT[3 * i + j];
            I[6 * (i + 3) + j + 3] = (i == j) ? m : 0;
        }
}
/* solve 6x6 SPD system by Gaussian elimination with partial pivoting */
static void solve6(const M6 A, const V6 b, V6 x) {
    real M[6][7];
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) M[i][j] = A[6 * i + j];
        M[i][6] = b[i];
    }
    for (int c = 0; c < 6; ++c) {
        int p = c;
        for (int r = c + 1; r < 6; ++r)
            if (fabs(M[r][c]) > fabs(M[p][c])) p = r;
        if (p != c)
            for (int k = 0; k < 7; ++k) { real t = M[c][k]; M[c][k] = M[p][k]; M[p][k] = t; }
        for (int r = c + 1; r < 6; ++r) {
            real f = M[r][c] / M[c][c];
            for (int k = c; k < 7; ++k) M[r][k] -= f * M[c][k];
        }
    }
    for (int r = 5; r >= 0; --r) {
        real s = M[r][6];
        for (int k = r + 1; k < 6; ++k) s -= M[r][k] * x[k];
        x[r] = s / M[r][r];
    }
}

/* ---------------------------------------------------------------- per-env workspace */
typedef struct {
    /* composite (per env, from locked positions + mass scale) */
    real gm[MAXG];
    V3 gc[MAXG];
    M3 gI[MAXG];
    M3 xtR[MAXG];      /* joint origin of each group, in parent group frame */
    V3 xtp[MAXG];
    V3 gaxis[MAXG];    /* joint axis in group frame */
    int gtype[MAXG];
    int gdof[MAXG];
    M3 shR[MAXC];      /* shape pose in its group frame */
    V3 shp[MAXC];
    int shg[MAXC];
    /* per substep */
    Xform X[MAXG];
    M3 Rw[MAXG];
    V3 pw[MAXG];            /* group origins relative to the root origin (world-oriented) */
    V3 org;                 /* the root origin in the world */
    V6 v[MAXG], c[MAXG], pA[MAXG], U[MAXG], S[MAXG];
    M6 IA[MAXG];
    real D[MAXG], u[MAXG];
} Work;

/* compose: per-env group composites (tgsim.h model grouping). lockq[D] = locked positions. */
static void compose(const tg_model_desc *m, const real *lockq, const float *mass_scale, Work *w) {
    M3 TR[MAXL];
    V3 Tp[MAXL];
    int G = m->num_groups;
    for (int g = 0; g < G; ++g) {
        w->gm[g] = 0;
        memset(w->gc[g], 0, sizeof(V3));
        memset(w->gI[g], 0, sizeof(M3));
    }
    /* pass A: link poses in group frames, mass and first moment */
    for (int l = 0; l < m->num_links; ++l) {
        int g = m->link_group[l];
        if (m->group_root[g] == l) {
            M3 I = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            memcpy(TR[l], I, sizeof I);
            memset(Tp[l], 0, sizeof(V3));
        } else {
            int p = m->link_parent[l];
            const float *o = m->link_origin + 12 * l;
            M3 Ro, Rj;
            V3 to = {o[9], o[10], o[11]}, ax = {m->link_axis[3 * l], m->link_axis[3 * l + 1], m->link_axis[3 * l + 2]};
            for (int k = 0; k < 9; ++k) Ro[k] = o[k];
            int d = m->link_dof[l];
            real q = d >= 0 ? lockq[d] : 0.0;
            if (m->link_jtype[l] == TG_JOINT_REVOLUTE) {
                axis_angle(ax, q, Rj);
                m3_mul(Ro, Rj, Ro);
            } else if (m->link_jtype[l] == TG_JOINT_PRISMATIC) {
                V3 s;
                m3_v(Ro, ax, s);
                for (int k = 0; k < 3; ++k) to[k] += s[k] * q;
            }
            /* T_l = T_p * (Ro, to) */
            m3_mul(TR[p], Ro, TR[l]);
            V3 t;
            m3_v(TR[p], to, t);
            for (int k = 0; k < 3; ++k) Tp[l][k] = Tp[p][k] + t[k];
        }
        const float *in = m->link_inertia + 10 * l;
        real s = mass_scale ? mass_scale[l] : 1.0;
        real ml = in[0] * s;
        V3 cl = {in[1], in[2], in[3]}, cg;
        m3_v(TR[l], cl, cg);
        for (int k = 0; k < 3; ++k) cg[k] += Tp[l][k];
        w->gm[g] += ml;
        for (int k = 0; k < 3; ++k) w->gc[g][k] += ml * cg[k];
    }
    for (int g = 0; g < G; ++g)
        if (w->gm[g] > 0)
            for (int k = 0; k < 3; ++k) w->gc[g][k] /= w->gm[g];
    /* pass B: rotational inertia about group com */
    for (int l = 0; l < m->num_links; ++l) {
        int g = m->link_group[l];
        const float *in = m->link_inertia + 10 * l;
        real s = mass_scale ? mass_scale[l] : 1.0;
        real ml = in[0] * s;
        M3 Il = {in[4] * s, in[7] * s, in[8] * s, in[7] * s, in[5] * s, in[9] * s, in[8] * s, in[9] * s, in[6] * s};
        M3 RI, RIRt, RT;
        m3_mul(TR[l], Il, RI);
        m3_T(TR[l], RT);
        m3_mul(RI, RT, RIRt);
        V3 cl = {in[1], in[2], in[3]}, cg;
        m3_v(TR[l], cl, cg);
        V3 dd;
        for (int k = 0; k < 3; ++k) dd[k] = cg[k] + Tp[l][k] - w->gc[g][k];
        real d2 = dot3(dd, dd);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                w->gI[g][3 * i + j] += RIRt[3 * i + j] + ml * ((i == j ? d2 : 0) - dd[i] * dd[j]);
    }
    /* joint placements and axes of active joints */
    for (int g = 0; g < G; ++g) {
        int r = m->group_root[g];
        w->gdof[g] = m->link_dof[r];
        w->gtype[g] = (g == 0) ? -1 : m->link_jtype[r];
        for (int k = 0; k < 3; ++k) w->gaxis[g][k] = m->link_axis[3 * r + k];
        if (g == 0) continue;
        int p = m->link_parent[r];
        const float *o = m->link_origin + 12 * r;
        M3 Ro;
        for (int k = 0; k < 9; ++k) Ro[k] = o[k];
        V3 to = {o[9], o[10], o[11]}, t;
        m3_mul(TR[p], Ro, w->xtR[g]);
        m3_v(TR[p], to, t);
        for (int k = 0; k < 3; ++k) w->xtp[g][k] = Tp[p][k] + t[k];
    }
    for (int s = 0; s < m->num_shapes; ++s) {
        int l = m->shape_link[s];
        const float *o = m->shape_pose + 12 * s;
        M3 Ro;
        for (int k = 0; k < 9; ++k) Ro[k] = o[k];
        V3 to = {o[9], o[10], o[11]}, t;
        m3_mul(TR[l], Ro, w->shR[s]);
        m3_v(TR[l], to, t);
        for (int k = 0; k < 3; ++k) w->shp[s][k] = Tp[l][k] + t[k];
        w->shg[s] = m->link_group[l];
    }
}

typedef struct {
    const tg_model_desc *m;
    const tg_sim_params *sp;
    const float *props;       /* [TG_NUM_PROPS][D] for this env (strided) */
    long prop_stride;         /* stride between prop fields */
    const float *pos_tgt, *vel_tgt, *act;
    const float *force;       /* [G,6] world wrench at group com or NULL */
    const float *mu;          /* [S] shape friction for this env */
    real g[3];
} Env;

static real prop(const Env *e, int f, int d) { return e->props[f * e->prop_stride + d]; }

/* ABA pass 1+2+3 with the given generalised state; fills qdd (dof-indexed) and a0.
 * Position/velocity drives are implicit (h*kd + h^2*kp folded into D).  Effort
 * limits follow "implicit, then clamp" (the drive impulse of an implicit solver
 * clamped to effort*h): with qdd_prev == NULL every drive is implicit and
 * unclamped; with the accelerations of that first solve, a drive whose implicit
 * end-of-substep torque te - K*qdd exceeds its effort becomes the explicit
 * torque +-effort (continuous at the limit, exact beyond it). */
static void aba(const Env *e, Work *w, real h, const real *q, const real *qd, const V6 v0, real *qdd, V6 a0,
                int with_bias, const real *qdd_prev) {
    const tg_model_desc *m = e->m;
    int G = m->num_groups;
    for (int g = 0; g < G; ++g) {
        int d = w->gdof[g];
        /* joint transform */
        if (g == 0) {
            memcpy(w->v[0], v0, sizeof(V6));
            memset(w->c[0], 0, sizeof(V6));
            memset(w->S[0], 0, sizeof(V6));
        } else {
            int p = m->group_parent[g];
            M3 Rpc;
            V3 t;
            memcpy(t, w->xtp[g], sizeof t);
            if (w->gtype[g] == TG_JOINT_REVOLUTE) {
                M3 Rj;
                axis_angle(w->gaxis[g], q[d], Rj);
                m3_mul(w->xtR[g], Rj, Rpc);
            } else {
                memcpy(Rpc, w->xtR[g], sizeof(M3));
                V3 s;
                m3_v(w->xtR[g], w->gaxis[g], s);
                for (int k = 0; k < 3; ++k) t[k] += s[k] * q[d];
            }
            m3_T(Rpc, w->X[g].E);
            memcpy(w->X[g].r, t, sizeof t);
            V6 S = {0};
            if (w->gtype[g] == TG_JOINT_REVOLUTE) { S[0] = w->gaxis[g][0]; S[1] = w->gaxis[g][1]; S[2] = w->gaxis[g][2]; }
            else { S[3] = w->gaxis[g][0]; S[4] = w->gaxis[g][1]; S[5] = w->gaxis[g][2]; }
            memcpy(w->S[g], S, sizeof S);
            V6 vp, vJ;
            X_motion(&w->X[g], w->v[p], vp);
            for (int k = 0; k < 6; ++k) { vJ[k] = S[k] * qd[d]; w->v[g][k] = vp[k] + vJ[k]; }
            crm(w->v[g], vJ, w->c[g]);
            /* world pose */
            m3_mul(w->Rw[p], Rpc, w->Rw[g]);
            V3 tw;
            m3_v(w->Rw[p], t, tw);
            for (int k = 0; k < 3; ++k) w->pw[g][k] = w->pw[p][k] + tw[k];
        }
        rb_inertia(w->gm[g], w->gc[g], w->gI[g], w->IA[g]);
        memset(w->pA[g], 0, sizeof(V6));
        if (with_bias) {
            V6 Iv, b;
            m6_v(w->IA[g], w->v[g], Iv);
            crf(w->v[g], Iv, b);
            /* gravity + damping + applied wrench (group frame, about group origin) */
            V3 gl, F, n;
            m3T_v(w->Rw[g], e->g, gl);
            for (int k = 0; k < 3; ++k) F[k] = w->gm[g] * gl[k];
            V3 wv = {w->v[g][0], w->v[g][1], w->v[g][2]}, vo = {w->v[g][3], w->v[g][4], w->v[g][5]}, vc, wxc;
            cross3(wv, w->gc[g], wxc);
            for (int k = 0; k < 3; ++k) vc[k] = vo[k] + wxc[k];
            for (int k = 0; k < 3; ++k) F[k] -= e->sp->linear_damping * w->gm[g] * vc[k];
            V3 Iw;
            m3_v(w->gI[g], wv, Iw);
            cross3(w->gc[g], F, n);
            for (int k = 0; k < 3; ++k) n[k] -= e->sp->angular_damping * Iw[k];
            if (e->force) {
                const float *fw = e->force + 6 * g;
                V3 fwv = {fw[0], fw[1], fw[2]}, twv = {fw[3], fw[4], fw[5]}, fl, tl, cxf;
                m3T_v(w->Rw[g], fwv, fl);
                m3T_v(w->Rw[g], twv, tl);
                cross3(w->gc[g], fl, cxf);
                for (int k = 0; k < 3; ++k) { F[k] += fl[k]; n[k] += tl[k] + cxf[k]; }
            }
            for (int k = 0; k < 3; ++k) { b[k] -= n[k]; b[3 + k] -= F[k]; }
            memcpy(w->pA[g], b, sizeof b);
        }
    }
    /* pass 2 */
    for (int g = G - 1; g >= 1; --g) {
        int d = w->gdof[g], p = m->group_parent[g];
        m6_v(w->IA[g], w->S[g], w->U[g]);
        real D0 = 0;
        for (int k = 0; k < 6; ++k) D0 += w->S[g][k] * w->U[g][k];
        D0 += prop(e, TG_PROP_ARMATURE, d);
        real Dimp = 0, tau = 0;
        if (with_bias) {
            int mode = (int)lrint(prop(e, TG_PROP_DRIVE_MODE, d));
            real kp = prop(e, TG_PROP_STIFFNESS, d), kd = prop(e, TG_PROP_DAMPING, d), eff = prop(e, TG_PROP_EFFORT, d);
            if (mode == TG_DOF_MODE_POS || mode == TG_DOF_MODE_VEL) {
                real te = kp * (e->pos_tgt[d] - q[d] - h * qd[d]) + kd * (e->vel_tgt[d] - qd[d]);
                real K = h * kd + h * h * kp;
                real ti = qdd_prev ? te - K * qdd_prev[d] : 0;
                if (!qdd_prev || fabs(ti) <= eff) { tau += te; Dimp += K; }
                else tau += ti > 0 ? eff : -eff;
            } else if (mode == TG_DOF_MODE_EFFORT && e->act) {
                real a = e->act[d];
                tau += a > eff ? eff : (a < -eff ? -eff : a);
            }
            real lo = prop(e, TG_PROP_LOWER, d), hi = prop(e, TG_PROP_UPPER, d);
            real qp = q[d] + h * qd[d];
            real kl = e->sp->limit_stiffness * D0 / (h * h), cl = e->sp->limit_damping * D0 / h;
            /* limit spring k(lo - qp) plus damping; the damping and the implicit
             * terms ramp in over the first TG_LIMIT_RAMP past the limit, so the
             * step is continuous when a joint reaches its limit */
            if (qp < lo && lo > -1e30) {
                real r = (lo - qp) / TG_LIMIT_RAMP;
                r = r > 1 ? 1 : r;
                tau += kl * (lo - qp) - r * cl * qd[d];
                Dimp += r * (h * cl + h * h * kl);
            } else if (qp > hi && hi < 1e30) {
                real r = (qp - hi) / TG_LIMIT_RAMP;
                r = r > 1 ? 1 : r;
                tau += kl * (hi - qp) - r * cl * qd[d];
                Dimp += r * (h * cl + h * h * kl);
            }
        } else {
            /* impulse response: same effective inertia as the dynamics pass */
            Dimp = w->D[g] - D0;
        }
        w->D[g] = D0 + Dimp;
        real sp = 0;
        for (int k = 0; k < 6; ++k) sp += w->S[g][k] * w->pA[g][k];
        w->u[g] = tau - sp;
        M6 Ia;
        V6 pa, Iac;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) Ia[6 * i + j] = w->IA[g][6 * i + j] - w->U[g][i] * w->U[g][j] / w->D[g];
        m6_v(Ia, w->c[g], Iac);
        for (int k = 0; k < 6; ++k) pa[k] = w->pA[g][k] + (with_bias ? Iac[k] : 0) + w->U[g][k] * w->u[g] / w->D[g];
        /* parent += X^T Ia X ; X^T pa */
        M6 X, T, XT;
        X_dense(&w->X[g], X);
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) XT[6 * i + j] = X[6 * j + i];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                real s = 0;
                for (int k = 0; k < 6; ++k) s += Ia[6 * i + k] * X[6 * k + j];
                T[6 * i + j] = s;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                real s = 0;
                for (int k = 0; k < 6; ++k) s += XT[6 * i + k] * T[6 * k + j];
                w->IA[p][6 * i + j] += s;
            }
        V6 pp;
        XT_force(&w->X[g], pa, pp);
        for (int k = 0; k < 6; ++k) w->pA[p][k] += pp[k];
    }
    /* pass 3 */
    if (e->sp->fix_base) memset(a0, 0, sizeof(V6));
    else {
        V6 mp;
        for (int k = 0; k < 6; ++k) mp[k] = -w->pA[0][k];
        solve6(w->IA[0], mp, a0);
    }
    V6 a[MAXG];
    memcpy(a[0], a0, sizeof(V6));
    for (int g = 1; g < G; ++g) {
        int d = w->gdof[g], p = m->group_parent[g];
        V6 ap;
        X_motion(&w->X[g], a[p], ap);
        for (int k = 0; k < 6; ++k) ap[k] += with_bias ? w->c[g][k] : 0;
        real ua = 0;
        for (int k = 0; k < 6; ++k) ua += w->U[g][k] * ap[k];
        qdd[d] = (w->u[g] - ua) / w->D[g];
        for (int k = 0; k < 6; ++k) a[g][k] = ap[k] + w->S[g][k] * qdd[d];
    }
}

/* does any position/velocity drive's implicit torque te - K*qdd exceed its effort? */
static int drives_saturated(const Env *e, Work *w, real h, const real *q, const real *qd, const real *qdd) {
    for (int g = 1; g < e->m->num_groups; ++g) {
        int d = w->gdof[g];
        int mode = (int)lrint(prop(e, TG_PROP_DRIVE_MODE, d));
        if (mode != TG_DOF_MODE_POS && mode != TG_DOF_MODE_VEL) continue;
        real kp = prop(e, TG_PROP_STIFFNESS, d), kd = prop(e, TG_PROP_DAMPING, d), eff = prop(e, TG_PROP_EFFORT, d);
        real te = kp * (e->pos_tgt[d] - q[d] - h * qd[d]) + kd * (e->vel_tgt[d] - qd[d]);
        if (fabs(te - (h * kd + h * h * kp) * qdd[d]) > eff) return 1;
    }
    return 0;
}

/* developer dump: the drive closest to its effort limit after the implicit
 * solve -- | |te - K qdd| - effort |, and its dof in *dof */
static real drive_margin(const Env *e, Work *w, real h, const real *q, const real *qd, const real *qdd, int *dof) {
    real best = 1e30;
    *dof = -1;
    for (int g = 1; g < e->m->num_groups; ++g) {
        int d = w->gdof[g];
        int mode = (int)lrint(prop(e, TG_PROP_DRIVE_MODE, d));
        if (mode != TG_DOF_MODE_POS && mode != TG_DOF_MODE_VEL) continue;
        real kp = prop(e, TG_PROP_STIFFNESS, d), kd = prop(e, TG_PROP_DAMPING, d), eff = prop(e, TG_PROP_EFFORT, d);
        real te = kp * (e->pos_tgt[d] - q[d] - h * qd[d]) + kd * (e->vel_tgt[d] - qd[d]);
        real m = fabs(fabs(te - (h * kd + h * h * kp) * qdd[d]) - eff);
        if (m < best) { best = m; *dof = d; }
    }
    return best;
}

/* velocity of group g's spatial velocity for generalised velocity (qd, v0) with current X */
static void group_vels(const tg_model_desc *m, Work *w, const real *qd, const V6 v0, V6 *vg) {
    memcpy(vg[0], v0, sizeof(V6));
    for (int g = 1; g < m->num_groups; ++g) {
        V6 vp;
        X_motion(&w->X[g], vg[m->group_parent[g]], vp);
        for (int k = 0; k < 6; ++k) vg[g][k] = vp[k] + w->S[g][k] * qd[w->gdof[g]];
    }
}

/* impulse response: spatial impulses fi[G] (group frames) -> dqd, dv0 */
static void impulse_response(const Env *e, Work *w, const V6 *fi, real *dqd, V6 dv0) {
    const tg_model_desc *m = e->m;
    int G = m->num_groups;
    V6 p[MAXG];
    for (int g = 0; g < G; ++g)
        for (int k = 0; k < 6; ++k) p[g][k] = -fi[g][k];
    real u[MAXG];
    for (int g = G - 1; g >= 1; --g) {
        real sp = 0;
        for (int k = 0; k < 6; ++k) sp += w->S[g][k] * p[g][k];
        u[g] = -sp;
        V6 pa, pp;
        for (int k = 0; k < 6; ++k) pa[k] = p[g][k] + w->U[g][k] * u[g] / w->D[g];
        XT_force(&w->X[g], pa, pp);
        for (int k = 0; k < 6; ++k) p[m->group_parent[g]][k] += pp[k];
    }
    V6 a[MAXG];
    if (e->sp->fix_base) memset(a[0], 0, sizeof(V6));
    else {
        V6 mp;
        for (int k = 0; k < 6; ++k) mp[k] = -p[0][k];
        solve6(w->IA[0], mp, a[0]);
    }
    memcpy(dv0, a[0], sizeof(V6));
    for (int g = 1; g < G; ++g) {
        V6 ap;
        X_motion(&w->X[g], a[m->group_parent[g]], ap);
        real ua = 0;
        for (int k = 0; k < 6; ++k) ua += w->U[g][k] * ap[k];
        real x = (u[g] - ua) / w->D[g];
        dqd[w->gdof[g]] = x;
        for (int k = 0; k < 6; ++k) a[g][k] = ap[k] + w->S[g][k] * x;
    }
}

/* Contact rows.  Per shape, the contact points (closest torus point, sphere
 * bottom, the 4 corners of a box's lowest face) each get a NORMAL row;
 * the shape's points form one friction patch (PhysX-style patch friction)
 * with two tangent rows at the patch centroid, coupled by a Coulomb cone
 * mu*sum(normal), and one torsional row about the normal limited by
 * mu*sum(normal)*r_eff. */
enum { ROW_NORMAL = 0, ROW_T1 = 1, ROW_T2 = 2, ROW_TORSION = 3 };
typedef struct {
    int g, type, angular, patch;
    V3 r;            /* application point in group frame (linear rows) */
    V3 d;            /* world direction (force) or axis (moment) */
    real target;     /* normal rows: velocity lower bound */
    real phi;        /* normal rows: separation at the start of the substep */
} Row;
typedef struct {
    int n0, nn;      /* first normal row, number of normal rows */
    int f0;          /* first of the friction rows: t1, t2, then torsion when nf == 3 */
    int nf;          /* friction rows: 3, or 2 for a one-point patch (torus, sphere), whose
                        torsion radius is 0 -- PhysX applies no torsional friction without a
                        torsional patch radius either */
    real mu, reff;
} Patch;

/* developer instrumentation (scripts/dev/contact_dump.py): the contact solve
 * of env oracle_dump_env in substep oracle_dump_sub of a call -- Delassus matrix
 * [16 + i K + j], free row velocities [2000 + i], the stored-velocity
 * multipliers [2500 + i] and the positions' [2600 + i] -- for a side-by-side
 * with the kernel's dump (TG_DUMP_ENV builds).  Off (-1) by default. */
int oracle_dump_env = -1, oracle_dump_sub = 0;
double oracle_dump_buf[4096];
static __thread int t_env = -1, t_substep = -1;
void oracle_dump_set(int e, int substep) { oracle_dump_env = e; oracle_dump_sub = substep; }
void oracle_dump_read(double *out, int n) { memcpy(out, oracle_dump_buf, sizeof(double) * (n > 4096 ? 4096 : n)); }

/* a normal row's velocity lower bound over a step dt at separation phi: the
 * speculative approach bound -(phi - rest)/dt above the rest offset, the
 * Baumgarte push-out capped by max_depenetration_velocity below it */
static real row_target(const tg_sim_params *sp, real phi, real dt) {
    const real rest = sp->rest_offset;
    if (phi > rest) return -(phi - rest) / dt;
    real t = sp->baumgarte * (rest - phi) / dt;
    return t > sp->max_depenetration_velocity ? sp->max_depenetration_velocity : t;
}

static void row_force(const Work *w, const Row *r, real lam, V6 *fi) {
    V3 dl, rxd;
    m3T_v(w->Rw[r->g], r->d, dl);
    if (r->angular) {
        for (int k = 0; k < 3; ++k) fi[r->g][k] += lam * dl[k];
    } else {
        cross3(r->r, dl, rxd);
        for (int k = 0; k < 3; ++k) { fi[r->g][k] += lam * rxd[k]; fi[r->g][3 + k] += lam * dl[k]; }
    }
}
static real row_vel(const Work *w, const Row *r, const V6 *vg) {
    V3 om = {vg[r->g][0], vg[r->g][1], vg[r->g][2]}, vl = {vg[r->g][3], vg[r->g][4], vg[r->g][5]}, loc, out;
    if (r->angular) {
        m3_v(w->Rw[r->g], om, out);
    } else {
        V3 wxr;
        cross3(om, r->r, wxr);
        for (int k = 0; k < 3; ++k) loc[k] = vl[k] + wxr[k];
        m3_v(w->Rw[r->g], loc, out);
    }
    return dot3(out, r->d);
}

/* Terrain (tg_set_heightfield; gym.add_triangle_mesh of the
 * convert_heightfield_to_trimesh mesh, tasks/gogoro_new.py:164-181): vertex
 * (i, j) at (ox + i hs, oy + j hs, vs h[i][j]); cell (i, j) is split into
 * (i,j)-(i+1,j+1)-(i,j+1) (fv >= fu) and (i,j)-(i+1,j)-(i+1,j+1) (fu >= fv).
 * The z = 0 plane stays (gogoro_new.py:157-159 adds both), so the ground is
 * the higher of the two.  Test infrastructure: one terrain for all envs. */
static struct {
    const float *h;
    int rows, cols;
    real hs, vs, ox, oy, mu;
} g_hf;

void oracle_set_heightfield(const float *heights, int rows, int cols, float hs, float vs, float ox, float oy,
                            float friction) {
    g_hf.h = rows > 0 ? heights : NULL;
    g_hf.rows = rows;
    g_hf.cols = cols;
    g_hf.hs = hs;
    g_hf.vs = vs;
    g_hf.ox = ox;
    g_hf.oy = oy;
    g_hf.mu = friction;
}

/* height of the ground under (x, y); unit normal in n, *on_hf = terrain is the surface */
static real ground_at(real x, real y, V3 n, int *on_hf) {
    n[0] = 0; n[1] = 0; n[2] = 1;
    *on_hf = 0;
    if (!g_hf.h) return 0;
    real u = (x - g_hf.ox) / g_hf.hs, v = (y - g_hf.oy) / g_hf.hs;
    if (!(u >= 0 && v >= 0 && u <= g_hf.rows - 1 && v <= g_hf.cols - 1)) return 0;
    int i = (int)u, j = (int)v;
    if (i > g_hf.rows - 2) i = g_hf.rows - 2;
    if (j > g_hf.cols - 2) j = g_hf.cols - 2;
    real fu = u - i, fv = v - j;
    const float *r0 = g_hf.h + (long)i * g_hf.cols + j, *r1 = r0 + g_hf.cols;
    real h00 = g_hf.vs * r0[0], h01 = g_hf.vs * r0[1], h10 = g_hf.vs * r1[0], h11 = g_hf.vs * r1[1];
    real gx, gy;
    if (fu >= fv) { gx = h10 - h00; gy = h11 - h10; }
    else          { gx = h11 - h01; gy = h01 - h00; }
    real H = h00 + fu * gx + fv * gy;
    if (!(H > 0)) return 0;
    gx /= g_hf.hs;
    gy /= g_hf.hs;
    real inv = 1 / sqrt(gx * gx + gy * gy + 1);
    n[0] = -gx * inv; n[1] = -gy * inv; n[2] = inv;
    *on_hf = 1;
    return H;
}

/* contact points of shape s (centre c, world rotation R) against the ground
 * with normal n: the support point (torus, sphere) or the 4 corners of the
 * box face whose outward normal points most against n */
static int support_points(const tg_model_desc *m, int s, const M3 R, const V3 c, const V3 n, V3 *pts) {
    if (m->shape_kind[s] == TG_SHAPE_TORUS) {
        real Rm = m->shape_params[4 * s], rm = m->shape_params[4 * s + 1];
        V3 a = {R[2], R[5], R[8]};
        real an = dot3(a, n);
        V3 d = {n[0] - an * a[0], n[1] - an * a[1], n[2] - an * a[2]};
        real nd = sqrt(dot3(d, d));
        if (nd < 1e-9) { d[0] = 1; d[1] = 0; d[2] = 0; nd = 1; }
        for (int k = 0; k < 3; ++k) pts[0][k] = c[k] - Rm * d[k] / nd - rm * n[k];
        return 1;
    }
    if (m->shape_kind[s] == TG_SHAPE_SPHERE) {
        for (int k = 0; k < 3; ++k) pts[0][k] = c[k] - m->shape_params[4 * s] * n[k];
        return 1;
    }
    if (m->shape_kind[s] == TG_SHAPE_BOX) {
        V3 z;   /* box axes . n */
        for (int k = 0; k < 3; ++k) z[k] = R[k] * n[0] + R[3 + k] * n[1] + R[6 + k] * n[2];
        real zx = fabs(z[0]), zy = fabs(z[1]), zz = fabs(z[2]);
        int ax = (zz >= zx && zz >= zy) ? 2 : (zy >= zx ? 1 : 0);
        real sgn = z[ax] > 0 ? -1.0 : 1.0;
        int a1 = ax == 0 ? 1 : 0, a2 = ax == 2 ? 1 : 2;
        for (int k = 0; k < 4; ++k) {
            V3 l = {0, 0, 0}, wv;
            l[ax] = sgn * m->shape_params[4 * s + ax];
            l[a1] = (k & 1 ? 1 : -1) * m->shape_params[4 * s + a1];
            l[a2] = (k & 2 ? 1 : -1) * m->shape_params[4 * s + a2];
            m3_v(R, l, wv);
            for (int j = 0; j < 3; ++j) pts[k][j] = c[j] + wv[j];
        }
        return 4;
    }
    return 0;
}

/* physx.contact_offset (round 6: PhysX's pair rule): a point
 * generates a contact (a speculative normal row) only while its separation is
 * below the pair's contact distance, the sum of the shape's and the ground
 * plane's offsets, both the scene's contact_offset -- 2 x contact_offset.
 * Beyond it the separation becomes NO_ROW, whose target -NO_ROW/h no row
 * velocity reaches, so its multiplier stays 0 (the kernel's contact_row_phi,
 * articulation_kernels.h, which records why round 5's velocity-dependent
 * gate was dropped).  contact_offset <= 0: every point speculative. */
#define NO_ROW ((real)1e30f)
static real contact_row_phi(const tg_sim_params *sp, real phi) {
    const real off = sp->contact_offset;
    return (off > 0 && !(phi < 2 * off)) ? NO_ROW : phi;
}

static int collect_rows(const Env *e, Work *w, real h, const V6 *vg, Row *rows, Patch *patches, int *npatch) {
    const tg_model_desc *m = e->m;
    int nr = 0, np_ = 0;
    for (int s = 0; s < m->num_shapes; ++s) {
        int g = w->shg[s];
        M3 R;
        V3 c;
        m3_mul(w->Rw[g], w->shR[s], R);
        m3_v(w->Rw[g], w->shp[s], c);
        for (int k = 0; k < 3; ++k) c[k] += w->pw[g][k];
        /* patch normal n: the ground normal under the support point (found
         * from the normal under the centre, refined once); e_z on the plane */
        V3 pts[8], n = {0, 0, 1};
        real gmu = e->sp->ground_friction;
        if (g_hf.h) {
            int th;
            ground_at(w->org[0] + c[0], w->org[1] + c[1], n, &th);
            support_points(m, s, R, c, n, pts);
            ground_at(w->org[0] + pts[0][0], w->org[1] + pts[0][1], n, &th);
            if (th) gmu = g_hf.mu;
        }
        int np = support_points(m, s, R, c, n, pts);
        /* every point carries a speculative normal row (continuous in the
         * state: a row only pushes when the point would pass the rest offset
         * within the substep).  The friction patch is anchored at the
         * centroid of the points weighted by w = clamp((margin - phi)/margin,
         * 0, 1) (plain centroid when no point is within the margin), with
         * r_eff the weighted mean planar distance to it. */
        Patch *P = &patches[np_];
        P->n0 = nr;
        P->nn = np;
        V3 cen = {0, 0, 0}, cen0 = {0, 0, 0};
        real wk[8], wsum = 0;
        const real margin = e->sp->contact_margin;
        for (int k = 0; k < np; ++k) {
            real phi = w->org[2] + pts[k][2];
            if (g_hf.h) {   /* separation along the normal of the point's own triangle */
                V3 nk;
                int th;
                real gz = ground_at(w->org[0] + pts[k][0], w->org[1] + pts[k][1], nk, &th);
                phi = (w->org[2] + pts[k][2] - gz) * nk[2];
            }
            Row *r = &rows[nr++];
            r->g = g; r->type = ROW_NORMAL; r->angular = 0; r->patch = np_;
            V3 rel;
            for (int j = 0; j < 3; ++j) rel[j] = pts[k][j] - w->pw[g][j];
            m3T_v(w->Rw[g], rel, r->r);
            memcpy(r->d, n, sizeof(V3));
            r->phi = contact_row_phi(e->sp, phi);
            r->target = row_target(e->sp, r->phi, h);
            real wv = (margin - phi) / margin;
            wk[k] = wv < 0 ? 0 : (wv > 1 ? 1 : wv);
            wsum += wk[k];
            for (int j = 0; j < 3; ++j) { cen[j] += wk[k] * pts[k][j]; cen0[j] += pts[k][j]; }
        }
        for (int j = 0; j < 3; ++j) cen[j] = wsum > 0 ? cen[j] / wsum : cen0[j] / np;
        P->reff = 0;
        for (int k = 0; k < np; ++k) {   /* distance in the contact plane */
            V3 d = {pts[k][0] - cen[0], pts[k][1] - cen[1], pts[k][2] - cen[2]};
            real dn = dot3(d, n);
            for (int j = 0; j < 3; ++j) d[j] -= dn * n[j];
            P->reff += (wsum > 0 ? wk[k] / wsum : 1.0 / np) * sqrt(dot3(d, d));
        }
        P->mu = 0.5 * (e->mu[s] + gmu);
        /* tangent basis: rolling direction for tori (axis x n), else world x in the plane */
        V3 t1 = {1, 0, 0}, t2, x;
        if (m->shape_kind[s] == TG_SHAPE_TORUS) {
            V3 a = {R[2], R[5], R[8]};
            cross3(a, n, x);
        } else {
            for (int j = 0; j < 3; ++j) x[j] = (j == 0) - n[0] * n[j];
        }
        real nx = sqrt(dot3(x, x));
        if (nx > 1e-6) for (int j = 0; j < 3; ++j) t1[j] = x[j] / nx;
        cross3(n, t1, t2);
        P->f0 = nr;
        V3 rel, rl;
        for (int j = 0; j < 3; ++j) rel[j] = cen[j] - w->pw[g][j];
        m3T_v(w->Rw[g], rel, rl);
        P->nf = np == 1 ? 2 : 3;
        for (int t = 0; t < P->nf; ++t) {
            Row *r = &rows[nr++];
            r->g = g; r->type = ROW_T1 + t; r->angular = (t == 2); r->patch = np_; r->target = 0;
            memcpy(r->r, rl, sizeof rl);
            memcpy(r->d, t == 0 ? t1 : (t == 1 ? t2 : n), sizeof(V3));
        }
        ++np_;
    }
    *npatch = np_;
    return nr;
}

/* Contact solve of one substep.  sp->contact_iterations projected
 * Gauss-Seidel sweeps with the push-out bias (PhysX's position iterations),
 * then sp->velocity_iterations bias-free sweeps continuing from those
 * multipliers (PhysX's velocity iterations: a normal row's target becomes
 * min(target, 0) -- the speculative approach bound stays, the push-out goes).
 * qds / v0s leave with the velocity of the biased multipliers, which the
 * positions integrate; qdv / v0v with the bias-free one, which is stored. */
static void pgs_sweeps(int K, int npatch, const Patch *patches, const Row *rows, const real *target,
                       real (*W)[3 * MAXC], const real *vfree, real *lam, int iters) {
#define ROWV(i) ({ real v_ = vfree[i]; for (int j_ = 0; j_ < K; ++j_) v_ += W[i][j_] * lam[j_]; v_; })
    /* a row with no response (a shape on a fixed base, a normal row through a
     * fixed-base scooter's wheel) takes no impulse; real rows have W_ii of
     * 1e-3 .. 1e1, the threshold only catches rounding residue (the kernel's
     * inv_diag) */
#define OVERW(x, i) (W[i][i] > 1e-9 ? (x) / W[i][i] : 0)
    for (int it = 0; it < iters; ++it) {
        for (int p = 0; p < npatch; ++p) {
            const Patch *P = &patches[p];
            real N = 0;
            for (int i = P->n0; i < P->n0 + P->nn; ++i) {
                real l = lam[i] + OVERW(target[i] - ROWV(i), i);
                lam[i] = l > 0 ? l : 0;
                N += lam[i];
            }
            int f = P->f0;
            lam[f] -= OVERW(ROWV(f), f);
            lam[f + 1] -= OVERW(ROWV(f + 1), f + 1);
            real lt = sqrt(lam[f] * lam[f] + lam[f + 1] * lam[f + 1]), lim = P->mu * N;
            if (lt > lim) {
                real sc = lt > 0 ? lim / lt : 0;
                lam[f] *= sc;
                lam[f + 1] *= sc;
            }
            if (P->nf == 3) {
                real lt3 = lam[f + 2] - OVERW(ROWV(f + 2), f + 2), lim3 = P->mu * N * P->reff;
                lam[f + 2] = lt3 > lim3 ? lim3 : (lt3 < -lim3 ? -lim3 : lt3);
            }
        }
    }
#undef ROWV
#undef OVERW
}

static void apply_impulses(const Env *e, Work *w, const Row *rows, int K, const real *lam, real *qd, V6 v0) {
    const tg_model_desc *m = e->m;
    int G = m->num_groups;
    V6 fi[MAXG];
    memset(fi, 0, sizeof(V6) * G);
    for (int i = 0; i < K; ++i) row_force(w, &rows[i], lam[i], fi);
    real dqd[MAXD] = {0};
    V6 dv0;
    impulse_response(e, w, fi, dqd, dv0);
    for (int g = 1; g < G; ++g) qd[w->gdof[g]] += dqd[w->gdof[g]];
    for (int k = 0; k < 6; ++k) v0[k] += dv0[k];
}

static void solve_contacts(const Env *e, Work *w, real h, real *qds, V6 v0s, real *qdv, V6 v0v) {
    const tg_model_desc *m = e->m;
    int G = m->num_groups, D = m->num_dofs;
    memcpy(qdv, qds, sizeof(real) * D);
    memcpy(v0v, v0s, sizeof(V6));
    Row rows[3 * MAXC];
    Patch patches[MAXC];
    int npatch = 0;
    V6 vg[MAXG];
    group_vels(m, w, qds, v0s, vg);
    int K = collect_rows(e, w, h, vg, rows, patches, &npatch);
    if (K == 0) return;
    static __thread real W[3 * MAXC][3 * MAXC];
    real vfree[3 * MAXC], lam[3 * MAXC], target[3 * MAXC];
    for (int i = 0; i < K; ++i) vfree[i] = row_vel(w, &rows[i], vg);
    for (int col = 0; col < K; ++col) {
        V6 fi[MAXG];
        memset(fi, 0, sizeof(V6) * G);
        row_force(w, &rows[col], 1.0, fi);
        real dqd[MAXD] = {0};
        V6 dv0, dvg[MAXG];
        impulse_response(e, w, fi, dqd, dv0);
        group_vels(m, w, dqd, dv0, dvg);
        for (int i = 0; i < K; ++i) W[i][col] = row_vel(w, &rows[i], dvg);
    }
    const int dump = t_env >= 0 && t_env == oracle_dump_env && t_substep == oracle_dump_sub;
    if (dump) {
        oracle_dump_buf[0] = K;
        for (int i = 0; i < K; ++i) {
            for (int j = 0; j < K; ++j) oracle_dump_buf[16 + i * K + j] = W[i][j];
            oracle_dump_buf[2000 + i] = vfree[i];
            oracle_dump_buf[2100 + i * 8 + 6] = rows[i].type == ROW_NORMAL ? rows[i].phi : 0;
        }
    }
    memset(lam, 0, sizeof(real) * K);
    for (int i = 0; i < K; ++i) target[i] = rows[i].target;
    const int tgs = e->sp->solver_type == 1 && e->sp->contact_iterations > 0;
    if (tgs) {
        /* TGS: the N position iterations are sub-steps of hs = h / N.  Before
         * each sweep a normal row's target is re-formed over hs from its
         * separation advanced by the row's displacement so far (hs times its
         * velocity after every earlier sweep, the linearised motion of the
         * sub-steps); the positions integrate the mean of the N sweeps'
         * multipliers (the mean sub-step velocity, velocity being affine in
         * the multipliers); the velocity iterations start from that mean
         * (warm start) with the push-out removed and the targets formed over h. */
        const int N = e->sp->contact_iterations;
        const real hs = h / N;
        real disp[3 * MAXC], lbar[3 * MAXC];
        for (int i = 0; i < K; ++i) disp[i] = lbar[i] = 0;
        for (int it = 0; it < N; ++it) {
            for (int i = 0; i < K; ++i)
                if (rows[i].type == ROW_NORMAL) target[i] = row_target(e->sp, rows[i].phi + disp[i], hs);
            pgs_sweeps(K, npatch, patches, rows, target, W, vfree, lam, 1);
            for (int i = 0; i < K; ++i) {
                lbar[i] += lam[i];
                if (rows[i].type == ROW_NORMAL) {
                    real v = vfree[i];
                    for (int j = 0; j < K; ++j) v += W[i][j] * lam[j];
                    disp[i] += hs * v;
                }
            }
        }
        /* the bias-free targets: a normal row's from its final separation over
         * the whole substep h (not hs): the velocity the velocity iterations
         * leave is the one the next substep starts from, and a speculative
         * bound over hs gave it a gain of N/h on the residual gap -- 1e-6 of
         * state became 1.3e-3 of roll rate at the spawn landings (DESIGN.md §2
         * "TGS conditioning", scripts/dev/tgs_landing_study.py) */
        for (int i = 0; i < K; ++i) {
            if (rows[i].type == ROW_NORMAL) target[i] = row_target(e->sp, rows[i].phi + disp[i], h);
            target[i] = target[i] < 0 ? target[i] : 0;
            lbar[i] /= N;
        }
        /* the velocity iterations are warm-started from the sub-steps' MEAN
         * multipliers (the velocity of the step's displacement), not the last
         * sub-step's: a contact that closes its gap in the last sub-step
         * leaves that sub-step with the velocity -gap/hs, a gain of N/h on the
         * gap, which one bias-free sweep does not undo (ThormangWalk one-step
         * f32-vs-f64 error 1.5e-4 -> 4.2e-5, the PGS level; DESIGN.md §2 "TGS
         * conditioning").  Without velocity iterations the stored velocity is
         * the last sub-step's, as the position iterations leave it. */
        real lamv[3 * MAXC];
        memcpy(lamv, e->sp->velocity_iterations > 0 ? lbar : lam, sizeof(real) * K);
        if (e->sp->velocity_iterations > 0)
            pgs_sweeps(K, npatch, patches, rows, target, W, vfree, lamv, e->sp->velocity_iterations);
        if (dump)
            for (int i = 0; i < K; ++i) { oracle_dump_buf[2500 + i] = lamv[i]; oracle_dump_buf[2600 + i] = lbar[i]; }
        apply_impulses(e, w, rows, K, lamv, qdv, v0v);
        apply_impulses(e, w, rows, K, lbar, qds, v0s);
        return;
    }
    pgs_sweeps(K, npatch, patches, rows, target, W, vfree, lam, e->sp->contact_iterations);
    if (e->sp->velocity_iterations > 0) {
        real lamv[3 * MAXC];
        memcpy(lamv, lam, sizeof(real) * K);
        for (int i = 0; i < K; ++i) target[i] = target[i] < 0 ? target[i] : 0;
        pgs_sweeps(K, npatch, patches, rows, target, W, vfree, lamv, e->sp->velocity_iterations);
        apply_impulses(e, w, rows, K, lamv, qdv, v0v);
    }
    apply_impulses(e, w, rows, K, lam, qds, v0s);
    if (e->sp->velocity_iterations <= 0) {
        memcpy(qdv, qds, sizeof(real) * D);
        memcpy(v0v, v0s, sizeof(V6));
    }
}

/* One env, one control step (all substeps).  root[13], dof[2D] updated in place. */
void oracle_physics_step_env(const tg_model_desc *m, const tg_sim_params *sp, float *root, float *dof,
                             const float *props, long prop_stride, const float *pos_tgt, const float *vel_tgt,
                             const float *act, const float *force, const float *mass_scale, const float *mu,
                             const float *gravity) {
    static __thread Work w;   /* large; per thread */
    Env e = {m, sp, props, prop_stride, pos_tgt, vel_tgt, act, force, mu, {gravity[0], gravity[1], gravity[2]}};
    int D = m->num_dofs, G = m->num_groups;
    real lockq[MAXD], q[MAXD], qd[MAXD], qdd[MAXD];
    for (int d = 0; d < D; ++d) {
        lockq[d] = m->dof_locked[d] ? 0.5 * ((real)props[TG_PROP_LOWER * prop_stride + d] + props[TG_PROP_UPPER * prop_stride + d]) : 0;
        q[d] = dof[2 * d];
        qd[d] = dof[2 * d + 1];
        qdd[d] = 0;
    }
    compose(m, lockq, mass_scale, &w);
    real h = sp->substeps > 0 ? sp->dt / sp->substeps : 0;
    /* floating base state */
    real pos[3] = {root[0], root[1], root[2]}, quat[4] = {root[3], root[4], root[5], root[6]};
    real qn = sqrt(quat[0] * quat[0] + quat[1] * quat[1] + quat[2] * quat[2] + quat[3] * quat[3]);
    for (int k = 0; k < 4; ++k) quat[k] /= qn;
    M3 R;
    quat_to_m3(quat, R);
    const float *li0 = m->link_inertia;
    V3 c0 = {li0[1], li0[2], li0[3]}, c0w, ww = {root[10], root[11], root[12]}, wxc, vo;
    m3_v(R, c0, c0w);
    cross3(ww, c0w, wxc);
    for (int k = 0; k < 3; ++k) vo[k] = root[7 + k] - wxc[k];
    V6 v0;
    V3 wb, vb;
    m3T_v(R, ww, wb);
    m3T_v(R, vo, vb);
    for (int k = 0; k < 3; ++k) { v0[k] = wb[k]; v0[3 + k] = vb[k]; }
    if (sp->fix_base) memset(v0, 0, sizeof v0);

    for (int s = 0; s < sp->substeps; ++s) {
        t_substep = s;
        memcpy(w.Rw[0], R, sizeof(M3));
        /* (positions about the root origin: the contact geometry never forms
         * world coordinates, as the kernel's, step_par.h PL::CGP) */
        memset(w.pw[0], 0, sizeof(V3));
        memcpy(w.org, pos, sizeof(V3));
        V6 a0;
        aba(&e, &w, h, q, qd, v0, qdd, a0, 1, NULL);
        const int sat = drives_saturated(&e, &w, h, q, qd, qdd);
        if (t_env >= 0 && t_env == oracle_dump_env && s == oracle_dump_sub) {
            int dm;
            oracle_dump_buf[2791] = drive_margin(&e, &w, h, q, qd, qdd, &dm);
            oracle_dump_buf[2792] = dm;
        }
        if (sat) {
            real qdd0[MAXD];
            memcpy(qdd0, qdd, sizeof(real) * D);
            aba(&e, &w, h, q, qd, v0, qdd, a0, 1, qdd0);
        }
        if (t_env >= 0 && t_env == oracle_dump_env && s == oracle_dump_sub) {   /* developer dump (contact_dump.py) */
            oracle_dump_buf[2790] = sat;
            for (int k = 0; k < 6; ++k) { oracle_dump_buf[2700 + k] = a0[k]; oracle_dump_buf[2710 + k] = v0[k]; }
            for (int d = 0; d < D; ++d) oracle_dump_buf[2800 + d] = qdd[d];
        }
        real qds[MAXD];
        V6 v0s;
        memcpy(qds, qd, sizeof(real) * D);
        for (int g = 1; g < G; ++g) qds[w.gdof[g]] = qd[w.gdof[g]] + h * qdd[w.gdof[g]];
        for (int k = 0; k < 6; ++k) v0s[k] = v0[k] + h * a0[k];
        {   /* classical (world-fixed) linear acceleration: spatial + w x v */
            V3 wv = {v0[0], v0[1], v0[2]}, vv = {v0[3], v0[4], v0[5]}, wxv;
            cross3(wv, vv, wxv);
            for (int k = 0; k < 3; ++k) v0s[3 + k] += h * wxv[k];
        }
        real qdv[MAXD];
        V6 v0v;
        solve_contacts(&e, &w, h, qds, v0s, qdv, v0v);
        /* velocity limits, integrate: positions with the velocity of the
         * biased sweeps, the stored velocity the bias-free one */
        for (int g = 1; g < G; ++g) {
            int d = w.gdof[g];
            real vl = props[TG_PROP_VELOCITY * prop_stride + d];
            if (vl > 0) qds[d] = qds[d] > vl ? vl : (qds[d] < -vl ? -vl : qds[d]);
            if (vl > 0) qdv[d] = qdv[d] > vl ? vl : (qdv[d] < -vl ? -vl : qdv[d]);
            qd[d] = qdv[d];
            q[d] += h * qds[d];
        }
        if (!sp->fix_base) {
            memcpy(v0, v0s, sizeof v0);
            V3 vbw, vbl = {v0[3], v0[4], v0[5]};
            m3_v(R, vbl, vbw);
            for (int k = 0; k < 3; ++k) pos[k] += h * vbw[k];
            /* q <- q * exp(h w_b / 2) */
            real wx = v0[0], wy = v0[1], wz = v0[2], an = sqrt(wx * wx + wy * wy + wz * wz) * h;
            real dq[4] = {0, 0, 0, 1};
            if (an > 1e-12) {
                real sa = sin(an / 2) / (an / h);
                dq[0] = wx * sa; dq[1] = wy * sa; dq[2] = wz * sa; dq[3] = cos(an / 2);
            }
            real x1 = quat[0], y1 = quat[1], z1 = quat[2], w1 = quat[3];
            real x2 = dq[0], y2 = dq[1], z2 = dq[2], w2 = dq[3];
            quat[0] = w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2;
            quat[1] = w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2;
            quat[2] = w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2;
            quat[3] = w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2;
            qn = sqrt(quat[0] * quat[0] + quat[1] * quat[1] + quat[2] * quat[2] + quat[3] * quat[3]);
            for (int k = 0; k < 4; ++k) quat[k] /= qn;
            quat_to_m3(quat, R);
            /* the stored (bias-free) velocity, re-expressed in the rotated body
             * frame as a world-fixed vector: v <- Rot(dq)^T v */
            memcpy(v0, v0v, sizeof v0);
            M3 Rd;
            quat_to_m3(dq, Rd);
            V3 wv = {v0[0], v0[1], v0[2]}, vv = {v0[3], v0[4], v0[5]};
            m3T_v(Rd, wv, wv);
            m3T_v(Rd, vv, vv);
            for (int k = 0; k < 3; ++k) { v0[k] = wv[k]; v0[3 + k] = vv[k]; }
        }
    }
    /* write back: root pose, com velocity (world), angular velocity (world) */
    V3 wbw, vow, wb2 = {v0[0], v0[1], v0[2]}, vb2 = {v0[3], v0[4], v0[5]};
    m3_v(R, wb2, wbw);
    m3_v(R, vb2, vow);
    m3_v(R, c0, c0w);
    cross3(wbw, c0w, wxc);
    for (int k = 0; k < 3; ++k) {
        root[k] = (float)pos[k];
        root[7 + k] = (float)(vow[k] + wxc[k]);
        root[10 + k] = (float)wbw[k];
    }
    for (int k = 0; k < 4; ++k) root[3 + k] = (float)quat[k];
    for (int d = 0; d < D; ++d) {
        if (m->dof_locked[d]) {
            dof[2 * d] = (float)lockq[d];
            dof[2 * d + 1] = 0.0f;
        } else {
            dof[2 * d] = (float)q[d];
            dof[2 * d + 1] = (float)qd[d];
        }
    }
}

/* Batched driver: state arrays in the tgsim.h layouts. */
void oracle_physics_step(const tg_model_desc *m, const tg_sim_params *sp, int n, float *root, float *dof,
                         const float *props, const float *pos_tgt, const float *vel_tgt, const float *act,
                         const float *force, const float *mass_scale, const float *mu, const float *gravity,
                         int nthreads) {
    int D = m->num_dofs;
    long stride = (long)n * D;   /* props are [F][N][D] */
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int e = 0; e < n; ++e) {
        t_env = e;
        oracle_physics_step_env(m, sp, root + 13 * (long)e, dof + 2 * (long)e * D, props + (long)e * D, stride,
                                pos_tgt + (long)e * D, vel_tgt + (long)e * D, act ? act + (long)e * D : NULL,
                                force ? force + 6L * e * m->num_groups : NULL,
                                mass_scale ? mass_scale + (long)e * m->num_links : NULL, mu + (long)e * m->num_shapes,
                                gravity);
    }
}

/* World state of every link (tg_rigid_body_states): root link from the root
 * state (its linear velocity is the root link's com velocity), then every
 * link from its parent in model order: R_l = R_p Ro Rj(q), p_l = p_p + R_p (to
 * + q s); w_l = w_p + qd a_w (revolute); v_l(origin) = v_p + w_p x (p_l - p_p)
 * + qd a_w (prismatic), a_w = R_p Ro a.  out[e][l] = (p, quat xyzw, com
 * velocity, w).  Test infrastructure (fp64). */
static void m3_to_quat_d(const M3 R, real *q) {
    real tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        real s = 0.5 / sqrt(tr + 1);
        q[3] = 0.25 / s; q[0] = (R[7] - R[5]) * s; q[1] = (R[2] - R[6]) * s; q[2] = (R[3] - R[1]) * s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        real s = 2 * sqrt(1 + R[0] - R[4] - R[8]);
        q[3] = (R[7] - R[5]) / s; q[0] = 0.25 * s; q[1] = (R[1] + R[3]) / s; q[2] = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        real s = 2 * sqrt(1 + R[4] - R[0] - R[8]);
        q[3] = (R[2] - R[6]) / s; q[0] = (R[1] + R[3]) / s; q[1] = 0.25 * s; q[2] = (R[5] + R[7]) / s;
    } else {
        real s = 2 * sqrt(1 + R[8] - R[0] - R[4]);
        q[3] = (R[3] - R[1]) / s; q[0] = (R[2] + R[6]) / s; q[1] = (R[5] + R[7]) / s; q[2] = 0.25 * s;
    }
}

/* world pose and velocity of every link of env e (links in tree order):
 * R_l, P_l (link origin), W_l, V_l (velocity of the link origin) */
static void fk_links(const tg_model_desc *m, const float *r, const float *q, M3 *R, V3 *P, V3 *W, V3 *V) {
    int L = m->num_links;
    for (int l = 0; l < L; ++l) {
        int p = m->link_parent[l];
        const float *in = m->link_inertia + 10 * l;
        V3 c = {in[1], in[2], in[3]}, Rc;
        if (p < 0) {
            real qq[4] = {r[3], r[4], r[5], r[6]};
            real nq = sqrt(qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2] + qq[3] * qq[3]);
            for (int k = 0; k < 4; ++k) qq[k] /= nq;
            quat_to_m3(qq, R[l]);
            for (int k = 0; k < 3; ++k) { P[l][k] = r[k]; W[l][k] = r[10 + k]; }
            m3_v(R[l], c, Rc);
            V3 wxc;
            cross3(W[l], Rc, wxc);
            for (int k = 0; k < 3; ++k) V[l][k] = r[7 + k] - wxc[k];
            continue;
        }
        const float *o = m->link_origin + 12 * l;
        M3 Ro, Rj;
        V3 to = {o[9], o[10], o[11]}, ax = {m->link_axis[3 * l], m->link_axis[3 * l + 1], m->link_axis[3 * l + 2]};
        for (int k = 0; k < 9; ++k) Ro[k] = o[k];
        int d = m->link_dof[l];
        real qq = d >= 0 ? q[2 * d] : 0.0, qd = d >= 0 ? q[2 * d + 1] : 0.0;
        V3 s, aw;
        m3_v(Ro, ax, s);
        m3_v(R[p], s, aw);
        memcpy(W[l], W[p], sizeof(V3));
        if (m->link_jtype[l] == TG_JOINT_REVOLUTE) {
            axis_angle(ax, qq, Rj);
            m3_mul(Ro, Rj, Ro);
            for (int k = 0; k < 3; ++k) W[l][k] += qd * aw[k];
        } else if (m->link_jtype[l] == TG_JOINT_PRISMATIC) {
            for (int k = 0; k < 3; ++k) to[k] += qq * s[k];
        }
        m3_mul(R[p], Ro, R[l]);
        V3 t, dp, wxd;
        m3_v(R[p], to, t);
        for (int k = 0; k < 3; ++k) { P[l][k] = P[p][k] + t[k]; dp[k] = t[k]; }
        cross3(W[p], dp, wxd);
        for (int k = 0; k < 3; ++k) V[l][k] = V[p][k] + wxd[k];
        if (m->link_jtype[l] == TG_JOINT_PRISMATIC)
            for (int k = 0; k < 3; ++k) V[l][k] += qd * aw[k];
    }
}

void oracle_rigid_body_states(const tg_model_desc *m, int n, const float *root, const float *dof, float *out) {
    int L = m->num_links, D = m->num_dofs;
    for (int e = 0; e < n; ++e) {
        M3 R[MAXL];
        V3 P[MAXL], W[MAXL], V[MAXL];
        fk_links(m, root + 13L * e, dof + 2L * e * D, R, P, W, V);
        for (int l = 0; l < L; ++l) {
            const float *in = m->link_inertia + 10 * l;
            V3 c = {in[1], in[2], in[3]}, Rc, wxc;
            m3_v(R[l], c, Rc);
            cross3(W[l], Rc, wxc);
            real qo[4];
            m3_to_quat_d(R[l], qo);
            float *o = out + (13L * L) * e + 13L * l;
            for (int k = 0; k < 3; ++k) o[k] = (float)P[l][k];
            for (int k = 0; k < 4; ++k) o[3 + k] = (float)qo[k];
            for (int k = 0; k < 3; ++k) { o[7 + k] = (float)(V[l][k] + wxc[k]); o[10 + k] = (float)W[l][k]; }
        }
    }
}

/* apply_rigid_body_force_tensors (isaacgym gymapi; reference call site
 * tasks/gogoro_realistic_turning_sim_paper.py:457): per-link forces f_l
 * [N*L,3] acting at the link's centre of mass and optional torques t_l
 * [N*L,3], in the world frame (space 0, ENV_SPACE) or the link frame (space 1,
 * LOCAL_SPACE), reduced to one wrench per group at the group's centre of mass
 * (the tg_apply_body_forces layout [N,G,6], world frame):
 *   F_g = sum f_l,   T_g = sum t_l + (p_l - c_g) x f_l,
 * p_l = P_l + R_l c_l the link's com and c_g = sum m_l s_l p_l / sum m_l s_l
 * (s_l: the per-env mass scale, NULL = 1) from the current root / dof state
 * (massless group: its root link's origin).  Sums in link order. */
void oracle_rigid_body_force_wrench(const tg_model_desc *m, int n, const float *root, const float *dof,
                                    const float *mass_scale, const float *forces, const float *torques, int space,
                                    float *out) {
    int L = m->num_links, D = m->num_dofs, G = m->num_groups;
    for (int e = 0; e < n; ++e) {
        M3 R[MAXL];
        V3 P[MAXL], W[MAXL], V[MAXL], pc[MAXL], f[MAXL], t[MAXL];
        fk_links(m, root + 13L * e, dof + 2L * e * D, R, P, W, V);
        real gm[MAXL], gc[MAXL][3];
        for (int g = 0; g < G; ++g) { gm[g] = 0; gc[g][0] = gc[g][1] = gc[g][2] = 0; }
        for (int l = 0; l < L; ++l) {
            const float *in = m->link_inertia + 10 * l;
            V3 c = {in[1], in[2], in[3]}, Rc;
            m3_v(R[l], c, Rc);
            for (int k = 0; k < 3; ++k) pc[l][k] = P[l][k] + Rc[k];
            real ml = in[0] * (mass_scale ? mass_scale[(size_t)e * L + l] : 1.0f);
            int g = m->link_group[l];
            gm[g] += ml;
            for (int k = 0; k < 3; ++k) gc[g][k] += ml * pc[l][k];
            V3 fl = {forces[3 * ((size_t)e * L + l)], forces[3 * ((size_t)e * L + l) + 1],
                     forces[3 * ((size_t)e * L + l) + 2]};
            V3 tl = {0, 0, 0};
            if (torques)
                for (int k = 0; k < 3; ++k) tl[k] = torques[3 * ((size_t)e * L + l) + k];
            if (space == 1) {
                m3_v(R[l], fl, f[l]);
                m3_v(R[l], tl, t[l]);
            } else {
                memcpy(f[l], fl, sizeof(V3));
                memcpy(t[l], tl, sizeof(V3));
            }
        }
        for (int g = 0; g < G; ++g) {
            int r = m->group_root[g];
            for (int k = 0; k < 3; ++k) gc[g][k] = gm[g] > 0 ? gc[g][k] / gm[g] : P[r][k];
        }
        float *o = out + (size_t)6 * G * e;
        real acc[MAXL][6];
        memset(acc, 0, sizeof(real) * 6 * G);
        for (int l = 0; l < L; ++l) {
            int g = m->link_group[l];
            V3 d = {pc[l][0] - gc[g][0], pc[l][1] - gc[g][1], pc[l][2] - gc[g][2]}, dxf;
            cross3(d, f[l], dxf);
            for (int k = 0; k < 3; ++k) { acc[g][k] += f[l][k]; acc[g][3 + k] += t[l][k] + dxf[k]; }
        }
        for (int g = 0; g < G; ++g)
            for (int k = 0; k < 6; ++k) o[6 * g + k] = (float)acc[g][k];
    }
}
