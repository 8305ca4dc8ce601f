// Device-side small linear algebra for the articulation kernels (fp32).
// Spatial conventions: motion [w; v], force [n; f]; Xf = child-from-parent
// (E: parent->child coordinates, r: child origin in parent coordinates).
#pragma once
#include <hip/hip_runtime.h>

namespace tg {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

struct M3 {
    float a[9];   // row-major
};
__device__ __forceinline__ M3 eye3() { return M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}}; }
__device__ __forceinline__ V3 mul(const M3 &m, V3 v) {
    return V3{m.a[0] * v.x + m.a[1] * v.y + m.a[2] * v.z, m.a[3] * v.x + m.a[4] * v.y + m.a[5] * v.z,
              m.a[6] * v.x + m.a[7] * v.y + m.a[8] * v.z};
}
#ifndef TG_PK
#define TG_PK 0   // developer switch, measured off (round 5, profiles/r5/packed_m3_static.txt)
#endif
#if TG_PK
// packed FP32 (v_pk_mul_f32 / v_pk_fma_f32, two products in one VALU issue):
// a row-major row pair times a broadcast scalar (op_sel picks the scalar's
// half); the same products and contraction order as the scalar forms, so the
// results are bit-identical.  Off: on the walk kernel it turns 316 scalar
// multiply-adds into 159 packed ones but adds 211 v_mov_b32 (the M3 values
// live in arbitrary registers, a packed operand needs an aligned pair), net
// +114 VALU instructions
typedef float tg_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ tg_f2 f2of(float a, float b) { return tg_f2{a, b}; }
__device__ __forceinline__ tg_f2 f2bc(float a) { return tg_f2{a, a}; }
__device__ __forceinline__ tg_f2 fma2(tg_f2 a, tg_f2 b, tg_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ V3 mulT(const M3 &m, V3 v) {
    const tg_f2 p = fma2(f2of(m.a[6], m.a[7]), f2bc(v.z),
                         fma2(f2of(m.a[3], m.a[4]), f2bc(v.y), f2of(m.a[0], m.a[1]) * f2bc(v.x)));
    return V3{p.x, p.y, __builtin_fmaf(m.a[8], v.z, __builtin_fmaf(m.a[5], v.y, m.a[2] * v.x))};
}
__device__ __forceinline__ M3 mul(const M3 &x, const M3 &y) {
    M3 o;
    const tg_f2 y0 = f2of(y.a[0], y.a[1]), y1 = f2of(y.a[3], y.a[4]), y2 = f2of(y.a[6], y.a[7]);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const tg_f2 p = fma2(f2bc(x.a[3 * i + 2]), y2, fma2(f2bc(x.a[3 * i + 1]), y1, f2bc(x.a[3 * i]) * y0));
        o.a[3 * i] = p.x;
        o.a[3 * i + 1] = p.y;
        o.a[3 * i + 2] = __builtin_fmaf(x.a[3 * i + 2], y.a[8], __builtin_fmaf(x.a[3 * i + 1], y.a[5], x.a[3 * i] * y.a[2]));
    }
    return o;
}
#else
__device__ __forceinline__ V3 mulT(const M3 &m, V3 v) {
    return V3{m.a[0] * v.x + m.a[3] * v.y + m.a[6] * v.z, m.a[1] * v.x + m.a[4] * v.y + m.a[7] * v.z,
              m.a[2] * v.x + m.a[5] * v.y + m.a[8] * v.z};
}
__device__ __forceinline__ M3 mul(const M3 &x, const M3 &y) {
    M3 o;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o.a[3 * i + j] = x.a[3 * i] * y.a[j] + x.a[3 * i + 1] * y.a[3 + j] + x.a[3 * i + 2] * y.a[6 + j];
    return o;
}
#endif
__device__ __forceinline__ M3 transpose(const M3 &m) {
    return M3{{m.a[0], m.a[3], m.a[6], m.a[1], m.a[4], m.a[7], m.a[2], m.a[5], m.a[8]}};
}
// sine and cosine of a joint angle: the hardware approximation (v_sin /
// v_cos on the angle in revolutions), or with TG_PRECISE_SINCOS (developer
// build, the drift study scripts/parity_drift.py --variants) the libm one
__device__ __forceinline__ void tg_sincos(float x, float *s, float *c) {
#ifdef TG_PRECISE_SINCOS
    sincosf(x, s, c);
#else
    __sincosf(x, s, c);
#endif
}
// rotation about a unit axis (Rodrigues); axis components are usually compile-time constants
__device__ __forceinline__ M3 rot_axis(float x, float y, float z, float q) {
    float s, c;
    tg_sincos(q, &s, &c);
    float t = 1.0f - c;
    return M3{{t * x * x + c, t * x * y - s * z, t * x * z + s * y, t * x * y + s * z, t * y * y + c, t * y * z - s * x,
               t * x * z - s * y, t * y * z + s * x, t * z * z + c}};
}
__device__ __forceinline__ M3 quat_to_m3(float x, float y, float z, float w) {
    return M3{{1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w), 2 * (x * y + z * w),
               1 - 2 * (x * x + z * z), 2 * (y * z - x * w), 2 * (x * z - y * w), 2 * (y * z + x * w),
               1 - 2 * (x * x + y * y)}};
}

// spatial vectors
struct SV {
    V3 w, v;
};
__device__ __forceinline__ SV sv0() { return SV{V3{0, 0, 0}, V3{0, 0, 0}}; }
__device__ __forceinline__ SV operator+(const SV &a, const SV &b) { return SV{a.w + b.w, a.v + b.v}; }
__device__ __forceinline__ SV operator*(float s, const SV &a) { return SV{s * a.w, s * a.v}; }
__device__ __forceinline__ float dot(const SV &a, const SV &b) { return dot(a.w, b.w) + dot(a.v, b.v); }
__device__ __forceinline__ SV crm(const SV &v, const SV &m) { return SV{cross(v.w, m.w), cross(v.w, m.v) + cross(v.v, m.w)}; }
__device__ __forceinline__ SV crf(const SV &v, const SV &f) { return SV{cross(v.w, f.w) + cross(v.v, f.v), cross(v.w, f.v)}; }

struct Xf {
    M3 E;
    V3 r;
};
__device__ __forceinline__ SV xmotion(const Xf &X, const SV &m) {   // X m
    return SV{mul(X.E, m.w), mul(X.E, m.v - cross(X.r, m.w))};
}
__device__ __forceinline__ SV xTforce(const Xf &X, const SV &f) {   // X^T f (child force -> parent)
    V3 Ef = mulT(X.E, f.v);
    return SV{mulT(X.E, f.w) + cross(X.r, Ef), Ef};
}

// symmetric 6x6 = [[A, B], [B^T, C]], A and C symmetric (xx yy zz xy xz yz), B row-major
struct SI {
    float A[6], B[9], C[6];
};
__device__ __forceinline__ V3 symmul(const float *S, V3 v) {
    return V3{S[0] * v.x + S[3] * v.y + S[4] * v.z, S[3] * v.x + S[1] * v.y + S[5] * v.z,
              S[4] * v.x + S[5] * v.y + S[2] * v.z};
}
__device__ __forceinline__ V3 bmul(const float *B, V3 v) {
    return V3{B[0] * v.x + B[1] * v.y + B[2] * v.z, B[3] * v.x + B[4] * v.y + B[5] * v.z, B[6] * v.x + B[7] * v.y + B[8] * v.z};
}
__device__ __forceinline__ V3 bTmul(const float *B, V3 v) {
    return V3{B[0] * v.x + B[3] * v.y + B[6] * v.z, B[1] * v.x + B[4] * v.y + B[7] * v.z, B[2] * v.x + B[5] * v.y + B[8] * v.z};
}
__device__ __forceinline__ SV mul(const SI &I, const SV &m) {
    return SV{symmul(I.A, m.w) + bmul(I.B, m.v), bTmul(I.B, m.w) + symmul(I.C, m.v)};
}
// rigid-body inertia at the frame origin: mass m, com c, rotational inertia about com Ic (xx yy zz xy xz yz)
__device__ __forceinline__ SI rb_inertia(float m, V3 c, const float *Ic) {
    SI I;
    I.A[0] = Ic[0] + m * (c.y * c.y + c.z * c.z);
    I.A[1] = Ic[1] + m * (c.x * c.x + c.z * c.z);
    I.A[2] = Ic[2] + m * (c.x * c.x + c.y * c.y);
    I.A[3] = Ic[3] - m * c.x * c.y;
    I.A[4] = Ic[4] - m * c.x * c.z;
    I.A[5] = Ic[5] - m * c.y * c.z;
    // B = m [c]x
    I.B[0] = 0;        I.B[1] = -m * c.z; I.B[2] = m * c.y;
    I.B[3] = m * c.z;  I.B[4] = 0;        I.B[5] = -m * c.x;
    I.B[6] = -m * c.y; I.B[7] = m * c.x;  I.B[8] = 0;
    I.C[0] = m; I.C[1] = m; I.C[2] = m; I.C[3] = 0; I.C[4] = 0; I.C[5] = 0;
    return I;
}
__device__ __forceinline__ void sym_from(float *S, const M3 &M) {
    S[0] = M.a[0]; S[1] = M.a[4]; S[2] = M.a[8]; S[3] = M.a[1]; S[4] = M.a[2]; S[5] = M.a[5];
}
__device__ __forceinline__ M3 sym_to(const float *S) { return M3{{S[0], S[3], S[4], S[3], S[1], S[5], S[4], S[5], S[2]}}; }
__device__ __forceinline__ void si_add(SI &a, const SI &b) {
#pragma unroll
    for (int k = 0; k < 6; ++k) { a.A[k] += b.A[k]; a.C[k] += b.C[k]; }
#pragma unroll
    for (int k = 0; k < 9; ++k) a.B[k] += b.B[k];
}
// I -= s * U U^T
__device__ __forceinline__ void si_sub_outer(SI &I, const SV &U, float s) {
    float uw[3] = {U.w.x, U.w.y, U.w.z}, uv[3] = {U.v.x, U.v.y, U.v.z};
    const int ii[6] = {0, 1, 2, 0, 0, 1}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        I.A[k] -= s * uw[ii[k]] * uw[jj[k]];
        I.C[k] -= s * uv[ii[k]] * uv[jj[k]];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) I.B[3 * i + j] -= s * uw[i] * uv[j];
}
// X^T I X : express an inertia given at the child frame in the parent frame.
// With X = [E 0; -E rx E] and I = [A B; B^T C]:
//   C' = E^T C E,  B' = E^T B E + rx C',  A' = E^T A E + Y + Y^T - (rx C') rx,  Y = rx (E^T B E)^T
// (symmetric blocks rotated as E^T (S E) keeping only the upper triangle).
__device__ __forceinline__ void sym_rot(const float *S, const M3 &E, float *o) {   // o = E^T S E (sym)
    const M3 T = mul(sym_to(S), E);
    const int ii[6] = {0, 1, 2, 0, 0, 1}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int i = ii[k], j = jj[k];
        o[k] = E.a[i] * T.a[j] + E.a[3 + i] * T.a[3 + j] + E.a[6 + i] * T.a[6 + j];
    }
}
__device__ __forceinline__ SI si_to_parent(const SI &I, const Xf &X) {
    SI o;
    sym_rot(I.A, X.E, o.A);
    sym_rot(I.C, X.E, o.C);
    const M3 Bq = mul(transpose(X.E), mul(M3{{I.B[0], I.B[1], I.B[2], I.B[3], I.B[4], I.B[5], I.B[6], I.B[7], I.B[8]}},
                                          X.E));
    const V3 r = X.r;
    const M3 C = sym_to(o.C);
    // Z = rx C'
    M3 Z;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        Z.a[j] = r.y * C.a[6 + j] - r.z * C.a[3 + j];
        Z.a[3 + j] = r.z * C.a[j] - r.x * C.a[6 + j];
        Z.a[6 + j] = r.x * C.a[3 + j] - r.y * C.a[j];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) o.B[k] = Bq.a[k] + Z.a[k];
    // Y = rx Bq^T: Y_ij = (r x Bq_row_j)_i
    M3 Y;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float b0 = Bq.a[3 * j], b1 = Bq.a[3 * j + 1], b2 = Bq.a[3 * j + 2];
        Y.a[j] = r.y * b2 - r.z * b1;
        Y.a[3 + j] = r.z * b0 - r.x * b2;
        Y.a[6 + j] = r.x * b1 - r.y * b0;
    }
    // W = Z rx (symmetric): W_ij = (Z_row_i x r)_j
    const int ii[6] = {0, 1, 2, 0, 0, 1}, jj[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int i = ii[k], j = jj[k];
        const float z0 = Z.a[3 * i], z1 = Z.a[3 * i + 1], z2 = Z.a[3 * i + 2];
        const float w = j == 0 ? z1 * r.z - z2 * r.y : (j == 1 ? z2 * r.x - z0 * r.z : z0 * r.y - z1 * r.x);
        o.A[k] += Y.a[3 * i + j] + Y.a[3 * j + i] - w;
    }
    return o;
}

// 6x6 SPD solve via LDL^T on the dense expansion of SI
struct LDL6 {
    float L[15];   // strictly lower, row-major packed
    float Dinv[6];
};
__device__ __forceinline__ LDL6 ldl6(const SI &I) {
    float M[6][6];
    M3 A = sym_to(I.A), C = sym_to(I.C);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            M[i][j] = A.a[3 * i + j];
            M[i][j + 3] = I.B[3 * i + j];
            M[i + 3][j] = I.B[3 * j + i];
            M[i + 3][j + 3] = C.a[3 * i + j];
        }
    LDL6 f;
    float Lf[6][6], D[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        float d = M[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= Lf[j][k] * Lf[j][k] * D[k];
        D[j] = d;
        f.Dinv[j] = 1.0f / d;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            float s = M[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) s -= Lf[i][k] * Lf[j][k] * D[k];
            Lf[i][j] = s * f.Dinv[j];
        }
    }
    int p = 0;
#pragma unroll
    for (int i = 1; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) f.L[p++] = Lf[i][j];
    return f;
}
__device__ __forceinline__ SV ldl6_solve(const LDL6 &f, const SV &b) {
    float x[6] = {b.w.x, b.w.y, b.w.z, b.v.x, b.v.y, b.v.z};
    // forward L y = b
#pragma unroll
    for (int i = 1; i < 6; ++i) {
        int base = i * (i - 1) / 2;
#pragma unroll
        for (int j = 0; j < i; ++j) x[i] -= f.L[base + j] * x[j];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] *= f.Dinv[i];
#pragma unroll
    for (int i = 4; i >= 0; --i) {
#pragma unroll
        for (int j = i + 1; j < 6; ++j) x[i] -= f.L[j * (j - 1) / 2 + i] * x[j];
    }
    return SV{V3{x[0], x[1], x[2]}, V3{x[3], x[4], x[5]}};
}

}  // namespace tg
