// articulation.hip -- the per-env articulated-body step that replaces PhysX's
// gym.simulate (reference: isaacgymenvs/tasks/base/vec_task.py:332-335; model
// and drive set-up tasks/gogoro_new.py:196-294, cfg/task/Gogoro.yaml:9-31).
//
// The step kernel (step_par.h) is specialised per compiled model
// (generated/Model_*.inc, model/codegen.py): 8 lanes per env work through a
// list schedule of the joint tree with the env's articulated state resident in
// LDS.  This file holds the per-env composite cache (compose_kernel), the
// contact-row layout and the dispatch.
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

// ---------------------------------------------------------------- contact row layout
// rows of shape s: shape_nrows[s] normal rows, then friction t1, t2 and torsion
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

}  // namespace tg

#include "step_par.h"

namespace tg {

// ---------------------------------------------------------------- dispatch
// compose (dirty envs only), then the tree-parallel LDS-resident step,
// M::EPB envs x M::LPE lanes per workgroup (Thormang: 16 envs, 151 KB of LDS).

template <class M> int launch_model(const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    const dim3 cgrid((a.N + 63) / 64), cblock(64);
    hipLaunchKernelGGL(compose_kernel<M>, cgrid, cblock, 0, stream, a);
    constexpr size_t bytes = ParLayout<M>::template bytes<M::EPB>();
    static_assert(bytes <= 160 * 1024, "LDS budget");
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void *)step_par_kernel<M, M::EPB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)bytes) != hipSuccess)
            return TG_ERR_HIP;
        attr = true;
    }
    if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
    hipLaunchKernelGGL((step_par_kernel<M, M::EPB>), dim3((a.N + M::EPB - 1) / M::EPB), dim3(M::EPB * M::LPE), bytes,
                       stream, a);
    if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

#define TG_LAUNCH(MODEL) \
    if (hash == MODEL::hash) return launch_model<MODEL>(a, stream, ev_begin, ev_end);

int launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
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
