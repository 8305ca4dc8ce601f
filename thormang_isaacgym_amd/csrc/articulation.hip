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

#include <atomic>

#include "generated/models.inc"
#include "articulation_kernels.h"

namespace tg {

// ---------------------------------------------------------------- dispatch
// compose (dirty envs only), then the tree-parallel LDS-resident step,
// M::EPB envs x M::LPE lanes per workgroup (Thormang: 16 envs, 151 KB of LDS).

// the compose launch before a step kernel: none (no env can be dirty and no
// prologue), the listed envs of the last fused epilogue (compose_list_kernel),
// or every dirty env (compose_kernel)
template <class M> void launch_compose(const StepArgs &a, hipStream_t stream) {
    if (a.skip_compose) return;
    if (a.compose_list) {
        hipLaunchKernelGGL(compose_list_kernel<M>, dim3((a.N + COMPOSE_WPB - 1) / COMPOSE_WPB), dim3(64), 0, stream,
                           a);
    } else {
        hipLaunchKernelGGL(compose_kernel<M>, dim3((a.N + COMPOSE_WPB - 1) / COMPOSE_WPB), dim3(64 * COMPOSE_WPB), 0,
                           stream, a);
        if (a.cuni) {   // shared-cache flag for the step kernels that follow
            (void)hipMemsetD32Async(a.cuni, 1, 1, stream);
            hipLaunchKernelGGL(uniform_check_kernel<M>, dim3(a.N), dim3(64), 0, stream, a);
        }
    }
}

// HF: terrain heightfield present (tg_set_heightfield); the flat-ground
// instantiation keeps the contact normal a compile-time e_z.
template <class M, bool HF, class P = NoPost>
int launch_par(const StepArgs &a, hipStream_t stream, const typename P::Args &pa = {}) {
    constexpr size_t bytes = ParLayout<M>::template bytes<alias_slots<M>(M::EPB)>();
    static_assert(bytes <= 160 * 1024, "LDS budget");
#ifdef TG_EPB_DEV   // developer experiment: fewer envs per workgroup, the full LDS allocated (waves per CU)
    constexpr int EPBX = M::PAIR ? TG_EPB_DEV : M::EPB;
#else
    constexpr int EPBX = M::EPB;
#endif
    // the dynamic-LDS attribute is per device: one bit per device of this
    // instantiation, set the first time the kernel launches there (sims on
    // several devices in one process, from any thread)
    static std::atomic<uint64_t> attr_set{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return TG_ERR_HIP;
    const uint64_t bit = 1ull << dev;
    if (!(attr_set.load(std::memory_order_acquire) & bit)) {
        if (hipFuncSetAttribute((const void *)step_par_kernel<M, EPBX, HF, P>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess)
            return TG_ERR_HIP;
        attr_set.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL((step_par_kernel<M, EPBX, HF, P>), dim3((a.N + EPBX - 1) / EPBX), dim3(EPBX * M::LPE),
                       bytes, stream, a, pa);
    return 0;
}

template <class M> int launch_model(const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    launch_compose<M>(a, stream);
    if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
    if (int rc = a.hf ? launch_par<M, true>(a, stream) : launch_par<M, false>(a, stream)) return rc;
    if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
}

#define TG_LAUNCH(MODEL) \
    if (hash == MODEL::hash) return launch_model<MODEL>(a, stream, ev_begin, ev_end);

int launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_LAUNCH)
    return jit_launch_step(hash, a, stream, ev_begin, ev_end);
}

// the fused walk epilogue is instantiated for the lane-pair (humanoid-size)
// trees on flat ground only
template <class M>
int launch_model_walk(const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream, hipEvent_t ev_begin,
                      hipEvent_t ev_end) {
    if constexpr (M::PAIR == 0 || M::ND > 64) {
        return 1;
    } else {
        if (a.hf || pa.p.num_dof != M::ND) return 1;
        launch_compose<M>(a, stream);
        if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
        if (int rc = launch_par<M, false, WalkPost>(a, stream, pa)) return rc;
        if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
    }
}

// the fused Gogoro epilogue is instantiated for the registered task's model
// (codegen FUSED bit 1), flat ground and terrain
template <class M>
int launch_model_gogoro(const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream, hipEvent_t ev_begin,
                        hipEvent_t ev_end) {
    if constexpr ((M::FUSED & 2) == 0) {
        return 1;
    } else {
        if (pa.p.num_dof != M::ND) return 1;
        launch_compose<M>(a, stream);
        if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
        if (int rc = a.hf ? launch_par<M, true, GogoroPost>(a, stream, pa) : launch_par<M, false, GogoroPost>(a, stream, pa))
            return rc;
        if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
    }
}

#define TG_LAUNCH_GOGORO(MODEL) \
    if (hash == MODEL::hash) return launch_model_gogoro<MODEL>(a, pa, stream, ev_begin, ev_end);

int launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                       hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_LAUNCH_GOGORO)
    return jit_has(hash) ? 1 : TG_ERR_MODEL;   // run-time models: no fused epilogue
}

#define TG_LAUNCH_WALK(MODEL) \
    if (hash == MODEL::hash) return launch_model_walk<MODEL>(a, pa, stream, ev_begin, ev_end);

int launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                     hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_LAUNCH_WALK)
    return jit_has(hash) ? 1 : TG_ERR_MODEL;
}

#ifdef TG_SECTION_PROF
extern "C" int tg_cprof_read(unsigned long long *out, int n) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_cprof_acc), sizeof(unsigned long long) * (n < 8 ? n : 8)) != hipSuccess)
        return -1;
    return 0;
}
extern "C" int tg_prof_read(unsigned long long *out, int n) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_prof_acc), sizeof(unsigned long long) * (n < 24 ? n : 24)) != hipSuccess)
        return -1;
    return 0;
}
#endif

#define TG_HASH(MODEL) if (n < cap) out[n] = MODEL::hash; ++n;
#define TG_KC(MODEL) if (hash == MODEL::hash) return MODEL::KC;

#define TG_BODY_STATES(MODEL)                                                                              \
    if (hash == MODEL::hash) {                                                                             \
        hipLaunchKernelGGL(body_state_kernel<MODEL>, dim3(n), dim3(64), 0, stream, root, dof, n, out);   \
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;                                           \
    }

int launch_body_states(uint64_t hash, const float *root, const float *dof, int n, float *out, hipStream_t stream) {
    TG_FOR_EACH_MODEL(TG_BODY_STATES)
    return jit_launch_body_states(hash, root, dof, n, out, stream);
}

#define TG_RB_FORCES(MODEL)                                                                               \
    if (hash == MODEL::hash) {                                                                            \
        hipLaunchKernelGGL(rb_force_kernel<MODEL>, dim3((n + COMPOSE_WPB - 1) / COMPOSE_WPB), dim3(64 * COMPOSE_WPB), \
                           0, stream, root, dof, comp, n,                                                 \
                           mass_scale, forces, torques, space, out, props);                               \
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;                                          \
    }

int launch_rb_forces(uint64_t hash, const float *root, const float *dof, const float *comp, int n,
                     const float *mass_scale, const float *forces, const float *torques, int space, float *out,
                     const float *props, hipStream_t stream) {
    TG_FOR_EACH_MODEL(TG_RB_FORCES)
    return jit_launch_rb_forces(hash, root, dof, comp, n, mass_scale, forces, torques, space, out, props, stream);
}

int compiled_hashes(uint64_t *out, int cap) {
    int n = 0;
    TG_FOR_EACH_MODEL(TG_HASH)
    return n;
}
#define TG_COMPOSE_ONLY(MODEL)                                                                            \
    if (hash == MODEL::hash) {                                                                            \
        hipLaunchKernelGGL(compose_kernel<MODEL>, dim3((a.N + COMPOSE_WPB - 1) / COMPOSE_WPB),            \
                           dim3(64 * COMPOSE_WPB), 0, stream, a);                                         \
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;                                          \
    }
int launch_compose_only(uint64_t hash, const StepArgs &a, hipStream_t stream) {
    TG_FOR_EACH_MODEL(TG_COMPOSE_ONLY)
    return TG_ERR_MODEL;
}
#define TG_FUSED(MODEL) if (hash == MODEL::hash) return MODEL::FUSED;
int model_fused(uint64_t hash) {
    TG_FOR_EACH_MODEL(TG_FUSED)
    return 0;
}
#define TG_TL(MODEL) if (hash == MODEL::hash) return MODEL::NTL;
int model_tl(uint64_t hash) {
    TG_FOR_EACH_MODEL(TG_TL)
    return 0;
}
int model_kc(uint64_t hash) {
    TG_FOR_EACH_MODEL(TG_KC)
    return jit_kc(hash);
}

}  // namespace tg

#ifdef TG_DUMP_ENV
// developer build only: select the env whose first-substep contact solve the
// step kernel dumps, and read the dump back (scripts/dev/contact_dump.py)
extern "C" int tg_debug_dump_env(int e, int substep) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg::tg_dump_sub), &substep, sizeof(int)) != hipSuccess) return -2;
    return hipMemcpyToSymbol(HIP_SYMBOL(tg::tg_dump_env), &e, sizeof(int)) == hipSuccess ? 0 : -2;
}
extern "C" int tg_debug_dump_read(float *out, int n) {
    if (n > 4096) n = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tg::tg_dump_buf), (size_t)n * 4) == hipSuccess ? 0 : -2;
}
#endif
