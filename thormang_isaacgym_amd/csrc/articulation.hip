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
#include "launch.h"

namespace tg {

// dispatch: this unit's models, then the humanoid unit's
// (articulation_tree.hip), then the run-time (hipRTC) models
int launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    int rc = unit_launch_step(hash, a, stream, ev_begin, ev_end);
    if (rc == TG_OTHER_UNIT) rc = tree_launch_step(hash, a, stream, ev_begin, ev_end);
    return rc == TG_OTHER_UNIT ? jit_launch_step(hash, a, stream, ev_begin, ev_end) : rc;
}

int launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                       hipEvent_t ev_begin, hipEvent_t ev_end) {
    int rc = unit_launch_step_gogoro(hash, a, pa, stream, ev_begin, ev_end);
    if (rc == TG_OTHER_UNIT) rc = tree_launch_step_gogoro(hash, a, pa, stream, ev_begin, ev_end);
    if (rc != TG_OTHER_UNIT) return rc;
    return jit_has(hash) ? 1 : TG_ERR_MODEL;   // run-time models: no fused epilogue
}

int launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                     hipEvent_t ev_begin, hipEvent_t ev_end) {
    int rc = unit_launch_step_walk(hash, a, pa, stream, ev_begin, ev_end);
    if (rc == TG_OTHER_UNIT) rc = tree_launch_step_walk(hash, a, pa, stream, ev_begin, ev_end);
    if (rc != TG_OTHER_UNIT) return rc;
    return jit_has(hash) ? 1 : TG_ERR_MODEL;
}

int launch_step_paper(uint64_t hash, const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream,
                      hipEvent_t ev_begin, hipEvent_t ev_end) {
    int rc = unit_launch_step_paper(hash, a, pa, stream, ev_begin, ev_end);
    if (rc == TG_OTHER_UNIT) rc = tree_launch_step_paper(hash, a, pa, stream, ev_begin, ev_end);
    if (rc != TG_OTHER_UNIT) return rc;
    return jit_has(hash) ? 1 : TG_ERR_MODEL;
}

#ifdef TG_DUMP_ENV
// developer build only: select the env whose contact solve the step kernels
// dump (first-substep or the given substep), in BOTH units -- the scooters and
// the known-answer models run in this unit, the humanoid trees in
// articulation_tree.hip -- and read back whichever unit's kernel fired (its
// buffer's word 0 holds the row count; scripts/dev/contact_dump.py)
int tree_dump_arm(int e, int substep);
int tree_dump_read(float *out, int n);
extern "C" int tg_debug_dump_env(int e, int substep) {
    static float zero[4096];
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_buf), zero, sizeof zero) != hipSuccess) return -2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_sub), &substep, sizeof(int)) != hipSuccess) return -2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_env), &e, sizeof(int)) != hipSuccess) return -2;
    return tree_dump_arm(e, substep);
}
extern "C" int tg_debug_dump_read(float *out, int n) {
    if (n > 4096) n = 4096;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_dump_buf), (size_t)n * 4) != hipSuccess) return -2;
    if (n > 0 && out[0] != 0.f) return 0;          // this unit's kernel dumped
    return tree_dump_read(out, n);              // else the humanoid unit's (or nothing: zeros)
}
#endif

#ifdef TG_SECTION_PROF
// developer builds: the section counters, summed over both units' step kernels
int tree_cprof_read(unsigned long long *out, int n);
int tree_prof_read(unsigned long long *out, int n);
extern "C" int tg_cprof_read(unsigned long long *out, int n) {
    unsigned long long a[8] = {}, b[8] = {};
    if (hipMemcpyFromSymbol(a, HIP_SYMBOL(tg_cprof_acc), sizeof a) != hipSuccess || tree_cprof_read(b, 8)) return -1;
    for (int k = 0; k < n && k < 8; ++k) out[k] = a[k] + b[k];
    return 0;
}
extern "C" int tg_prof_read(unsigned long long *out, int n) {
    unsigned long long a[24] = {}, b[24] = {};
    if (hipMemcpyFromSymbol(a, HIP_SYMBOL(tg_prof_acc), sizeof a) != hipSuccess || tree_prof_read(b, 24)) return -1;
    for (int k = 0; k < n && k < 24; ++k) out[k] = a[k] + b[k];
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
#define TG_EPB(MODEL) if (hash == MODEL::hash) return MODEL::EPB;
int model_epb(uint64_t hash) {
    TG_FOR_EACH_MODEL(TG_EPB)
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

