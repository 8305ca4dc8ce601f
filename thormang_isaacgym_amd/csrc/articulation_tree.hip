// articulation_tree.hip -- the step kernels of the humanoid-size trees
// (NG >= 16: Thormang and its whole-body variant), the same templates as
// articulation.hip (launch.h, step_par.h), in a unit of their own so that
// build_ext.py can compile them with the machine scheduler that measured
// fastest for them ("Scheduler per unit").
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#define TG_UNIT_TREE 1
#include "generated/models.inc"
#include "articulation_kernels.h"
#include "launch.h"

namespace tg {

int tree_launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    return unit_launch_step(hash, a, stream, ev_begin, ev_end);
}
int tree_launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                            hipEvent_t ev_begin, hipEvent_t ev_end) {
    return unit_launch_step_gogoro(hash, a, pa, stream, ev_begin, ev_end);
}
int tree_launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                          hipEvent_t ev_begin, hipEvent_t ev_end) {
    return unit_launch_step_walk(hash, a, pa, stream, ev_begin, ev_end);
}
int tree_launch_step_paper(uint64_t hash, const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream,
                           hipEvent_t ev_begin, hipEvent_t ev_end) {
    return unit_launch_step_paper(hash, a, pa, stream, ev_begin, ev_end);
}

// developer builds: the section counters of this unit's step kernels
// (articulation.hip's tg_prof_read / tg_cprof_read add them to its own)
#ifdef TG_SECTION_PROF
int tree_cprof_read(unsigned long long *out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_cprof_acc), sizeof(unsigned long long) * (n < 8 ? n : 8)) ==
                   hipSuccess ? 0 : -1;
}
int tree_prof_read(unsigned long long *out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_prof_acc), sizeof(unsigned long long) * (n < 24 ? n : 24)) ==
                   hipSuccess ? 0 : -1;
}
#endif

}  // namespace tg

#ifdef TG_DUMP_ENV
// developer build only (scripts/dev/contact_dump.py): this unit's copies of
// the dump symbols (tg_dump_* are static __device__, so each unit's step
// kernels have their own); articulation.hip's tg_debug_dump_env /
// tg_debug_dump_read arm and read both units
namespace tg {
int tree_dump_arm(int e, int substep) {
    static float zero[4096];
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_buf), zero, sizeof zero) != hipSuccess) return -2;
    if (hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_sub), &substep, sizeof(int)) != hipSuccess) return -2;
    return hipMemcpyToSymbol(HIP_SYMBOL(tg_dump_env), &e, sizeof(int)) == hipSuccess ? 0 : -2;
}
int tree_dump_read(float *out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(tg_dump_buf), (size_t)n * 4) == hipSuccess ? 0 : -2;
}
}  // namespace tg
#endif
