// launch.h -- the per-model launch templates of the step path (compose, the
// step kernel, the fused task epilogues), shared by the two units that
// instantiate them: articulation.hip (the scooters and the known-answer
// models) and articulation_tree.hip (the humanoid-size trees, NG >= 16).
// The units differ only in the machine scheduler they are compiled with
// (build_ext.py): each model's step kernel is instantiated in exactly one of
// them, chosen by TG_UNIT_TREE.
#pragma once

namespace tg {

#ifndef TG_UNIT_TREE
#define TG_UNIT_TREE 0
#endif
// a launch_* call for a model the other unit instantiates
constexpr int TG_OTHER_UNIT = -1000;
template <class M> constexpr bool in_unit() { return (M::NG >= 16) == (TG_UNIT_TREE != 0); }

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
#ifdef TG_GHOST_DEV   // (two real envs per wave: half the envs per workgroup)
    constexpr int EPRX = (M::PAIR && M::LPE == 16 && M::NG >= 16) ? EPBX / 2 : EPBX;
#else
    constexpr int EPRX = EPBX;
#endif
    hipLaunchKernelGGL((step_par_kernel<M, EPBX, HF, P>), dim3((a.N + EPRX - 1) / EPRX), dim3(EPBX * M::LPE),
                       bytes, stream, a, pa);
    return 0;
}

template <class M> int launch_model(const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    if constexpr (!in_unit<M>()) {
        return TG_OTHER_UNIT;
    } else {
    launch_compose<M>(a, stream);
    if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
    if (int rc = a.hf ? launch_par<M, true>(a, stream) : launch_par<M, false>(a, stream)) return rc;
    if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
    return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
    }
}

// the fused walk epilogue is instantiated for the lane-pair (humanoid-size)
// trees on flat ground only
template <class M>
int launch_model_walk(const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream, hipEvent_t ev_begin,
                      hipEvent_t ev_end) {
    if constexpr (!in_unit<M>()) {
        return TG_OTHER_UNIT;
    } else if constexpr (M::PAIR == 0 || M::ND > 64) {
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
    if constexpr (!in_unit<M>()) {
        return TG_OTHER_UNIT;
    } else if constexpr ((M::FUSED & 2) == 0) {
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

// the fused GogoroPaper epilogue (one launch per step): the paper model with
// in-place seat composites (codegen FUSED bit 4), flat ground
template <class M>
int launch_model_paper(const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream, hipEvent_t ev_begin,
                       hipEvent_t ev_end) {
    if constexpr (!in_unit<M>()) {
        return TG_OTHER_UNIT;
    } else if constexpr ((M::FUSED & 4) == 0 || M::NTL == 0 || !M::LCOM || M::NG > M::LPE || M::LPE < 8) {
        return 1;
    } else {
        if (a.hf || pa.p.num_dof != M::ND || a.N % M::EPB != 0) return 1;
        launch_compose<M>(a, stream);
        if (ev_begin && hipEventRecord(ev_begin, stream) != hipSuccess) return TG_ERR_HIP;
        if (int rc = launch_par<M, false, PaperPost>(a, stream, pa)) return rc;
        if (ev_end && hipEventRecord(ev_end, stream) != hipSuccess) return TG_ERR_HIP;
        return hipGetLastError() == hipSuccess ? 0 : TG_ERR_HIP;
    }
}

// this unit's dispatch (TG_OTHER_UNIT: a model this unit does not instantiate)
#define TG_U_LAUNCH(MODEL) \
    if (in_unit<MODEL>() && hash == MODEL::hash) return launch_model<MODEL>(a, stream, ev_begin, ev_end);
#define TG_U_LAUNCH_GOGORO(MODEL) \
    if (in_unit<MODEL>() && hash == MODEL::hash) return launch_model_gogoro<MODEL>(a, pa, stream, ev_begin, ev_end);
#define TG_U_LAUNCH_WALK(MODEL) \
    if (in_unit<MODEL>() && hash == MODEL::hash) return launch_model_walk<MODEL>(a, pa, stream, ev_begin, ev_end);
static int unit_launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin,
                            hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_U_LAUNCH)
    return TG_OTHER_UNIT;
}
static int unit_launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                                   hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_U_LAUNCH_GOGORO)
    return TG_OTHER_UNIT;
}
#define TG_U_LAUNCH_PAPER(MODEL) \
    if (in_unit<MODEL>() && hash == MODEL::hash) return launch_model_paper<MODEL>(a, pa, stream, ev_begin, ev_end);
static int unit_launch_step_paper(uint64_t hash, const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream,
                                  hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_U_LAUNCH_PAPER)
    return TG_OTHER_UNIT;
}
static int unit_launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                                 hipEvent_t ev_begin, hipEvent_t ev_end) {
    TG_FOR_EACH_MODEL(TG_U_LAUNCH_WALK)
    return TG_OTHER_UNIT;
}

// the humanoid unit's entries (articulation_tree.hip)
int tree_launch_step(uint64_t hash, const StepArgs &a, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end);
int tree_launch_step_gogoro(uint64_t hash, const StepArgs &a, const GogoroPostArgs &pa, hipStream_t stream,
                            hipEvent_t ev_begin, hipEvent_t ev_end);
int tree_launch_step_walk(uint64_t hash, const StepArgs &a, const WalkPostArgs &pa, hipStream_t stream,
                          hipEvent_t ev_begin, hipEvent_t ev_end);
int tree_launch_step_paper(uint64_t hash, const StepArgs &a, const PaperPostArgs &pa, hipStream_t stream,
                           hipEvent_t ev_begin, hipEvent_t ev_end);

}  // namespace tg
