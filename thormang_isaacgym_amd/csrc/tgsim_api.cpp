// tgsim_api.cpp -- host side of the C-ABI (include/tgsim.h, include/tg_gogoro.h).
//
// Owns the per-sim device buffers (struct-of-arrays where the kernels want
// coalescing, the reference's AoS row layouts where the Python side expects
// IsaacGym-compatible tensor views), validates every call and reports errors
// through tg_last_error().  All work is stream-ordered on the sim's stream.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <cstdlib>
#include <memory>
#include <vector>

#include "../../include/tg_gogoro.h"
#include "../../include/tg_gogoro_paper.h"
#include "../../include/tgsim.h"
#include "tg_kernels.h"

namespace {
thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return fail(TG_ERR_HIP, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)
}  // namespace

struct tg_sim {
    int device = 0;
    int N = 0, D = 0, G = 0, L = 0, S = 0, KC = 0;
    uint64_t hash = 0;
    tg_sim_params params{};
    hipStream_t stream = nullptr;
    float gravity[3] = {0, 0, -9.81f};
    bool forces_pending = false;
    // apply_rigid_body_force_tensors waiting for the next simulate: reduced to
    // group wrenches by that simulate's compose launch, or by rb_force_kernel
    bool rbf_pending = false;
    const float *rbf_f = nullptr, *rbf_t = nullptr;
    int rbf_space = 0;
    // some env may be dirty (its composite cache stale): set by every call that
    // can mark envs dirty or change what compose reads (creation, state
    // binding, tg_refresh -- the contract for writes through the zero-copy
    // views --, property / mass-scale setters, the Gogoro and paper task
    // kernels, whose resets rewrite properties), cleared by a compose launch.
    // While false, a simulate without a compose prologue skips the compose
    // launch (one launch less per step; ThormangWalk's envs never go dirty)
    bool dirty_possible = true;
    // reset lists of the fused Gogoro epilogue (compose_list_kernel): two
    // slots of N ids + counts; the epilogue appends to slot list_cur, the next
    // compose reads the other one and zeroes list_cur's count; list_pending:
    // the last step kernel had that epilogue (its resets await their compose)
    int *clist = nullptr, *ccount = nullptr;
    int list_cur = 0;
    bool list_pending = false;
    // device buffers
    float *root = nullptr, *dof = nullptr, *pos_tgt = nullptr, *vel_tgt = nullptr, *act = nullptr;
    float *props = nullptr, *force = nullptr, *mass_scale = nullptr, *shape_mu = nullptr, *comp = nullptr;
    float *zero_link3 = nullptr;   // [N*L*3] zeros (torque-only rigid-body force calls), lazily allocated
    float *env_origin = nullptr;
    uint8_t *dirty = nullptr;
    int *err = nullptr;   // sticky state-error flag set by kernels (tg_sync reports it)
    // shared-cache flag (StepArgs::cuni) for compiled-in models whose task
    // kernels never edit composites / properties in place (not FUSED 2|4)
    int *cuni = nullptr;
    bool uni_ok = false;
    // terrain heightfield (tg_set_heightfield)
    float *hf = nullptr;
    int hf_rows = 0, hf_cols = 0;
    float hf_hs = 0.f, hf_vs = 0.f, hf_ox = 0.f, hf_oy = 0.f, hf_mu = 0.f;
    std::vector<void *> allocs;
    // kernel timing (tg_set_kernel_timing): event pairs recorded, not yet read
    bool walk_unfused = false;   // tg_walk_step: separate post-physics launch (TG_WALK_UNFUSED=1)
    bool post_unfused = false;   // tg_gogoro_step: separate post-physics launch (TG_POST_UNFUSED=1)
    bool always_compose = false; // never skip the compose launch (TG_ALWAYS_COMPOSE=1)
    bool pre_in_compose = false; // tg_walk_step: pre-physics in the compose launch, not the step kernel (TG_PRE_IN_COMPOSE=1)
    bool no_inplace = false;     // tg_gogoro_step: reset envs re-composed, not updated in place (TG_SEAT_RECOMPOSE=1)
    bool paper_finish_launch = false;   // tg_paper_step: term 7 summed by the finish launch (TG_PAPER_FINISH=1)
    bool paper_rb_launch = false;       // tg_paper_step: rb_forces reduced by rb_force_kernel (TG_PAPER_RB_LAUNCH=1)
    bool paper_two_launch = false;      // tg_paper_step: step kernel + post launch, never one launch (TG_PAPER_TWO_LAUNCH=1)
    // tg_paper_step in one launch (PaperPost): the term-7 arrival counter and
    // the total it reaches after the last launch; the device's CU count (the
    // grid must be resident at once)
    unsigned *t7cnt = nullptr;
    unsigned t7_total = 0;
    int num_cus = 0;
    int timing = 0;          // period (0: off; < 0: windows of -timing launches)
    int64_t timing_count = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_free;
    std::vector<int> ev_launches;   // step-kernel launches each pending pair brackets
    // windowed timing (tg_set_kernel_timing with a negative period): one event
    // pair around -timing consecutive step-kernel launches, dropped when any
    // other launch of the library falls inside it (win_dirty)
    std::pair<hipEvent_t, hipEvent_t> win{nullptr, nullptr};
    int win_n = 0;
    bool win_dirty = false;
    // tg_paper_step reduced its rb_forces (rbf_f) to the next simulate's group
    // wrenches already, from the state it left; any later call that can change
    // that state (every other launching entry point, tg_refresh, tg_bind_state)
    // turns them back into a pending tensor, reduced at the next simulate
    bool rbf_prereduced = false;
    double timed_ms = 0.0;
    int64_t timed_launches = 0;

    template <class T> int alloc(T **p, size_t count) {
        void *q = nullptr;
        if (count == 0) count = 1;
        hipError_t e = hipMalloc(&q, count * sizeof(T));
        if (e != hipSuccess) return fail(TG_ERR_HIP, "hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
        e = hipMemset(q, 0, count * sizeof(T));
        if (e != hipSuccess) return fail(TG_ERR_HIP, "hipMemset: %s", hipGetErrorString(e));
        allocs.push_back(q);
        *p = (T *)q;
        return 0;
    }
    ~tg_sim() {
        for (void *p : allocs) (void)hipFree(p);
        if (hf) (void)hipFree(hf);
        for (auto *v : {&ev_pending, &ev_free})
            for (auto &e : *v) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
        if (win.first) { (void)hipEventDestroy(win.first); (void)hipEventDestroy(win.second); }
    }
};

namespace {
// a launch other than the step kernel: an open timing window no longer
// brackets step kernels only
inline void win_touch(tg_sim *s) {
    if (s->win.first) s->win_dirty = true;
    if (s->rbf_prereduced) {
        s->rbf_pending = true;
        s->rbf_prereduced = false;
    }
}

int check_sim(tg_sim *s) { return s ? 0 : fail(TG_ERR_ARG, "null tg_sim"); }
int check_ids(tg_sim *s, const int32_t *ids, int32_t n) {
    if (n < 0 || n > s->N) return fail(TG_ERR_ARG, "index count %d out of range [0, %d]", n, s->N);
    if (n > 0 && !ids) return fail(TG_ERR_ARG, "null index pointer with n=%d", n);
    return 0;
}
tg::StepArgs step_args(tg_sim *s) {
    tg::StepArgs a{};
    const tg_sim_params &p = s->params;
    a.N = s->N;
    a.D = s->D;
    a.h = p.substeps > 0 ? p.dt / (float)p.substeps : 0.f;   // (0 substeps: tg_set_sim_params replay mode)
    a.substeps = p.substeps;
    a.gx = s->gravity[0]; a.gy = s->gravity[1]; a.gz = s->gravity[2];
    a.lin_damp = p.linear_damping;
    a.ang_damp = p.angular_damping;
    a.max_depen = p.max_depenetration_velocity;
    a.rest = p.rest_offset;
    a.margin = p.contact_margin;
    a.coff = p.contact_offset;
    a.ground_mu = p.ground_friction;
    a.baumgarte = p.baumgarte;
    a.lim_k = p.limit_stiffness;
    a.lim_c = p.limit_damping;
    a.iters = p.contact_iterations;
    a.viters = p.velocity_iterations;
    a.fix_base = p.fix_base;
    a.tgs = p.solver_type == 1 && p.contact_iterations > 0;
    a.root = s->root;
    a.dof = s->dof;
    a.pos_tgt = s->pos_tgt;
    a.vel_tgt = s->vel_tgt;
    a.act = s->act;
    a.props = s->props;
    a.force = s->forces_pending ? s->force : nullptr;
    a.shape_mu = s->shape_mu;
    a.mass_scale = s->mass_scale;
    a.comp = s->comp;
    a.dirty = s->dirty;
    a.err = s->err;
    a.cuni = s->uni_ok ? s->cuni : nullptr;
    a.hf = s->hf_rows > 0 ? s->hf : nullptr;
    a.hf_rows = s->hf_rows;
    a.hf_cols = s->hf_cols;
    a.hf_hs = s->hf_hs;
    a.hf_vs = s->hf_vs;
    a.hf_ox = s->hf_ox;
    a.hf_oy = s->hf_oy;
    a.hf_mu = s->hf_mu;
    return a;
}
}  // namespace

extern "C" {

const char *tg_last_error(void) { return g_err.c_str(); }

uint64_t tg_compiled_model_hashes(uint64_t *out, int32_t cap) { return (uint64_t)tg::compiled_hashes(out, cap); }

int tg_model_jit(uint64_t model_hash, const char *struct_name, const char *model_source, const char *include_dir,
                 const char *cache_dir) {
    if (!struct_name || !model_source) return fail(TG_ERR_ARG, "tg_model_jit: null argument");
    if (tg::model_kc(model_hash) >= 0 && !tg::jit_has(model_hash)) return TG_OK;   // compiled in
    std::string err;
    if (int rc = tg::jit_compile(model_hash, struct_name, model_source, include_dir, cache_dir, err))
        return fail(rc, "tg_model_jit(0x%016llx): %s", (unsigned long long)model_hash, err.c_str());
    return TG_OK;
}

int tg_sim_create(const tg_model_desc *m, const tg_sim_params *params, int32_t num_envs, int32_t device,
                  tg_sim **out) {
    if (!m || !params || !out) return fail(TG_ERR_ARG, "tg_sim_create: null argument");
    *out = nullptr;
    if (num_envs <= 0) return fail(TG_ERR_ARG, "num_envs must be positive (got %d)", num_envs);
    if (params->substeps <= 0 || !(params->dt > 0.f)) return fail(TG_ERR_ARG, "dt and substeps must be positive");
    if (params->contact_iterations < 0 || params->velocity_iterations < 0)
        return fail(TG_ERR_ARG, "contact / velocity iterations must be >= 0");
    if (params->solver_type != 0 && params->solver_type != 1)
        return fail(TG_ERR_ARG, "solver_type must be 0 (PGS) or 1 (TGS), got %d", params->solver_type);
    int kc = tg::model_kc(m->model_hash);
    if (kc < 0)
        return fail(TG_ERR_MODEL,
                    "model hash 0x%016llx has no specialisation in libtgsim.so: compiled-in models are listed by "
                    "tg_compiled_model_hashes; any other model must first be compiled with tg_model_jit",
                    (unsigned long long)m->model_hash);
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(TG_ERR_ARG, "device %d not present (%d visible)", device, ndev);
    HIPCHK(hipSetDevice(device));
    std::unique_ptr<tg_sim> owner(new tg_sim());   // released to the caller on success only
    tg_sim *s = owner.get();
    if (const char *u = getenv("TG_WALK_UNFUSED")) s->walk_unfused = u[0] == '1';
    if (const char *u = getenv("TG_POST_UNFUSED")) s->post_unfused = u[0] == '1';
    if (const char *u = getenv("TG_ALWAYS_COMPOSE")) s->always_compose = u[0] == '1';
    if (const char *u = getenv("TG_PRE_IN_COMPOSE")) s->pre_in_compose = u[0] == '1';
    if (const char *u = getenv("TG_SEAT_RECOMPOSE")) s->no_inplace = u[0] == '1';
    if (const char *u = getenv("TG_PAPER_FINISH")) s->paper_finish_launch = u[0] == '1';
    if (const char *u = getenv("TG_PAPER_RB_LAUNCH")) s->paper_rb_launch = u[0] == '1';
    if (const char *u = getenv("TG_PAPER_TWO_LAUNCH")) s->paper_two_launch = u[0] == '1';
    // (TG_NO_SHARED_CACHE=1: every env reads its own block, the A/B control)
    const char *nsc = getenv("TG_NO_SHARED_CACHE");
    s->uni_ok = !(nsc && nsc[0] == '1') && (tg::model_fused(m->model_hash) & 6) == 0 && !tg::jit_has(m->model_hash);
    s->device = device;
    s->N = num_envs;
    s->D = m->num_dofs;
    s->G = m->num_groups;
    s->L = m->num_links;
    s->S = m->num_shapes;
    s->KC = kc;
    s->hash = m->model_hash;
    s->params = *params;
    memcpy(s->gravity, params->gravity, sizeof s->gravity);
    const size_t N = num_envs;
    int rc = 0;
    rc |= s->alloc(&s->root, N * 13);
    rc |= s->alloc(&s->dof, N * s->D * 2);
    rc |= s->alloc(&s->pos_tgt, N * s->D);
    rc |= s->alloc(&s->vel_tgt, N * s->D);
    rc |= s->alloc(&s->act, N * s->D);
    rc |= s->alloc(&s->props, (size_t)TG_NUM_PROPS * N * s->D);
    rc |= s->alloc(&s->force, N * s->G * 6);
    rc |= s->alloc(&s->mass_scale, N * s->L);
    rc |= s->alloc(&s->shape_mu, N * (s->S > 0 ? s->S : 1));
    rc |= s->alloc(&s->comp, (size_t)kc * N);
    rc |= s->alloc(&s->env_origin, N * 3);
    rc |= s->alloc(&s->dirty, N);
    rc |= s->alloc(&s->err, 1);
    rc |= s->alloc(&s->cuni, 1);   // 0: not uniform until a compose checked it
    rc |= s->alloc(&s->clist, 2 * N);
    rc |= s->alloc(&s->ccount, 2);
    if (rc) return TG_ERR_HIP;   // g_err holds the failing allocation; owner frees the rest
    // host-side initial values: identity root pose at the env origin grid,
    // unit mass scale, per-shape friction from the model, defaults for props
    std::vector<float> h_root(N * 13, 0.f), h_org(N * 3, 0.f), h_ms(N * s->L, 1.f);
    std::vector<float> h_mu(N * (s->S > 0 ? s->S : 1), 1.f);
    std::vector<uint8_t> h_dirty(N, 1);
    const int per_row = params->envs_per_row > 0 ? params->envs_per_row : 1;
    for (size_t e = 0; e < N; ++e) {
        h_org[3 * e + 0] = 2.f * params->env_spacing * (float)(e % per_row);
        h_org[3 * e + 1] = 2.f * params->env_spacing * (float)(e / per_row);
        h_root[13 * e + 0] = h_org[3 * e + 0];
        h_root[13 * e + 1] = h_org[3 * e + 1];
        h_root[13 * e + 6] = 1.f;
        for (int k = 0; k < s->S; ++k) h_mu[e * s->S + k] = m->shape_friction[k];
    }
    std::vector<float> h_props((size_t)TG_NUM_PROPS * N * s->D, 0.f);
    for (size_t i = 0; i < N * s->D; ++i) {
        h_props[(size_t)TG_PROP_LOWER * N * s->D + i] = -3.4e38f;
        h_props[(size_t)TG_PROP_UPPER * N * s->D + i] = 3.4e38f;
    }
    HIPCHK(hipMemcpy(s->root, h_root.data(), h_root.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(s->env_origin, h_org.data(), h_org.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(s->mass_scale, h_ms.data(), h_ms.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(s->shape_mu, h_mu.data(), h_mu.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(s->dirty, h_dirty.data(), N, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(s->ccount, 0, 2 * sizeof(int)));
    HIPCHK(hipMemcpy(s->props, h_props.data(), h_props.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipDeviceSynchronize());
    *out = owner.release();
    return TG_OK;
}

int tg_sim_destroy(tg_sim *s) {
    if (!s) return TG_OK;
    (void)hipSetDevice(s->device);
    (void)hipDeviceSynchronize();
    delete s;
    return TG_OK;
}

int tg_set_stream(tg_sim *s, void *stream) {
    if (int rc = check_sim(s)) return rc;
    s->stream = (hipStream_t)stream;
    return TG_OK;
}

int tg_state_ptrs(tg_sim *s, tg_state_view *v) {
    if (int rc = check_sim(s)) return rc;
    if (!v) return fail(TG_ERR_ARG, "null view");
    v->root_state = s->root;
    v->dof_state = s->dof;
    v->dof_pos_target = s->pos_tgt;
    v->dof_vel_target = s->vel_tgt;
    v->dof_actuation = s->act;
    v->dof_props = s->props;
    v->body_force = s->force;
    v->env_origin = s->env_origin;
    v->env_dirty = s->dirty;
    v->num_envs = s->N;
    v->num_dofs = s->D;
    v->num_groups = s->G;
    v->num_links = s->L;
    return TG_OK;
}

int tg_refresh(tg_sim *s) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;   // writes through the zero-copy views (env_dirty, dof_props) take effect
    win_touch(s);
    return TG_OK;
}

int tg_bind_state(tg_sim *s, const tg_state_view *v) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    win_touch(s);
    if (!v) return fail(TG_ERR_ARG, "null view");
    const size_t N = s->N, D = s->D;
    struct B {
        void *src;
        void **dst;
        size_t bytes;
    } binds[] = {
        {v->root_state, (void **)&s->root, N * 13 * 4},
        {v->dof_state, (void **)&s->dof, N * D * 2 * 4},
        {v->dof_pos_target, (void **)&s->pos_tgt, N * D * 4},
        {v->dof_vel_target, (void **)&s->vel_tgt, N * D * 4},
        {v->dof_actuation, (void **)&s->act, N * D * 4},
        {v->dof_props, (void **)&s->props, (size_t)TG_NUM_PROPS * N * D * 4},
        {v->body_force, (void **)&s->force, N * s->G * 6 * 4},
        {v->env_origin, (void **)&s->env_origin, N * 3 * 4},
        {v->env_dirty, (void **)&s->dirty, N},
    };
    for (auto &b : binds) {
        if (!b.src || b.src == *b.dst) continue;
        HIPCHK(hipMemcpyAsync(b.src, *b.dst, b.bytes, hipMemcpyDeviceToDevice, s->stream));
        *b.dst = b.src;
    }
    HIPCHK(hipStreamSynchronize(s->stream));
    return TG_OK;
}

static int copy_full(tg_sim *s, float *dst, const float *src, size_t count) {
    if (!src) return fail(TG_ERR_ARG, "null source tensor");
    if (src == dst) return TG_OK;
    if (s->win.first) s->win_dirty = true;   // (a copy inside a timing window)
    HIPCHK(hipMemcpyAsync(dst, src, count * sizeof(float), hipMemcpyDeviceToDevice, s->stream));
    return TG_OK;
}

int tg_set_dof_position_targets(tg_sim *s, const float *pos) {
    if (int rc = check_sim(s)) return rc;
    return copy_full(s, s->pos_tgt, pos, (size_t)s->N * s->D);
}
int tg_set_dof_velocity_targets(tg_sim *s, const float *vel) {
    if (int rc = check_sim(s)) return rc;
    return copy_full(s, s->vel_tgt, vel, (size_t)s->N * s->D);
}
int tg_set_dof_actuation_forces(tg_sim *s, const float *eff) {
    if (int rc = check_sim(s)) return rc;
    return copy_full(s, s->act, eff, (size_t)s->N * s->D);
}

int tg_set_actor_root_state_indexed(tg_sim *s, const float *root, const int32_t *ids, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (!root) return fail(TG_ERR_ARG, "null root state");
    if (root == s->root) return TG_OK;
    win_touch(s);
    if (int rc = tg::launch_scatter_rows(s->root, root, ids, n, 13, s->stream)) return fail(rc, "scatter failed");
    return TG_OK;
}

int tg_set_dof_state_indexed(tg_sim *s, const float *dof, const int32_t *ids, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (!dof) return fail(TG_ERR_ARG, "null dof state");
    if (dof == s->dof) return TG_OK;
    win_touch(s);
    if (int rc = tg::launch_scatter_rows(s->dof, dof, ids, n, 2 * s->D, s->stream)) return fail(rc, "scatter failed");
    return TG_OK;
}

int tg_set_dof_properties_indexed(tg_sim *s, int32_t field, const float *vals, const int32_t *ids, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (field < 0 || field >= TG_NUM_PROPS) return fail(TG_ERR_ARG, "unknown dof property field %d", field);
    if (!vals) return fail(TG_ERR_ARG, "null property values");
    float *dst = s->props + (size_t)field * s->N * s->D;
    win_touch(s);
    if (vals != dst) {   // (writes through the zero-copy props view need no copy)
        if (int rc = tg::launch_scatter_field(dst, vals, ids, n, s->D, s->stream)) return fail(rc, "scatter failed");
    }
    if (int rc = tg::launch_mark_dirty(s->dirty, ids, n, s->stream)) return fail(rc, "mark dirty failed");
    return TG_OK;
}

int tg_set_body_mass_scale_indexed(tg_sim *s, const float *scale, const int32_t *ids, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (!scale) return fail(TG_ERR_ARG, "null mass scale");
    win_touch(s);
    if (int rc = tg::launch_scatter_rows(s->mass_scale, scale, ids, n, s->L, s->stream)) return fail(rc, "scatter failed");
    win_touch(s);
    if (int rc = tg::launch_mark_dirty(s->dirty, ids, n, s->stream)) return fail(rc, "mark dirty failed");
    return TG_OK;
}

int tg_set_shape_friction_indexed(tg_sim *s, const float *mu, const int32_t *ids, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (!mu) return fail(TG_ERR_ARG, "null friction");
    if (s->S == 0) return TG_OK;
    win_touch(s);
    if (int rc = tg::launch_scatter_rows(s->shape_mu, mu, ids, n, s->S, s->stream)) return fail(rc, "scatter failed");
    return TG_OK;
}

int tg_set_gravity(tg_sim *s, const float *g3) {
    if (int rc = check_sim(s)) return rc;
    if (!g3) return fail(TG_ERR_ARG, "null gravity");
    memcpy(s->gravity, g3, sizeof s->gravity);
    return TG_OK;
}

int tg_apply_body_forces(tg_sim *s, const float *wrench) {
    if (int rc = check_sim(s)) return rc;
    if (!wrench) return fail(TG_ERR_ARG, "null wrench tensor");
    if (int rc = copy_full(s, s->force, wrench, (size_t)s->N * s->G * 6)) return rc;
    s->forces_pending = true;
    s->rbf_pending = false;   // the group wrenches given here replace a pending per-link tensor
    s->rbf_prereduced = false;
    return TG_OK;
}

int tg_set_heightfield(tg_sim *s, const float *heights, int32_t rows, int32_t cols, float horizontal_scale,
                       float vertical_scale, float origin_x, float origin_y, float friction) {
    if (int rc = check_sim(s)) return rc;
    if (rows == 0) {
        s->hf_rows = s->hf_cols = 0;
        return TG_OK;
    }
    if (!heights || rows < 2 || cols < 2) return fail(TG_ERR_ARG, "heightfield needs >= 2 x 2 samples");
    if (!(horizontal_scale > 0.f)) return fail(TG_ERR_ARG, "heightfield horizontal_scale must be > 0");
    HIPCHK(hipStreamSynchronize(s->stream));
    if (s->hf) {
        HIPCHK(hipFree(s->hf));
        s->hf = nullptr;
    }
    const size_t bytes = (size_t)rows * cols * sizeof(float);
    HIPCHK(hipMalloc(&s->hf, bytes));
    HIPCHK(hipMemcpy(s->hf, heights, bytes, hipMemcpyHostToDevice));
    s->hf_rows = rows;
    s->hf_cols = cols;
    s->hf_hs = horizontal_scale;
    s->hf_vs = vertical_scale;
    s->hf_ox = origin_x;
    s->hf_oy = origin_y;
    s->hf_mu = friction;
    return TG_OK;
}

// compose (+ optional prologue in a) and the step kernel of one simulate call;
// with wp, the step kernel carrying the walk post-physics epilogue (returns 1,
// nothing launched, when the model has no such instantiation)
// makes the sim's device current for the launches of one call (per-device
// kernel attributes, tg_set_stream's stream), restoring the caller's device
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

static int simulate_args(tg_sim *s, const tg::StepArgs &a_in, const tg::WalkPostArgs *wp = nullptr,
                         const tg::GogoroPostArgs *gp = nullptr, const tg::PaperPostArgs *pp = nullptr) {
    DeviceGuard dg(s->device);
    tg::StepArgs a = a_in;
    // the compose launch: every dirty env (host-side changes possible), the
    // last fused epilogue's reset list, the task prologue alone, or none
    const bool walk_prologue = a.pm_actions && !a.pm_in_step;
    const bool gogoro_prologue = a.gp.actions && !a.gp_in_step;
    // (a pending per-link force tensor with listed envs: the full compose, which
    // reduces it after composing them)
    const bool paper_prologue = a.pp.actions && !a.pp_in_step;   // (one wavefront per env: the full compose launch)
    const bool full = s->dirty_possible || s->always_compose || walk_prologue || paper_prologue ||
                      (s->rbf_pending && s->list_pending);
    a.skip_compose = !full && !s->list_pending && !gogoro_prologue;
    a.compose_list = !full && !a.skip_compose;
    a.cnext = s->ccount + s->list_cur;
    if (a.compose_list && s->list_pending) {
        const int prev = 1 - s->list_cur;
        a.clist = s->clist + (size_t)prev * s->N;
        a.ccount = s->ccount + prev;
    }
    bool rb_launch = false, rb_in_compose = false;
    if (s->rbf_pending) {   // the pending per-link forces: in the full compose launch, else on their own
        if (!a.skip_compose && !a.compose_list) {
            // reduced by the compose launch below: still pending until that
            // launch went through (a fused launcher may decline the call,
            // rc 1, and the caller's fallback simulate must reduce them then)
            rb_in_compose = true;
            a.rbf_forces = s->rbf_f;
            a.rbf_torques = s->rbf_t;
            a.rbf_space = s->rbf_space;
            a.rbf_out = s->force;
        } else {
            rb_launch = true;
            if (int rc = tg::launch_rb_forces(s->hash, s->root, s->dof, s->comp, (int)s->N, s->mass_scale, s->rbf_f,
                                              s->rbf_t, s->rbf_space, s->force, s->props, s->stream))
                return fail(rc, "rigid-body force launch failed");
            s->rbf_pending = false;   // s->force holds the reduced wrenches now
        }
    }
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    const bool timed = s->timing > 0 && s->timing_count % s->timing == 0;
    // windowed timing: this call launches a compose / rigid-body force kernel
    // too (other), or only the step kernel
    const bool windowed = s->timing < 0, other = !a.skip_compose || rb_launch;
    if (windowed && s->win.first && other) s->win_dirty = true;
    if (windowed && !s->win.first && !other) {
        if (!s->ev_free.empty()) {
            s->win = s->ev_free.back();
            s->ev_free.pop_back();
        } else {
            HIPCHK(hipEventCreate(&s->win.first));
            HIPCHK(hipEventCreate(&s->win.second));
        }
        s->win_n = 0;
        s->win_dirty = false;
        HIPCHK(hipEventRecord(s->win.first, s->stream));
    }
    if (timed) {
        if (!s->ev_free.empty()) {
            ev = s->ev_free.back();
            s->ev_free.pop_back();
        } else {
            HIPCHK(hipEventCreate(&ev.first));
            HIPCHK(hipEventCreate(&ev.second));
        }
    }
    int rc = wp   ? tg::launch_step_walk(s->hash, a, *wp, s->stream, ev.first, ev.second)
             : gp ? tg::launch_step_gogoro(s->hash, a, *gp, s->stream, ev.first, ev.second)
             : pp ? tg::launch_step_paper(s->hash, a, *pp, s->stream, ev.first, ev.second)
                  : tg::launch_step(s->hash, a, s->stream, ev.first, ev.second);
    // the pair joins the pending list only once both events were recorded by a
    // launch that went through; otherwise it goes back to the free list
    if (rc != 0) {
        if (ev.first) s->ev_free.push_back(ev);
        if (s->win.first) {   // the open window is dropped
            s->ev_free.push_back(s->win);
            s->win = {nullptr, nullptr};
        }
        if (rc == 1) return 1;   // not launched (no such instantiation): caller falls back
        return fail(rc, "step launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
    if (rb_in_compose) s->rbf_pending = false;
    if (s->timing > 0) s->timing_count++;
    if (ev.first) {
        s->ev_pending.push_back(ev);
        s->ev_launches.push_back(1);
    }
    if (windowed && s->win.first && ++s->win_n == -s->timing) {   // the window closes
        if (!s->win_dirty) {
            HIPCHK(hipEventRecord(s->win.second, s->stream));
            s->ev_pending.push_back(s->win);
            s->ev_launches.push_back(s->win_n);
        } else {
            s->ev_free.push_back(s->win);
        }
        s->win = {nullptr, nullptr};
    }
    s->forces_pending = false;   // apply_rigid_body_force_tensors acts for one simulate call
    s->rbf_prereduced = false;
    if (!a.skip_compose) {   // every dirty env, or every listed one, is composed now
        if (!a.compose_list) s->dirty_possible = false;
        s->list_pending = false;
    }
    if (gp && !gp->tl_inplace) {   // the Gogoro epilogue's resets rewrite properties
        if (gp->reset_list) {       // ... and are listed for the next compose
            s->list_pending = true;
            s->list_cur = 1 - s->list_cur;
        } else {
            s->dirty_possible = true;
        }
    }
    return TG_OK;
}

int tg_get_sim_params(tg_sim *s, tg_sim_params *out) {
    if (int rc = check_sim(s)) return rc;
    if (!out) return fail(TG_ERR_ARG, "tg_get_sim_params: null output");
    *out = s->params;
    memcpy(out->gravity, s->gravity, sizeof s->gravity);
    return TG_OK;
}

int tg_set_sim_params(tg_sim *s, const tg_sim_params *p) {
    if (int rc = check_sim(s)) return rc;
    if (!p) return fail(TG_ERR_ARG, "tg_set_sim_params: null argument");
    if (p->substeps < 0 || !(p->dt > 0.f)) return fail(TG_ERR_ARG, "dt must be positive and substeps >= 0");
    if (p->contact_iterations < 0 || p->velocity_iterations < 0)
        return fail(TG_ERR_ARG, "contact / velocity iterations must be >= 0");
    if (p->solver_type != 0 && p->solver_type != 1)
        return fail(TG_ERR_ARG, "solver_type must be 0 (PGS) or 1 (TGS), got %d", p->solver_type);
    const float spacing = s->params.env_spacing;
    const int32_t per_row = s->params.envs_per_row, fix_base = s->params.fix_base;
    s->params = *p;
    s->params.env_spacing = spacing;   // the env grid is fixed at creation,
    s->params.envs_per_row = per_row;
    s->params.fix_base = fix_base;     // and so is the asset option fix_base_link
    memcpy(s->gravity, p->gravity, sizeof s->gravity);
    return TG_OK;
}

int tg_simulate(tg_sim *s) {
    if (int rc = check_sim(s)) return rc;
    return simulate_args(s, step_args(s));
}

int tg_apply_rigid_body_force_tensors(tg_sim *s, const float *forces, const float *torques, int32_t space) {
    if (int rc = check_sim(s)) return rc;
    if (!forces && !torques) return fail(TG_ERR_ARG, "apply_rigid_body_force_tensors: no force or torque tensor");
    if (space != TG_ENV_SPACE && space != TG_LOCAL_SPACE) return fail(TG_ERR_ARG, "space must be TG_ENV_SPACE or TG_LOCAL_SPACE");
    DeviceGuard dg(s->device);
    const float *f = forces;
    if (!f) {   // torques only: a zero force tensor
        if (!s->zero_link3) {
            if (int rc = s->alloc(&s->zero_link3, (size_t)s->N * s->L * 3)) return fail(rc, "allocation failed");
            HIPCHK(hipMemsetAsync(s->zero_link3, 0, (size_t)s->N * s->L * 3 * 4, s->stream));
        }
        f = s->zero_link3;
    }
    // reduced when the next simulate runs (PhysX applies the forces during
    // simulate, at the state it starts from): inside its compose launch if it
    // has one, else by rb_force_kernel just before the step
    s->rbf_f = f;
    s->rbf_t = torques;
    s->rbf_space = space;
    s->rbf_pending = true;
    s->rbf_prereduced = false;
    s->forces_pending = true;
    return TG_OK;
}

int tg_rigid_body_states(tg_sim *s, float *out) {
    if (int rc = check_sim(s)) return rc;
    if (!out) return fail(TG_ERR_ARG, "tg_rigid_body_states: null output");
    win_touch(s);
    if (int rc = tg::launch_body_states(s->hash, s->root, s->dof, (int)s->N, out, s->stream))
        return fail(rc, "rigid-body state launch failed");
    return TG_OK;
}

int tg_composite(tg_sim *s, float *out, int32_t recompose) {
    if (int rc = check_sim(s)) return rc;
    if (!out) return fail(TG_ERR_ARG, "tg_composite: null output");
    DeviceGuard dg(s->device);
    if (recompose) {
        HIPCHK(hipMemsetAsync(s->dirty, 1, s->N, s->stream));
        tg::StepArgs a = step_args(s);
        a.cnext = s->ccount + s->list_cur;
        win_touch(s);
        if (int rc = tg::launch_compose_only(s->hash, a, s->stream)) return fail(rc, "compose launch failed");
        s->list_pending = false;
        s->dirty_possible = false;
    }
    HIPCHK(hipMemcpyAsync(out, s->comp, (size_t)s->N * s->KC * sizeof(float), hipMemcpyDeviceToDevice, s->stream));
    return TG_OK;
}

int tg_set_kernel_timing(tg_sim *s, int32_t period) {
    if (int rc = check_sim(s)) return rc;
    s->timing = period;
    s->timing_count = 0;
    if (s->win.first) {   // an open window is dropped
        s->ev_free.push_back(s->win);
        s->win = {nullptr, nullptr};
    }
    return TG_OK;
}

int tg_read_kernel_timing(tg_sim *s, double *total_ms, int64_t *launches) {
    if (int rc = check_sim(s)) return rc;
    if (!total_ms || !launches) return fail(TG_ERR_ARG, "tg_read_kernel_timing: null argument");
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pend;
    std::vector<int> cnt;
    pend.swap(s->ev_pending);   // every pair leaves the pending list, read or not
    cnt.swap(s->ev_launches);
    for (auto &e : pend) s->ev_free.push_back(e);
    for (size_t i = 0; i < pend.size(); ++i) {
        HIPCHK(hipEventSynchronize(pend[i].second));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, pend[i].first, pend[i].second));
        s->timed_ms += ms;
        s->timed_launches += cnt[i];
    }
    *total_ms = s->timed_ms;
    *launches = s->timed_launches;
    s->timed_ms = 0.0;
    s->timed_launches = 0;
    return TG_OK;
}

int tg_sync(tg_sim *s) {
    if (int rc = check_sim(s)) return rc;
    HIPCHK(hipStreamSynchronize(s->stream));
    int err = 0;
    HIPCHK(hipMemcpy(&err, s->err, sizeof err, hipMemcpyDeviceToHost));
    if (err) {
        HIPCHK(hipMemset(s->err, 0, sizeof err));
        if (err & 2)
            return fail(TG_ERR_STATE, "tg_paper_step: a workgroup of the one-launch step never became resident "
                                      "(reward term 7's batch sum timed out; set TG_PAPER_TWO_LAUNCH=1)");
        return fail(TG_ERR_STATE,
                    "a locked dof was given a [lower, upper] window wider than %g: locked joints are merged into "
                    "their parent's body in this model and stay rigid at the window centre (build the model "
                    "with that joint free instead)", (double)TG_LOCK_WINDOW_MAX);
    }
    return TG_OK;
}

void tg_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out) {
    const tg::U4 r = tg::philox(tg::U4{ctr[0], ctr[1], ctr[2], ctr[3]}, key[0], key[1]);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

int tg_rng_fill(tg_sim *s, int32_t kind, uint64_t seed, uint64_t counter, float *out, int32_t n) {
    if (int rc = check_sim(s)) return rc;
    if (n < 0 || (n > 0 && !out)) return fail(TG_ERR_ARG, "tg_rng_fill: bad output");
    if (kind < 0 || kind > 2) return fail(TG_ERR_ARG, "tg_rng_fill: unknown kind %d", kind);
    win_touch(s);
    if (int rc = tg::launch_rng_fill(kind, seed, counter, out, n, s->stream)) return fail(rc, "rng launch failed");
    return TG_OK;
}

int tg_debug_fill_lds(tg_sim *s, uint32_t pattern) {
    if (int rc = check_sim(s)) return rc;
    win_touch(s);
    if (int rc = tg::launch_fill_lds(pattern, s->stream)) return fail(rc, "LDS fill launch failed");
    return TG_OK;
}

int tg_gogoro_pre_physics(tg_sim *s, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const float *actions,
                          const float *pre_draws, uint64_t counter) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    if (!p || !b || !actions) return fail(TG_ERR_ARG, "tg_gogoro_pre_physics: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D) return fail(TG_ERR_ARG, "gogoro params do not match the sim");
    win_touch(s);
    if (int rc = tg::launch_gogoro_pre(*p, *b, actions, pre_draws, counter, s->stream)) return fail(rc, "launch failed");
    return TG_OK;
}

int tg_gogoro_step(tg_sim *s, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const float *actions,
                   int32_t n_simulate, const float *pre_draws, const float *reset_draws, const float *obs_draws,
                   const float *speed_draws, const float *yaw_draws, uint64_t counter_pre, uint64_t counter_post) {
    if (int rc = check_sim(s)) return rc;
    if (!p || !b || !actions) return fail(TG_ERR_ARG, "tg_gogoro_step: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D) return fail(TG_ERR_ARG, "gogoro params do not match the sim");
    if (n_simulate < 1) return fail(TG_ERR_ARG, "tg_gogoro_step: n_simulate %d < 1", n_simulate);
    if ((speed_draws == nullptr) != (yaw_draws == nullptr))
        return fail(TG_ERR_ARG, "speed_draws and yaw_draws must both be given or both be NULL");
    for (int i = 0; i < n_simulate; ++i) {
        tg::StepArgs a = step_args(s);
        if (i == 0) {   // pre_physics_step fused into the first compose launch
            tg::GogoroPre &g = a.gp;
            g.actions = actions;
            g.action_history = b->action_history;
            g.curent_command = b->curent_command;
            g.pos_target = b->pos_target;
            g.vel_target = b->vel_target;
            g.steer_offsets = b->steer_offsets;
            g.curent_speed = b->curent_speed;
            g.pre_draws = pre_draws;
            g.clip_actions = p->clip_actions;
            g.max_steering_change = p->max_steering_change;
            g.max_steering = p->max_steering;
            g.noise_mean = p->steering_action_noise[0];
            g.noise_std = p->steering_action_noise[1];
            g.dof_steer = p->dof_steer;
            g.dof_rear = p->dof_rear;
            g.absolute_steer = p->absolute_steer;
            g.k0 = (uint32_t)p->seed;
            g.k1 = (uint32_t)(p->seed >> 32);
            g.c_lo = (uint32_t)counter_pre;
            g.c_hi = (uint32_t)(counter_pre >> 32);
        }
        if (i == n_simulate - 1 && !s->post_unfused) {   // post-physics fused into the last step kernel
            // models whose resets only move translating locks (the seat chain)
            // update their composites in the epilogue; others list their resets
            const bool inplace = tg::model_tl(s->hash) > 0 && !s->no_inplace;
            const tg::GogoroPostArgs gp{*p, *b, (uint32_t)counter_post, (uint32_t)(counter_post >> 32),
                                        inplace ? nullptr : s->clist + (size_t)s->list_cur * s->N,
                                        inplace ? nullptr : s->ccount + s->list_cur, inplace ? 1 : 0,
                                        reset_draws, obs_draws, speed_draws, yaw_draws};
            // one launch: the pre-physics too runs in the step kernel
            a.gp_in_step = (n_simulate == 1 && !s->pre_in_compose) ? 1 : 0;
            const int rc = simulate_args(s, a, nullptr, &gp);
            if (rc == 0) return TG_OK;
            if (rc < 0) return rc;
            a.gp_in_step = 0;   // no fused instantiation: the prologue rides in compose
        }
        if (int rc = simulate_args(s, a)) return rc;
    }
    win_touch(s);
    if (int rc = tg::launch_gogoro_post(*p, *b, reset_draws, obs_draws, speed_draws, yaw_draws, counter_post,
                                        s->stream))
        return fail(rc, "launch failed");
    s->dirty_possible = true;   // the separate post kernel's resets mark envs dirty
    return TG_OK;
}

int tg_gogoro_post_physics(tg_sim *s, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const float *reset_draws,
                           const float *obs_draws, const float *speed_draws, const float *yaw_draws, uint64_t counter) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    if (!p || !b) return fail(TG_ERR_ARG, "tg_gogoro_post_physics: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D) return fail(TG_ERR_ARG, "gogoro params do not match the sim");
    if ((speed_draws == nullptr) != (yaw_draws == nullptr))
        return fail(TG_ERR_ARG, "speed_draws and yaw_draws must both be given or both be NULL");
    win_touch(s);
    if (int rc = tg::launch_gogoro_post(*p, *b, reset_draws, obs_draws, speed_draws, yaw_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

int tg_gogoro_reset_idx(tg_sim *s, const tg_gogoro_params *p, const tg_gogoro_buffers *b, const int32_t *ids,
                        int32_t n, const float *reset_draws, uint64_t counter) {
    if (int rc = check_sim(s)) return rc;
    s->dirty_possible = true;
    if (int rc = check_ids(s, ids, n)) return rc;
    if (!p || !b) return fail(TG_ERR_ARG, "tg_gogoro_reset_idx: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D) return fail(TG_ERR_ARG, "gogoro params do not match the sim");
    win_touch(s);
    if (int rc = tg::launch_gogoro_reset_idx(*p, *b, ids, n, reset_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

static int check_walk(tg_sim *s, const tg_walk_params *p, const tg_walk_buffers *b) {
    if (int rc = check_sim(s)) return rc;
    if (!p || !b) return fail(TG_ERR_ARG, "walk: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D || p->num_groups != s->G)
        return fail(TG_ERR_ARG, "walk params do not match the sim (N %d/%d, D %d/%d, G %d/%d)", p->num_envs, s->N,
                    p->num_dof, s->D, p->num_groups, s->G);
    if (p->num_dof > TG_WALK_MAX_DOF) return fail(TG_ERR_ARG, "walk: num_dof %d > %d", p->num_dof, TG_WALK_MAX_DOF);
    if (p->num_obs != TG_WALK_NUM_OBS_BASE + 3 * p->num_dof) return fail(TG_ERR_ARG, "walk: num_obs mismatch");
    return 0;
}

int tg_walk_pre_physics(tg_sim *s, const tg_walk_params *p, const tg_walk_buffers *b, const float *actions) {
    if (int rc = check_walk(s, p, b)) return rc;
    if (!actions) return fail(TG_ERR_ARG, "walk: null actions");
    win_touch(s);
    if (int rc = tg::launch_walk_pre(*p, *b, actions, s->stream)) return fail(rc, "launch failed");
    return TG_OK;
}

int tg_walk_step(tg_sim *s, const tg_walk_params *p, const tg_walk_buffers *b, const float *actions,
                 int32_t n_simulate, const float *reset_draws, const float *push_draws, uint64_t counter) {
    if (int rc = check_walk(s, p, b)) return rc;
    if (!actions || !b->actions || !b->pos_target) return fail(TG_ERR_ARG, "walk step: null actions / targets");
    if (n_simulate < 1) return fail(TG_ERR_ARG, "walk step: n_simulate %d < 1", n_simulate);
    if (p->num_dof > tg::TG_PM_MAX_DOF) return fail(TG_ERR_ARG, "walk step: num_dof %d > %d", p->num_dof, tg::TG_PM_MAX_DOF);
    if (b->body_force) {   // pre_physics_step: apply_rigid_body_force_tensors(body_force)
        if (int rc = copy_full(s, s->force, b->body_force, (size_t)s->N * s->G * 6)) return rc;
        s->forces_pending = true;
        s->rbf_pending = false;
        s->rbf_prereduced = false;
    }
    if (n_simulate == 1 && !s->walk_unfused && !s->pre_in_compose) {
        // one launch per step: pre-physics (drive targets formed from the
        // actions where pass 2a loads them), physics and post-physics all in
        // the step kernel; the compose launch runs only if an env may be dirty
        tg::StepArgs a = step_args(s);
        a.pm_actions = actions;
        a.pm_act_out = b->actions;
        a.pm_tgt_out = b->pos_target;
        a.pm_scale = p->action_scale;
        a.pm_clip = p->clip_actions;
        for (int d = 0; d < p->num_dof; ++d) a.pm_default[d] = p->default_pos[d];
        a.pm_in_step = 1;
        const tg::WalkPostArgs wp{*p, *b, reset_draws, push_draws, (uint32_t)counter, (uint32_t)(counter >> 32)};
        const int rc = simulate_args(s, a, &wp);
        if (rc <= 0) return rc;
        // rc == 1: no fused instantiation for this model / ground -- the general path below
    }
    for (int i = 0; i < n_simulate; ++i) {
        tg::StepArgs a = step_args(s);
        if (i == 0) {   // pre_physics_step fused into the first compose launch
            a.pm_actions = actions;
            a.pm_act_out = b->actions;
            a.pm_tgt_out = b->pos_target;
            a.pm_scale = p->action_scale;
            a.pm_clip = p->clip_actions;
            for (int d = 0; d < p->num_dof; ++d) a.pm_default[d] = p->default_pos[d];
        }
        if (i == n_simulate - 1 && !s->walk_unfused) {   // post-physics fused into the last step kernel
            const tg::WalkPostArgs wp{*p, *b, reset_draws, push_draws, (uint32_t)counter, (uint32_t)(counter >> 32)};
            const int rc = simulate_args(s, a, &wp);
            if (rc == 0) return TG_OK;
            if (rc < 0) return rc;
        }
        if (int rc = simulate_args(s, a)) return rc;
    }
    win_touch(s);
    if (int rc = tg::launch_walk_post(*p, *b, reset_draws, push_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

int tg_walk_post_physics(tg_sim *s, const tg_walk_params *p, const tg_walk_buffers *b, const float *reset_draws,
                         const float *push_draws, uint64_t counter) {
    if (int rc = check_walk(s, p, b)) return rc;
    win_touch(s);
    if (int rc = tg::launch_walk_post(*p, *b, reset_draws, push_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

int tg_walk_reset_idx(tg_sim *s, const tg_walk_params *p, const tg_walk_buffers *b, const int32_t *ids, int32_t n,
                      const float *reset_draws, uint64_t counter) {
    if (int rc = check_walk(s, p, b)) return rc;
    if (int rc = check_ids(s, ids, n)) return rc;
    win_touch(s);
    if (int rc = tg::launch_walk_reset_idx(*p, *b, ids, n, reset_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

static int check_paper(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b) {
    if (int rc = check_sim(s)) return rc;
    if (!p || !b) return fail(TG_ERR_ARG, "paper: null argument");
    if (p->num_envs != s->N || p->num_dof != s->D || p->num_groups != s->G)
        return fail(TG_ERR_ARG, "paper params do not match the sim (N %d/%d, D %d/%d, G %d/%d)", p->num_envs, s->N,
                    p->num_dof, s->D, p->num_groups, s->G);
    const int dofs[5] = {p->dof_steer, p->dof_rear, p->dof_base_x, p->dof_base_y, p->dof_base_z};
    for (int d : dofs)
        if (d < 0 || d >= p->num_dof) return fail(TG_ERR_ARG, "paper: dof index %d out of range", d);
    if ((int)p->command_delay[1] != TG_PAPER_CMD_HIST)
        return fail(TG_ERR_ARG, "paper: command_delay[1] must be %d", TG_PAPER_CMD_HIST);
    if (!b->scratch || !b->buffer_obs || !b->buffer_obs_noisy || !b->obs_buf)
        return fail(TG_ERR_ARG, "paper: missing history / scratch buffers");
    if (p->push_robot && p->push_interval <= 0) return fail(TG_ERR_ARG, "paper: push_interval must be > 0");
    return 0;
}

int tg_paper_pre_physics(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b, const float *actions,
                         uint64_t counter) {
    (void)counter;
    if (int rc = check_paper(s, p, b)) return rc;
    if (!actions) return fail(TG_ERR_ARG, "paper: null actions");   // (targets / history only: nothing to compose)
    win_touch(s);
    if (int rc = tg::launch_paper_pre(*p, *b, actions, s->stream)) return fail(rc, "launch failed");
    return TG_OK;
}

// tg_paper_step in one launch: the pre-physics, the simulate and the
// post-physics (PaperPost) in the step kernel.  Reward term 7's batch sum is
// exchanged inside the launch, so every workgroup must be resident at once:
// one workgroup per CU at most (TG_PAPER_T7_BLK envs each).  Returns 1 when
// the launch does not apply (model, ground, batch size, residency): the
// caller takes the two-launch path.
static tg::PaperPre paper_pre_args(const tg_paper_params *p, const tg_paper_buffers *b, const float *actions) {
    tg::PaperPre q{};
    q.actions = actions;
    q.command_history = b->command_history;
    q.steer_delay = b->steer_delay;
    q.curent_speed = b->curent_speed;
    q.curent_command = b->curent_command;
    q.pos_target = b->pos_target;
    q.vel_target = b->vel_target;
    q.max_steering = p->max_steering;
    q.use_steer_delay = p->use_steer_delay;
    q.dof_steer = p->dof_steer;
    q.dof_rear = p->dof_rear;
    return q;
}
static int paper_one_launch(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b, const float *actions,
                            uint64_t counter) {
    if (s->paper_two_launch || s->pre_in_compose || s->paper_finish_launch || s->no_inplace || s->hf_rows > 0 ||
        (b->rb_forces && s->paper_rb_launch) || !(tg::model_fused(s->hash) & 4) || tg::model_tl(s->hash) <= 0)
        return 1;
    const int epb = tg::model_epb(s->hash);
    if (epb != TG_PAPER_T7_BLK || s->N % epb != 0) return 1;
    if (s->num_cus == 0) {
        DeviceGuard dg(s->device);
        HIPCHK(hipDeviceGetAttribute(&s->num_cus, hipDeviceAttributeMultiprocessorCount, s->device));
    }
    const int nblk = s->N / epb;
    if (nblk > s->num_cus || nblk > TG_PAPER_T7_THREADS) return 1;
    if (!s->t7cnt) {
        DeviceGuard dg(s->device);
        if (s->alloc(&s->t7cnt, 1)) return TG_ERR_HIP;
        s->t7_total = 0;
    }
    tg::StepArgs a = step_args(s);
    a.pp = paper_pre_args(p, b, actions);
    a.pp_in_step = 1;
    a.pp.buffer_obs = b->buffer_obs;
    a.pp.reset_buf = b->reset_buf;
    a.pp.t7 = reinterpret_cast<double *>(b->scratch);   // (N floats hold N / 16 doubles)
    const bool rb = b->rb_forces != nullptr;
    const tg::PaperPostArgs pa{*p, *b, (uint32_t)counter, (uint32_t)(counter >> 32), rb ? s->force : nullptr,
                               s->t7cnt, s->t7_total + (unsigned)nblk, nblk};
    if (int rc = simulate_args(s, a, nullptr, nullptr, &pa)) return rc < 0 ? rc : 1;
    s->t7_total += (unsigned)nblk;   // (the launch adds nblk arrivals)
    if (rb) {   // the next simulate's rigid-body forces, reduced already
        s->rbf_f = b->rb_forces;
        s->rbf_t = nullptr;
        s->rbf_space = TG_ENV_SPACE;
        s->rbf_pending = false;
        s->rbf_prereduced = true;
        s->forces_pending = true;
    }
    return TG_OK;
}

int tg_paper_step(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b, const float *actions,
                  int32_t n_simulate, uint64_t counter) {
    if (int rc = check_paper(s, p, b)) return rc;
    if (!actions) return fail(TG_ERR_ARG, "paper: null actions");
    if (n_simulate < 1) return fail(TG_ERR_ARG, "tg_paper_step: n_simulate %d < 1", n_simulate);
    if (n_simulate == 1) {
        const int rc = paper_one_launch(s, p, b, actions, counter);
        if (rc != 1) return rc;
    }
    bool fin = false;
    for (int i = 0; i < n_simulate; ++i) {
        tg::StepArgs a = step_args(s);
        if (i == 0) {   // pre_physics_step as the first compose launch's prologue
            tg::PaperPre &q = a.pp;
            q.actions = actions;
            q.command_history = b->command_history;
            q.steer_delay = b->steer_delay;
            q.curent_speed = b->curent_speed;
            q.curent_command = b->curent_command;
            q.pos_target = b->pos_target;
            q.vel_target = b->vel_target;
            q.max_steering = p->max_steering;
            q.use_steer_delay = p->use_steer_delay;
            q.dof_steer = p->dof_steer;
            q.dof_rear = p->dof_rear;
            // in the step kernel itself when it is the only simulate and the
            // model's kernel has the pre-physics slots; else the compose prologue
            q.actions = actions;
            // (FUSED bit 4: the bit the step kernel tests before it runs the
            // paper pre-physics and forms the term-7 partials)
            a.pp_in_step = (n_simulate == 1 && (tg::model_fused(s->hash) & 4) && !s->pre_in_compose) ? 1 : 0;
            // the step kernel also forms reward term 7's partials, so the post
            // launch finishes the batch itself (no finish launch)
            if (a.pp_in_step && !s->paper_finish_launch && p->num_envs % 8 == 0) {   // 8: PAPER_EPW
                q.buffer_obs = b->buffer_obs;
                q.reset_buf = b->reset_buf;
                q.t7 = reinterpret_cast<double *>(b->scratch);   // (N floats hold N / 16 doubles)
                fin = true;
            }
        }
        if (int rc = simulate_args(s, a)) return rc < 0 ? rc : fail(TG_ERR_STATE, "no step kernel for this model");
    }
    bool inplace = false, rb_done = false;
    const bool rb_fuse = b->rb_forces && !s->paper_rb_launch;
    win_touch(s);
    if (int rc = tg::launch_paper_post(*p, *b, nullptr, nullptr, nullptr, nullptr, nullptr, counter, s->stream,
                                       s->hash, s->no_inplace ? nullptr : s->comp, &inplace, fin,
                                       rb_fuse ? s->force : nullptr, &rb_done))
        return fail(rc, "launch failed");
    if (b->rb_forces) {   // the next simulate's rigid-body forces: reduced already, or pending as if applied now
        s->rbf_f = b->rb_forces;
        s->rbf_t = nullptr;
        s->rbf_space = TG_ENV_SPACE;
        s->rbf_pending = !rb_done;
        s->rbf_prereduced = rb_done;
        s->forces_pending = true;
    }
    // the post kernel's resets either update the seat composites in place or
    // mark their envs for the next compose
    if (!inplace) s->dirty_possible = true;
    return TG_OK;
}

int tg_paper_post_physics(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b, const float *reset_draws,
                          const float *noise_draws, const float *speed_draws, const float *yaw_draws,
                          const float *push_draws, uint64_t counter) {
    if (int rc = check_paper(s, p, b)) return rc;
    const bool dirty_before = s->dirty_possible;
    s->dirty_possible = true;
    bool inplace = false;
    win_touch(s);
    if (int rc = tg::launch_paper_post(*p, *b, reset_draws, noise_draws, speed_draws, yaw_draws, push_draws, counter,
                                       s->stream, s->hash, s->no_inplace ? nullptr : s->comp, &inplace))
        return fail(rc, "launch failed");
    if (inplace) s->dirty_possible = dirty_before;
    return TG_OK;
}

int tg_paper_reset_idx(tg_sim *s, const tg_paper_params *p, const tg_paper_buffers *b, const int32_t *ids, int32_t n,
                       const float *reset_draws, uint64_t counter) {
    if (int rc = check_paper(s, p, b)) return rc;
    s->dirty_possible = true;
    if (int rc = check_ids(s, ids, n)) return rc;
    win_touch(s);
    if (int rc = tg::launch_paper_reset_idx(*p, *b, ids, n, reset_draws, counter, s->stream))
        return fail(rc, "launch failed");
    return TG_OK;
}

}  // extern "C"
