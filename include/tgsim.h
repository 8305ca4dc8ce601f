/*
 * tgsim.h -- C-ABI of libtgsim.so, the MI355X-native articulated-body
 * simulator that replaces the IsaacGym/PhysX tensor API as the reference task
 * code uses it.  Plain C types only (device pointers are passed as raw
 * pointers, sizes as ints); no torch or HIP types appear in any signature.
 *
 * Reference interface each entry point replaces (paths relative to
 * /root/reference/isaacgymenvs/):
 *
 *   tg_sim_create            gym.create_sim + load_asset + create_env/actor loop
 *                            + prepare_sim   (tasks/base/vec_task.py:51-57,217;
 *                            tasks/gogoro_new.py:155-162,196-294)
 *   tg_sim_destroy           (process teardown)
 *   tg_state_ptrs            acquire_actor_root_state_tensor /
 *                            acquire_dof_state_tensor + gymtorch.wrap_tensor
 *                            (tasks/gogoro_new.py:125-130)
 *   tg_refresh               refresh_actor_root_state_tensor /
 *                            refresh_dof_state_tensor (gogoro_new.py:141-142,426-427)
 *                            -- the views are the live state, nothing is copied; it
 *                            is REQUIRED after writes through the dof_props /
 *                            env_dirty views (it re-arms the compose launch the
 *                            library otherwise skips while no env can be dirty)
 *   tg_set_dof_position_targets / tg_set_dof_velocity_targets
 *                            set_dof_position_target_tensor /
 *                            set_dof_velocity_target_tensor (gogoro_new.py:364,369)
 *   tg_set_actor_root_state_indexed
 *                            set_actor_root_state_tensor_indexed (gogoro_new.py:547)
 *   tg_set_dof_state_indexed set_dof_state_tensor_indexed (gogoro_new.py:552)
 *   tg_set_dof_properties_indexed
 *                            set_actor_dof_properties per env (gogoro_new.py:294,601)
 *   tg_set_body_mass_scale_indexed / tg_set_gravity
 *                            rigid_body_properties.mass / sim_params.gravity
 *                            domain randomisation (vec_task.py:538-768)
 *   tg_set_shape_friction_indexed
 *                            set_actor_rigid_shape_properties (gogoro_new.py:284-293)
 *   tg_apply_rigid_body_force_tensors
 *                            apply_rigid_body_force_tensors(sim, forces [N*L,3],
 *                            torques [N*L,3] | None, space)
 *                            (tasks/gogoro_realistic_turning_sim_paper.py:457)
 *   tg_apply_body_forces     the same, pre-reduced: one wrench per group [N,G,6]
 *   tg_simulate              gym.simulate (vec_task.py:335): sim.substeps substeps
 *   tg_get_sim_params / tg_set_sim_params
 *                            gym.get_sim_params / set_sim_params (vec_task.py:650-660)
 *   tg_sync                  fetch_results(sim, True) (vec_task.py:339)
 *   tg_last_error            (replaces the reference's bool returns + assert,
 *                            gogoro_new.py:547,552, and quit() on creation
 *                            failure, vec_task.py:291-293)
 *
 * Every call returns 0 on success and a negative code on error; the message
 * is available from tg_last_error() (thread-local).  Calls are asynchronous
 * on the stream given by tg_set_stream(); inputs are caller-owned device
 * pointers read in stream order and never retained.
 */
#ifndef TGSIM_H
#define TGSIM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TG_OK 0
/* joint limits: damping and implicit stiffness ramp in over this distance past
 * the limit (rad or m), keeping the step continuous at the limit */
#define TG_LIMIT_RAMP 0.01f

/* widest [lower, upper] window a locked DOF may carry (the reference locks
 * with 1e-4, tasks/gogoro_new.py:257-262); wider is reported as TG_ERR_STATE */
#define TG_LOCK_WINDOW_MAX 1e-3f

#define TG_ERR_ARG -1
#define TG_ERR_HIP -2
#define TG_ERR_MODEL -3
#define TG_ERR_STATE -4

#define TG_JOINT_FIXED 0
#define TG_JOINT_REVOLUTE 1
#define TG_JOINT_PRISMATIC 2

#define TG_SHAPE_TORUS 0   /* params: R_major, r_minor; torus axis = shape z */
#define TG_SHAPE_BOX 1     /* params: half extents x,y,z                     */
#define TG_SHAPE_SPHERE 2  /* params: radius                                 */

/* DOF drive modes (gymapi.DOF_MODE_*) */
#define TG_DOF_MODE_NONE 0
#define TG_DOF_MODE_POS 1
#define TG_DOF_MODE_VEL 2
#define TG_DOF_MODE_EFFORT 3

/* per-env DOF property fields for tg_set_dof_properties_indexed */
#define TG_PROP_STIFFNESS 0
#define TG_PROP_DAMPING 1
#define TG_PROP_EFFORT 2
#define TG_PROP_VELOCITY 3
#define TG_PROP_LOWER 4
#define TG_PROP_UPPER 5
#define TG_PROP_DRIVE_MODE 6  /* values passed as float, rounded */
#define TG_PROP_ARMATURE 7
#define TG_NUM_PROPS 8

/* Articulation model, links in depth-first order (parents before children).
 * Link frames follow URDF: a link's frame is its incoming joint frame.
 * A "group" is a group-root link plus all descendants reached through fixed
 * or locked joints (locked = position fixed per env between resets, the
 * reference's limit-locked joints, tasks/gogoro_new.py:257-262,562-572). */
typedef struct tg_model_desc {
    int32_t num_links;
    int32_t num_dofs;
    int32_t num_groups;
    int32_t num_shapes;
    const int32_t *link_parent;   /* [L] parent link, -1 for the root       */
    const int32_t *link_group;    /* [L] group of each link                 */
    const int32_t *link_dof;      /* [L] dof of the incoming joint, -1 fixed */
    const int32_t *link_jtype;    /* [L] TG_JOINT_*                          */
    const float *link_origin;     /* [L,12] incoming joint origin in parent link frame: R row-major (9), p (3) */
    const float *link_axis;       /* [L,3] joint axis in the link frame      */
    const float *link_inertia;    /* [L,10] mass, com xyz, ixx iyy izz ixy ixz iyz (about com, link axes) */
    const int32_t *group_root;    /* [G] root link of each group             */
    const int32_t *group_parent;  /* [G] parent group, -1 for the floating root */
    const int32_t *dof_locked;    /* [D] 1 if the dof is locked              */
    const int32_t *shape_link;    /* [S] */
    const int32_t *shape_kind;    /* [S] TG_SHAPE_* */
    const float *shape_pose;      /* [S,12] R row-major, p in the link frame */
    const float *shape_params;    /* [S,4] */
    const float *shape_friction;  /* [S] */
    uint64_t model_hash;          /* selects the compiled kernel specialisation */
} tg_model_desc;

/* sim_params (cfg/task/<Task>.yaml "sim" + "physx" blocks, vec_task.py:442-490) */
typedef struct tg_sim_params {
    float dt;                     /* control dt (sim.dt)                   */
    int32_t substeps;             /* sim.substeps                          */
    float gravity[3];             /* sim.gravity                           */
    float linear_damping;         /* AssetOptions.linear_damping           */
    float angular_damping;        /* AssetOptions.angular_damping          */
    float max_depenetration_velocity; /* physx.max_depenetration_velocity  */
    float rest_offset;            /* physx.rest_offset                     */
    float contact_margin;         /* speculative contact distance          */
    float ground_friction;        /* PlaneParams.static_friction           */
    float baumgarte;              /* penetration push-out factor per substep */
    float limit_stiffness;        /* implicit limit spring, fraction of joint inertia / h^2 */
    float limit_damping;          /* implicit limit damper, fraction of joint inertia / h   */
    int32_t contact_iterations;   /* projected Gauss-Seidel sweeps per substep, with push-out bias
                                     (physx.num_position_iterations) */
    int32_t velocity_iterations;  /* bias-free sweeps after them (physx.num_velocity_iterations):
                                     the positions integrate the velocity of the biased sweeps,
                                     the stored velocity is the bias-free one */
    int32_t fix_base;             /* AssetOptions.fix_base_link            */
    float env_spacing;            /* create_env spacing (env origins grid) */
    int32_t envs_per_row;
    int32_t solver_type;          /* physx.solver_type: 0 PGS, 1 TGS (IsaacGym's default).  TGS runs
                                     the position iterations as sub-steps of h / contact_iterations:
                                     before each sweep a normal row's target is re-formed from its
                                     separation advanced by the row's accumulated displacement, and
                                     the positions integrate the mean of the sweeps' multipliers */
    float contact_offset;         /* physx.contact_offset (IsaacGym default 0.02): PhysX's pair rule --
                                     a shape point carries a (speculative) normal row only while its
                                     separation is below the pair's contact distance, the shape's plus
                                     the ground plane's offset, 2 x contact_offset (round 6; round 5
                                     used one offset plus the point's free approach); <= 0: every
                                     point speculative (the rounds 1-4 behaviour) */
} tg_sim_params;

/* zero-copy device views (gymtorch.wrap_tensor equivalents) */
typedef struct tg_state_view {
    float *root_state;            /* [N,13] pos(3) quat xyzw(4) linvel(3) angvel(3), world frame */
    float *dof_state;             /* [N*D,2] pos, vel */
    float *dof_pos_target;        /* [N,D] */
    float *dof_vel_target;        /* [N,D] */
    float *dof_actuation;         /* [N,D] effort-mode forces */
    float *dof_props;             /* [TG_NUM_PROPS,N,D] */
    float *body_force;            /* [N,G,6] external wrench per group, world frame (force, torque at group COM) */
    float *env_origin;            /* [N,3] */
    uint8_t *env_dirty;           /* [N] */
    int32_t num_envs, num_dofs, num_groups, num_links;
} tg_state_view;

typedef struct tg_sim tg_sim;

int tg_sim_create(const tg_model_desc *model, const tg_sim_params *params, int32_t num_envs, int32_t device,
                  tg_sim **out);
int tg_sim_destroy(tg_sim *sim);
int tg_set_stream(tg_sim *sim, void *hip_stream);
int tg_state_ptrs(tg_sim *sim, tg_state_view *view);
/* Adopt caller-owned device buffers (e.g. torch tensors) for any non-NULL
 * pointer of `view` (sizes as in tg_state_view); the sim's current contents
 * are copied into them first, so the caller's tensors become the live,
 * zero-copy state (the gymtorch.wrap_tensor contract).  Caller keeps them alive. */
int tg_bind_state(tg_sim *sim, const tg_state_view *view);
int tg_refresh(tg_sim *sim);
int tg_set_dof_position_targets(tg_sim *sim, const float *pos);
int tg_set_dof_velocity_targets(tg_sim *sim, const float *vel);
int tg_set_dof_actuation_forces(tg_sim *sim, const float *effort);
int tg_set_actor_root_state_indexed(tg_sim *sim, const float *root, const int32_t *ids, int32_t n);
int tg_set_dof_state_indexed(tg_sim *sim, const float *dof, const int32_t *ids, int32_t n);
int tg_set_dof_properties_indexed(tg_sim *sim, int32_t field, const float *vals, const int32_t *ids, int32_t n);
int tg_set_body_mass_scale_indexed(tg_sim *sim, const float *scale, const int32_t *ids, int32_t n);
int tg_set_shape_friction_indexed(tg_sim *sim, const float *mu, const int32_t *ids, int32_t n);
int tg_set_gravity(tg_sim *sim, const float *g3);
int tg_apply_body_forces(tg_sim *sim, const float *wrench);
/* apply_rigid_body_force_tensors (gymapi; tasks/gogoro_realistic_turning_sim_paper.py:457):
 * forces [N*L,3] acting at each rigid body's centre of mass and torques
 * [N*L,3], either may be NULL (the reference passes torqueTensor=None), in the
 * world frame (TG_ENV_SPACE, isaacgym's default; envs are translated, not
 * rotated) or each body's own frame (TG_LOCAL_SPACE).  Bodies in model.links
 * order (the order of get_actor_rigid_body_dict).  They act for the next
 * tg_simulate call, as PhysX's applied forces do for one simulate: that call
 * reduces them, from the state it starts from, to the group wrenches
 * tg_apply_body_forces takes (world force, torque about the group centre of
 * mass) -- so, unlike the other inputs, the tensors are read by the next
 * tg_simulate and must stay valid until it has been issued. */
#define TG_ENV_SPACE 0
#define TG_LOCAL_SPACE 1
int tg_apply_rigid_body_force_tensors(tg_sim *sim, const float *forces, const float *torques, int32_t space);
/* Terrain ground (gym.add_triangle_mesh of the heightfield trimesh,
 * tasks/gogoro_new.py:164-181 with terrain_utils.convert_heightfield_to_trimesh):
 * heights [rows, cols] row-major on the HOST, vertex (i, j) at
 * (origin_x + i*horizontal_scale, origin_y + j*horizontal_scale,
 * heights[i][j]*vertical_scale), each cell split into the triangles
 * (i,j)-(i+1,j+1)-(i,j+1) and (i,j)-(i+1,j)-(i+1,j+1); friction = the mesh's
 * static/dynamic friction (combined with the shape's by averaging, like the
 * plane's).  The z = 0 plane stays (gogoro_new.py:157-159 adds both): the
 * ground is whichever surface is higher, and the plane outside the grid.
 * rows = 0 removes the terrain. */
int tg_set_heightfield(tg_sim *sim, const float *heights, int32_t rows, int32_t cols, float horizontal_scale,
                       float vertical_scale, float origin_x, float origin_y, float friction);
int tg_simulate(tg_sim *sim);
/* gym.get_sim_params / gym.set_sim_params (vec_task.py:243,650-660; the
 * reference reads the params back, edits them and writes them again for its
 * gravity randomisation).  set takes effect at the next tg_simulate; the env
 * grid (env_spacing, envs_per_row) and the asset option fix_base are fixed at
 * creation and ignored here.  solver_type must be 0 (PGS) or 1 (TGS), here
 * and in tg_sim_create (TG_ERR_ARG otherwise).
 * substeps may be 0 in set: simulate then integrates nothing and a step
 * passes the state through unchanged -- the parity tests use it to replay
 * the reference's recorded post-simulate states through the fused step. */
int tg_get_sim_params(tg_sim *sim, tg_sim_params *out);
int tg_set_sim_params(tg_sim *sim, const tg_sim_params *params);
/* refresh_rigid_body_state_tensor on the tensor from acquire_rigid_body_state_tensor
 * (IsaacGym tensor API; SURVEY §8b lists it on the boundary, the reference
 * tasks do not read it): out [N, L, 13] device, caller-owned, links in model
 * order (model.links): world origin position (3), orientation quat xyzw (4),
 * linear velocity of the link's centre of mass (3, the root-state convention),
 * angular velocity (3); from the current root and dof state, stream-ordered. */
int tg_rigid_body_states(tg_sim *sim, float *out);
/* fetch_results(sim, True): waits for the sim stream.  Also reports (once, as
 * TG_ERR_STATE) a state error a kernel raised since the last call: a locked
 * DOF whose [lower, upper] window was widened beyond TG_LOCK_WINDOW_MAX. */
int tg_sync(tg_sim *sim);
const char *tg_last_error(void);
uint64_t tg_compiled_model_hashes(uint64_t *out, int32_t cap); /* returns count */
/* gym.load_asset of a model that is not compiled in (gogoro_new.py:198-213
 * loads its URDF at run time): compile the articulation kernels for it with
 * hipRTC (gfx950) and register them under model_hash, after which
 * tg_sim_create accepts a tg_model_desc with that hash.  model_source is the
 * model's constexpr table text as thormang_isaacgym_amd/model/codegen.py emits
 * it (one `struct <struct_name> {...}`; the Python host parses the URDF and
 * produces both it and the tg_model_desc).  include_dir: the kernel headers
 * (NULL: the csrc/ directory beside libtgsim.so); cache_dir: where code objects
 * are cached by hash and source digest (NULL: no cache).  A no-op for a
 * compiled-in hash or one already registered in this process. */
int tg_model_jit(uint64_t model_hash, const char *struct_name, const char *model_source, const char *include_dir,
                 const char *cache_dir);

/* gym.load_asset of a URDF without a Python host (gogoro_new.py:198-213, the
 * locked joints of :257-262): csrc/model_load.cpp parses the file (links
 * depth-first from the root, children in joint-declaration order, DOFs = the
 * non-fixed joints in that order, fixed and `locked_joints` merged into rigid
 * groups, collision boxes / spheres, a mesh collision as the torus fitted to
 * its OBJ profile when `mesh_root` names the mesh directory) and builds the
 * tg_model_desc and the specialisation's constexpr source exactly as the
 * Python host (model/urdf.py, abi.model_arrays, model/codegen.py) does.
 * tg_model_parse stops there (no device needed); tg_model_load then runs
 * tg_model_jit for it (a no-op for a compiled-in model).  `name`: the model
 * name (NULL: the file's stem).  The desc arrays live in the tg_model until
 * tg_model_free; errors: tg_model_last_error(). */
typedef struct tg_model tg_model;
int tg_model_parse(const char *urdf_path, const char *name, const char *const *locked_joints, int32_t num_locked,
                   const char *mesh_root, tg_model **out);
int tg_model_load(const char *urdf_path, const char *name, const char *const *locked_joints, int32_t num_locked,
                  const char *mesh_root, const char *cache_dir, tg_model **out);
int tg_model_get_desc(const tg_model *model, tg_model_desc *desc);   /* pointers into the model */
const char *tg_model_dof_name(const tg_model *model, int32_t dof);   /* gym.get_asset_dof_names order */
const char *tg_model_link_name(const tg_model *model, int32_t link); /* gym.get_asset_rigid_body_names */
/* gym.get_asset_dof_properties' URDF part (lower, upper, effort, velocity;
 * +-3.4e38 for an unlimited joint) */
int tg_model_dof_limits(const tg_model *model, int32_t dof, float *lower, float *upper, float *effort,
                        float *velocity);
const char *tg_model_source(const tg_model *model);   /* the constexpr traits text (codegen.emit) */
const char *tg_model_last_error(void);
void tg_model_free(tg_model *model);

/* Composite-cache instrumentation (no reference counterpart; tests): copies
 * the per-env composite cache [N, KC] (the group composites and placements
 * the step kernel reads, built from the lock windows and mass scales) to the
 * device buffer out; with recompose != 0 every env is first re-composed from
 * scratch.  Checks the Gogoro epilogue's in-place seat update against a full
 * compose. */
int tg_composite(tg_sim *sim, float *out, int32_t recompose);

/* Random-number instrumentation (no reference counterpart; the task kernels'
 * in-kernel draws replace the reference's torch.rand / torch.randn calls):
 * tg_philox4x32_10 is the library's Philox4x32-10 block function on the host
 * (ctr[4], key[2] -> out[4]; the same code the kernels run), checked against
 * Random123's published known-answer vectors.  tg_rng_fill runs it on the
 * device for blocks i = 0..n-1 with counter (i, counter lo, counter hi, 0) and
 * key = seed: kind 0 writes the 4 raw 32-bit words per block (out holds 4n
 * words), kind 1 the 4 uniforms u01(word) in [0, 1), kind 2 the 2 normals
 * gauss(w0, w1), gauss(w2, w3) per block (out holds 2n floats). */
void tg_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out);
int tg_rng_fill(tg_sim *sim, int32_t kind, uint64_t seed, uint64_t counter, float *out, int32_t n);

/* Debug instrumentation (no reference counterpart): fills the LDS of every CU
 * with a 32-bit pattern (a NaN, say) through a dummy launch on the sim's
 * stream.  LDS is not cleared between kernels, so a later step that read LDS
 * it had not written would see the pattern: the stale-LDS tests step two
 * identical envs, one with a fill before every step, and require bit-identical
 * results. */
int tg_debug_fill_lds(tg_sim *sim, uint32_t pattern);

/* Benchmark instrumentation (no reference counterpart): with period > 0,
 * tg_simulate brackets every period-th articulation step kernel launch with HIP
 * events on the sim stream (an event pair serialises the queue for ~5 us each
 * side, so sampling keeps the instrumented run's throughput honest); with
 * period = -W < 0 it brackets windows of W consecutive step-kernel launches
 * with one pair (no event between the kernels it times; a window another
 * launch of the library falls into is dropped); 0 turns timing off.
 * tg_read_kernel_timing waits for the recorded launches and returns (and
 * resets) the summed kernel time and the timed launch count. */
int tg_set_kernel_timing(tg_sim *sim, int32_t period);
int tg_read_kernel_timing(tg_sim *sim, double *total_ms, int64_t *launches);

#ifdef __cplusplus
}
#endif
#endif
