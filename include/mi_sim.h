/*
 * mi_sim.h — C ABI of libmi_sim.so, the MI355X-native replacement for the closed
 * PhysX GPU articulation pipeline + the task-layer TorchScript kernels that sit behind
 * OmniIsaacGymEnvs' VecEnvBase / RLTask for the Humanoid, Ant and Cartpole tasks.
 *
 * Every entry point replaces one call site of the reference (file:line under
 * tzmhuang/OmniIsaacGymEnvs v1.1.0, omniisaacgymenvs/...). The reference binds these from
 * Python; the binding a maintainer would add is the ctypes stub in INTEGRATION.md
 * (our own binding: omniisaacgymenvs_amd/native.py).
 *
 * Conventions
 *  - Return 0 (MI_OK) on success, a negative MI_E_* code on failure; the message is in
 *    mi_last_error() (thread-local). No C++ exception crosses this ABI.
 *  - Ownership: an mi_sim owns ALL physics state (struct-of-arrays in device memory).
 *    Every other buffer is caller-owned (PyTorch tensors); the library never frees or
 *    retains them past the call.
 *  - Pointers: tensor arguments are DEVICE pointers on the sim's device, row-major
 *    [N, ...] exactly like the reference's torch buffers. `model`, `params`, `env_origins`,
 *    `dof_limits` and task parameter structs are HOST pointers.
 *  - Dtypes are those of the reference buffers: f32 state/obs/reward, int64 reset_buf /
 *    progress_buf / reset indices, int32 effort indices.
 *  - Streams: `stream` is a hipStream_t passed as void* (torch's current stream); every
 *    call is stream-ordered and none blocks the host except create/destroy/info.
 *  - A handle is not re-entrant: one host thread at a time.
 */
#ifndef MI_SIM_H
#define MI_SIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_ABI_VERSION 4

enum {
    MI_OK = 0,
    MI_E_NULL = -1,    /* null pointer where a buffer is required            */
    MI_E_SHAPE = -2,   /* size / count out of range                          */
    MI_E_HIP = -3,     /* HIP runtime error                                  */
    MI_E_MODEL = -4,   /* model description rejected                         */
    MI_E_ARG = -5,     /* bad enum / parameter value                         */
    MI_E_NODEV = -6,   /* no GPU / bad device id                             */
    MI_E_STATE = -7    /* call out of order (e.g. task not configured)       */
};

/* Task kinds: which fused task kernels run on top of the physics. */
enum { MI_TASK_CARTPOLE = 0, MI_TASK_ANT = 1, MI_TASK_HUMANOID = 2 };

/* Dynamics kinds. */
enum {
    MI_DYN_ARTICULATION = 0, /* floating/fixed-base tree, CRBA + tree-LTDL + PGS contacts  */
    MI_DYN_CARTPOLE = 1      /* analytic 2-DOF cart-pole (prismatic cart + hinge pole)      */
};

enum { MI_JOINT_HINGE = 0, MI_JOINT_SLIDE = 1 };
enum { MI_GEOM_SPHERE = 0, MI_GEOM_CAPSULE = 1 };

/*
 * Compiled model description (host arrays). Produced from an MJCF-subset file by
 * omniisaacgymenvs_amd/robots/model.py; replaces the USD articulation the reference
 * pulls from Nucleus (robots/articulations/humanoid.py:57, ant.py:57, cartpole.py:56).
 *
 * Links: link 0 is the root. For a floating root (root_free=1) its 6 DOFs are the root
 * linear (x,y,z, world) and angular (x,y,z, world) velocities; they are NOT part of the
 * joint DOF vector the task sees. Links 1..L-1 each carry exactly ONE joint DOF
 * (multi-DOF MJCF bodies are chains of massless 1-DOF links) in BFS order, and
 * parent[l] < l. Joint DOF j belongs to link j+1.
 */
typedef struct mi_model_desc {
    int32_t dyn_kind;        /* MI_DYN_*                                             */
    int32_t root_free;       /* 1: floating base (free joint), 0: fixed base         */
    int32_t num_links;       /* L, incl. root link 0                                 */
    int32_t num_geoms;       /* G contact geoms                                      */
    int32_t num_sensors;     /* S force sensors                                      */
    int32_t num_pairs;       /* self-collision geom pairs (may be 0)                 */
    const int32_t* parent;   /* [L]   parent link (-1 for root)                      */
    const int32_t* jtype;    /* [L]   MI_JOINT_* (ignored for link 0)                */
    const float* axis;       /* [L,3] joint axis in the link's joint frame (unit)    */
    const float* pos;        /* [L,3] joint-frame origin in the parent link frame    */
    const float* quat;       /* [L,4] joint-frame rotation wrt parent frame (wxyz)   */
    const float* mass;       /* [L]                                                  */
    const float* com;        /* [L,3] centre of mass in link frame                   */
    const float* inertia;    /* [L,6] about com, link frame: xx yy zz xy xz yz       */
    const float* lower;      /* [L]   joint limits (rad or m); lower>=upper: unlimited */
    const float* upper;      /* [L]                                                  */
    const float* damping;    /* [L]   joint viscous damping (implicit)               */
    const float* armature;   /* [L]   joint armature (added to M diagonal)           */
    const int32_t* geom_link;/* [G]                                                  */
    const int32_t* geom_type;/* [G]   MI_GEOM_*                                      */
    const float* geom_p0;    /* [G,3] sphere centre / capsule end 0, link frame      */
    const float* geom_p1;    /* [G,3] capsule end 1 (ignored for spheres)            */
    const float* geom_radius;/* [G]                                                  */
    const int32_t* sensor_link; /* [S] force sensor body                              */
    const float* sensor_pos; /* [S,3] sensor site in link frame (wrench reference)   */
    const int32_t* pairs;    /* [P,2] self-collision geom pairs                      */
    /* analytic cart-pole parameters (dyn_kind == MI_DYN_CARTPOLE)                   */
    float cart_mass, pole_mass, pole_com, pole_inertia, cart_damping, pole_damping;
} mi_model_desc;

/* Scene / solver parameters — the task YAML `sim:` + `physx:` surface
 * (cfg/task/Humanoid.yaml:34-63, utils/config_utils/default_scene_params.py:30-112). */
typedef struct mi_sim_params {
    float dt;                       /* sim.dt                                         */
    float gravity[3];               /* sim.gravity                                    */
    int32_t solver_iterations;      /* PGS: position + velocity iteration counts;     */
                                    /* TGS: solver_position_iteration_count          */
    float contact_offset;           /* physx.contact_offset                           */
    float rest_offset;              /* physx.rest_offset                              */
    float friction;                 /* default_physics_material.dynamic_friction      */
    float max_depenetration_velocity;
    float erp;                      /* position-error reduction per substep (0..1)    */
    int32_t enable_self_collisions; /* <Actor>.enable_self_collisions                 */
    float max_angular_velocity;     /* rad/s, PhysX default 5729.58 deg/s             */
    float angular_damping;          /* 1/s, per-link angular velocity damping, PhysX  */
                                    /* default 0.05 (docs/transfering_policies_...:74) */
    int32_t solver_type;            /* physx.solver_type (cfg/config.yaml:31): 0 PGS, */
                                    /* 1 TGS (MI_SOLVER_*); anything else is refused  */
    int32_t velocity_iterations;    /* TGS: solver_velocity_iteration_count (PGS: 0)  */
} mi_sim_params;

/* Contact / limit solvers. Both build the same constraint rows from the same
 * state, with the rows' separation d (contact gap - rest_offset, or the joint's distance inside
 * its limit).
 *   MI_SOLVER_PGS: solver_iterations velocity-level Gauss-Seidel sweeps over the whole substep,
 *     bias b = d >= 0 ? -d / dt : -erp d / dt (capped at max_depenetration_velocity); positions
 *     integrated with the final velocity.
 *   MI_SOLVER_TGS (PhysX's default, solver_type 1): solver_iterations position iterations, each a
 *     sub-step h = dt / solver_iterations: one sweep with the bias of the row's CURRENT separation
 *     d + J (sum of h u over the earlier sub-steps) over h; then velocity_iterations sweeps with
 *     the speculative bias only (no position correction). Positions advance by the sub-steps'
 *     velocities (dt x their mean), the velocity state is the last sweep's. */
#define MI_SOLVER_PGS 0
#define MI_SOLVER_TGS 1

/* Task-layer parameters (cfg/task/{Humanoid,Ant,Cartpole}.yaml `env:` + task
 * constants from tasks/shared/locomotion.py:147-171, tasks/humanoid.py:81-112,
 * tasks/ant.py:79-86, tasks/cartpole.py:54-62). */
typedef struct mi_task_params {
    int32_t task_kind;              /* MI_TASK_*                                      */
    int32_t num_obs;                /* O                                              */
    int32_t num_actions;            /* A                                              */
    float clip_actions, clip_obs;   /* env.clipActions / env.clipObservations (inf)   */
    float max_episode_length;       /* env.episodeLength (cartpole: 500)              */
    /* locomotion */
    float power_scale, heading_weight, up_weight, actions_cost, energy_cost;
    float dof_vel_scale, angular_velocity_scale, contact_force_scale;
    float joints_at_limit_cost, death_cost, termination_height, alive_reward_scale;
    float task_dt;                  /* locomotion.py:163, 1/60                         */
    float target[3];                /* locomotion.py:161, (1000,0,0)                   */
    float init_root_pos[3];         /* spawn translation, env frame                   */
    float init_root_quat[4];        /* wxyz                                           */
    float dof_pos_noise, dof_vel_noise; /* locomotion.py:120,124: 0.2, 0.1            */
    const float* joint_gears;       /* [A] host                                       */
    const float* motor_effort_ratio;/* [A] host                                       */
    const float* init_dof_pos;      /* [D] host                                       */
    /* cartpole */
    float reset_dist, max_push_effort;
} mi_task_params;

/* Constraint-row budget per env-substep (every path, and the oracle): ground contact and joint-
 * limit rows always fit (3 * candidate points + D <= MI_MAX_ROWS is required); self-contacts
 * take what is left, (MI_MAX_ROWS - 3 * ground_contacts - limited_joints) / 3 of them, in pair
 * order. */
#define MI_MAX_ROWS 128

typedef struct mi_sim mi_sim;

/* --- lifecycle: replaces World/SimulationContext + GridCloner + ArticulationView init
 *     (tasks/base/rl_task.py:109-131, utils/task_util.py:70) ---------------------------- */
int mi_sim_create(const mi_model_desc* model, const mi_sim_params* params, int32_t num_envs,
                  int64_t env_id_offset, int32_t device_id, const float* env_origins /*[N,3]*/,
                  uint64_t seed, mi_sim** out);
/* Issues any deferred substeps, waits for the device, frees everything. */
int mi_sim_destroy(mi_sim* sim);
/* ArticulationView.num_dof / count / get_dof_limits (humanoid.py:110, ant.py:81) */
int mi_sim_info(const mi_sim* sim, int32_t* num_envs, int32_t* num_dof, int32_t* num_links,
                int32_t* num_sensors, float* dof_limits /*[D,2] host or NULL*/);

/* --- ArticulationView tensor API (call sites locomotion.py:81-89,114,130-134) -------- */
int mi_get_root_state(mi_sim* sim, float* pos /*[N,3]*/, float* quat /*[N,4] wxyz*/,
                      float* vel /*[N,6] lin,ang*/, void* stream);
int mi_get_dof_state(mi_sim* sim, float* q /*[N,D]*/, float* qd /*[N,D]*/, void* stream);
int mi_get_sensor_wrench(mi_sim* sim, float* out /*[N,S,6]*/, void* stream);
int mi_set_dof_efforts(mi_sim* sim, const float* eff /*[n,D]*/, const int32_t* idx /*[n]|NULL*/,
                       int32_t n, void* stream);
int mi_set_dof_state(mi_sim* sim, const float* q /*[n,D]|NULL*/, const float* qd /*[n,D]|NULL*/,
                     const int64_t* idx /*[n]|NULL*/, int32_t n, void* stream);
int mi_set_root_state(mi_sim* sim, const float* pos /*[n,3]|NULL*/, const float* quat /*[n,4]|NULL*/,
                      const float* vel /*[n,6]|NULL*/, const int64_t* idx /*[n]|NULL*/, int32_t n,
                      void* stream);
/* The same two setters with int32 env ids: the Cartpole task's reset passes int32 indices
 * (tasks/cartpole.py:129-130, set_joint_positions / set_joint_velocities), so the view forwards
 * them without an int64 conversion launch per call. */
int mi_set_dof_state_i32(mi_sim* sim, const float* q /*[n,D]|NULL*/, const float* qd /*[n,D]|NULL*/,
                         const int32_t* idx /*[n]|NULL*/, int32_t n, void* stream);
int mi_set_root_state_i32(mi_sim* sim, const float* pos /*[n,3]|NULL*/, const float* quat /*[n,4]|NULL*/,
                          const float* vel /*[n,6]|NULL*/, const int32_t* idx /*[n]|NULL*/, int32_t n,
                          void* stream);
/* State mirrors: row-major copies of the articulation state in caller-owned device buffers, the
 * tensors ArticulationView getters hand out with clone=False (get_world_poses, get_velocities,
 * get_joint_positions / velocities, _physics_view.get_force_sensor_forces: locomotion.py:81-89;
 * Isaac returns views of its own buffers there too). Register all six (or all NULL to stop);
 * mi_get_state_mirror issues any deferred substeps and refreshes every stale mirror in ONE launch
 * (none when nothing wrote the state since the last refresh), so the five getter calls of one
 * get_observations cost at most one gather launch. Every entry point that writes the state marks
 * the mirrors stale; mi_set_dof_efforts does not (efforts are not mirrored). A call on another
 * stream than the last refresh's waits for that refresh (stream-ordered, no host sync).
 * Contract: the mirrors are the library's copies — a caller must not write them (an in-place
 * edit would persist into later getters until the state changes; the reference's task code only
 * reads them, locomotion.py:81-89). */
int mi_sim_set_mirror(mi_sim* sim, float* pos /*[N,3]*/, float* quat /*[N,4]*/, float* vel /*[N,6]*/,
                      float* q /*[N,D]*/, float* qd /*[N,D]*/, float* sens /*[N,S,6]*/);
int mi_get_state_mirror(mi_sim* sim, void* stream);

/* --- physics step: World.step x controlFrequencyInv (envs/vec_env_rlgames.py:64-66) --- */
/* Substeps are deferred and coalesced: consecutive mi_sim_step calls on one stream with no
 * other call touching the state in between (the reference's controlFrequencyInv x World.step
 * loop) run as ONE launch, issued by the next entry point that reads or writes the state (or by
 * mi_sim_flush); results are identical to separate launches. Inside a stream capture, and with
 * the environment variable MI_SIM_DEFER=0, every call launches at once. substeps in [0, 64];
 * one launch never carries more than 64 (a call that would pass 64 issues the pending ones first). */
int mi_sim_step(mi_sim* sim, int32_t substeps, void* stream);
/* Issue any deferred substeps now (stream-ordered; no host sync). */
int mi_sim_flush(mi_sim* sim, void* stream);

/* --- fused task kernels ---------------------------------------------------------------- */
int mi_task_configure(mi_sim* sim, const mi_task_params* tp);
/* LocomotionTask.pre_physics_step / CartpoleTask.pre_physics_step
 * (locomotion.py:103-145, cartpole.py:101-134): mask-driven reset_idx for every env with
 * reset_buf != 0 (no host sync), actions_out = actions, efforts = actions*gear*power. */
int mi_task_pre_step(mi_sim* sim, const float* actions /*[N,A]*/, int64_t* reset_buf,
                     int64_t* progress_buf, float* potentials, float* prev_potentials,
                     float* actions_out /*[N,A]|NULL*/, void* stream);
/* reset_idx(env_ids) with explicit indices (locomotion.py:116-145, cartpole.py:114-134) */
int mi_task_reset_idx(mi_sim* sim, const int64_t* env_ids, int32_t n, int64_t* reset_buf,
                      int64_t* progress_buf, float* potentials, float* prev_potentials,
                      void* stream);
/* RLTask.post_physics_step (rl_task.py:231-251): progress += 1, get_observations,
 * calculate_metrics, is_done — one kernel (locomotion.py:80-101,173-321,
 * humanoid.py:116-127, ant.py:88-95, cartpole.py:80-99,143-162). */
int mi_task_post_step(mi_sim* sim, const float* actions /*[N,A]*/, float* obs /*[N,O]*/,
                      float* rew /*[N]*/, int64_t* reset_buf, int64_t* progress_buf,
                      float* potentials, float* prev_potentials, void* stream);
/* Which kernel the last mi_task_post_step launched and its grid (diagnostics, no reference
 * counterpart): 0..3 k_loco_post_tiled 64s/64d/32s/32d, 4 k_loco_post_pipe (32-env tiles),
 * 5 k_post_step (one lane per env), 6 k_loco_post_pipe with 16-env tiles; -1 before the first
 * launch. */
int mi_task_post_kernel(const mi_sim* sim, int32_t* kernel, int32_t* grid);
/* The three task methods RLTask.post_physics_step calls, as separate kernels
 * (rl_task.py:244-250) for tasks that override some of them in torch:
 * get_observations (locomotion.py:80-101 / cartpole.py:80-99) writes obs + potentials,
 * calculate_metrics (locomotion.py:173-178 / cartpole.py:143-153) reads obs,
 * is_done (locomotion.py:180-183 / cartpole.py:155-162) reads obs[:,0] and progress_buf. */
int mi_task_observations(mi_sim* sim, const float* actions /*[N,A]*/, float* obs /*[N,O]*/,
                         float* potentials, float* prev_potentials, void* stream);
int mi_task_metrics(mi_sim* sim, const float* actions, const float* obs, float* rew,
                    const float* potentials, const float* prev_potentials, void* stream);
int mi_task_is_done(mi_sim* sim, const float* obs, int64_t* reset_buf, const int64_t* progress_buf,
                    void* stream);
/* VecEnvRLGames.step (vec_env_rlgames.py:56-78) minus the Python: clamp actions,
 * pre_physics_step, `substeps` physics steps, post_physics_step and _process_data's obs
 * clamp, in ONE kernel launch. obs_task (unclamped task.obs_buf) may be NULL. */
int mi_env_step(mi_sim* sim, const float* actions /*[N,A]*/, int32_t substeps,
                float* obs_out /*[N,O] clamped*/, float* obs_task /*[N,O]|NULL*/,
                float* rew /*[N]*/, int64_t* reset_buf, int64_t* progress_buf,
                float* potentials, float* prev_potentials, float* actions_out /*[N,A]|NULL*/,
                float* rew_out /*[N]|NULL*/, int64_t* reset_out /*[N]|NULL*/, void* stream);
/* rew_out / reset_out: the fresh copies VecEnvRLGames._process_data returns
 * (vec_env_rlgames.py:41-46), written by the same launch instead of two clone kernels. */
/* Launch timing (measurement only, no reference counterpart; bench.py's roofline): from now on
 * every `every`-th mi_env_step / mi_task_post_step launch (up to `capacity` of them) carries a HIP start / stop event
 * pair on its own dispatch (hipExtLaunchKernelGGL), so the recorded interval is the kernel alone
 * and no marker packets are queued between launches. every <= 0 turns it off. Launches made while
 * the stream captures a graph are not timed. */
int mi_sim_time_launches(mi_sim* sim, int32_t every, int32_t capacity);
/* Durations (ms) of the launches timed since mi_sim_time_launches, in launch order: waits for
 * each one's stop event, writes min(recorded, max_out) values, *n_out = number recorded. */
int mi_sim_launch_times(mi_sim* sim, float* ms_out, int32_t max_out, int32_t* n_out);

/* --- observation / action noise DR (utils/domain_randomization/randomize.py:176-306) ------
 * The `domain_randomization.randomization_params.{observations,actions}` block of a task YAML.
 * Noise math and per-env schedule state: include/mi_dr.h. */
enum { MI_DR_OP_ADDITIVE = 0, MI_DR_OP_SCALING = 1 };
enum { MI_DR_DIST_GAUSSIAN = 0, MI_DR_DIST_UNIFORM = 1, MI_DR_DIST_LOGUNIFORM = 2 };
typedef struct mi_dr_noise {
    int32_t enabled;            /* 0: schedule absent                                  */
    int32_t operation;          /* MI_DR_OP_*          (randomize.py:277-282,298-303)  */
    int32_t distribution;       /* MI_DR_DIST_*        (randomize.py:270-275,290-296)  */
    int32_t frequency_interval; /* on_interval only    (randomize.py:228,252)          */
    float params[2];            /* distribution_parameters: (mean, std) | (lo, hi)     */
} mi_dr_noise;
typedef struct mi_dr_params {
    mi_dr_noise obs_on_reset, obs_on_interval, act_on_reset, act_on_interval;
} mi_dr_params;
/* Randomizer._set_up_{observations,actions}_randomization (randomize.py:176-210): configures
 * the schedules and zeroes the per-env state (counters, correlated-noise epochs). NULL or all
 * disabled turns DR off. Once on, mi_env_step applies the action noise after its clamp and the
 * observation noise before _process_data's clamp, in the same launch (vec_env_rlgames.py:59-71),
 * and requires actions_out (task.actions) for locomotion tasks. */
int mi_task_set_dr(mi_sim* sim, const mi_dr_params* dr /*host|NULL*/);
/* apply_actions_randomization / apply_observations_randomization (randomize.py:212-260) for the
 * method-by-method step: in place on [N,A] actions / [N,O] obs, with the step's reset_buf. */
int mi_dr_apply_actions(mi_sim* sim, float* actions /*[N,A]*/, const int64_t* reset_buf, void* stream);
int mi_dr_apply_observations(mi_sim* sim, float* obs /*[N,O]*/, const int64_t* reset_buf,
                             void* stream);
/* Per-env DR schedule state -> host [N,6] uint32: obs (counter, epoch, draws), act (same). */
int mi_get_dr_state(mi_sim* sim, uint32_t* out /*[N,6] host*/);

/* --- utilities --------------------------------------------------------------------- */
/* U(lo,hi) Philox4x32-10 actions for the random-policy driver (scripts/random_policy.py:57),
 * keyed on (seed, env_id_offset + env, step). */
int mi_fill_uniform(mi_sim* sim, float* out /*[N,cols]*/, int32_t cols, uint64_t seed,
                    uint64_t step, float lo, float hi, void* stream);
/* Per-env reset counters (the Philox counter of the reset noise stream) -> host [N]. */
int mi_get_reset_count(mi_sim* sim, uint32_t* out /*[N] host*/);
/* Host [N] -> the per-env reset counters (restores a recorded state, e.g. a golden fixture's,
 * so the next reset draws the same Philox noise; no reference counterpart: torch's global
 * generator state plays this role there, locomotion.py:120-124). Blocks the host. */
int mi_set_reset_count(mi_sim* sim, const uint32_t* in /*[N] host*/);
/* Pairing by load of the two-envs-per-wavefront kernels (no reference counterpart: tests and
 * diagnostics). Each 16-env workgroup ranks its envs by a per-env load key — the most constraint
 * rows of any substep in the env's last fused env-step — and pairs ranks w and 15 - w in wave w.
 * out: host [N] <- the keys; in: host [N] -> the keys (either may be NULL; in after out);
 * pairing: 0 index pairing (envs 2w, 2w + 1), 1 by load, -1 unchanged. Blocks the host. */
int mi_sim_pair_load(mi_sim* sim, int32_t* out /*[N] host|NULL*/, const int32_t* in /*[N] host|NULL*/,
                     int32_t pairing);
/* Number of env-steps whose physics produced a non-finite state and were forced to reset
 * (issues deferred substeps first and waits for them: blocks the host). */
int mi_sim_nan_count(mi_sim* sim, int64_t* count);
/* Diagnostics: which physics kernel runs. path: 0 one-lane-per-env, 1 wavefront-per-env,
 * 2 two envs per wavefront (the compiled topologies' default; MI_WAVE_PAIR=0 selects path 1);
 * topology: id of the compile-time (model-specialised) topology, 0 = runtime tables;
 * lds_bytes: LDS per env (= per workgroup) of the wave path. Any output may be NULL. */
int mi_sim_kernel_path(const mi_sim* sim, int32_t* path, int32_t* topology, int32_t* lds_bytes);
int mi_abi_version(void);
/* SHA-256 (hex) of the sources this library was compiled from: csrc/mi_sim.hip, the csrc .hpp headers and
 * the include headers in name order (__graft_entry__.source_hash); "unknown" when built without it. A
 * stale binary shows up as a mismatch against the tree (smoke(), tests/test_host.py). */
const char* mi_build_id(void);
const char* mi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MI_SIM_H */
