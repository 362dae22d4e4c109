/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement used as the parity checker for
 * libmi_sim.so. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so; the product (omniisaacgymenvs_amd) never does.
 *
 * Pinning status:
 *  - Task math (obs / reward / done / reset, locomotion + cartpole) restates the reference's
 *    TorchScript text (tasks/shared/locomotion.py:80-321, tasks/humanoid.py:116-127,
 *    tasks/ant.py:88-95, tasks/cartpole.py:80-162). The reference has no tests and its
 *    closed helpers (omni.isaac.core.utils.torch) are absent, so it is pinned by the
 *    hand-derived known-answer tests of SURVEY §8(c) (tests/test_oracle_kat.py).
 *  - Physics: the reference's physics is closed PhysX; physics parity is UNPINNED against
 *    PhysX. The articulated integrator here is the build's own algorithm written
 *    independently of the HIP path (dense Jacobian-sum mass matrix + dense Cholesky vs.
 *    the device's tree CRBA + LTDL) and is pinned by physical invariants (energy,
 *    momentum, ABA cross-check) in tests/test_oracle_physics.py.
 *  - Philox4x32-10 is pinned by Random123's published known-answer vectors.
 */
#ifndef MI_ORACLE_H
#define MI_ORACLE_H
#include <stdint.h>
#include "../include/mi_sim.h"   /* data-layout structs only (the boundary spec) */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_sim orc_sim;

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float orc_uniform(uint64_t seed, uint64_t env_id, uint32_t counter_hi, uint32_t slot,
                  uint32_t stream);

orc_sim* orc_sim_create(const mi_model_desc* model, const mi_sim_params* params, int32_t num_envs,
                        int64_t env_id_offset, const float* env_origins, uint64_t seed);
void orc_sim_destroy(orc_sim* s);
int orc_sim_num_dof(const orc_sim* s);
void orc_set_threads(int n);

/* state access (host arrays, row-major like the device API) */
void orc_get_root_state(const orc_sim* s, float* pos, float* quat, float* vel);
void orc_get_dof_state(const orc_sim* s, float* q, float* qd);
void orc_get_sensor_wrench(const orc_sim* s, float* out);
void orc_set_root_state(orc_sim* s, const float* pos, const float* quat, const float* vel);
void orc_set_dof_state(orc_sim* s, const float* q, const float* qd);
void orc_set_dof_efforts(orc_sim* s, const float* eff);
void orc_get_reset_count(const orc_sim* s, uint32_t* out);
void orc_set_reset_count(orc_sim* s, const uint32_t* in);
int64_t orc_nan_count(const orc_sim* s);

void orc_sim_step(orc_sim* s, int substeps);

/* task layer */
void orc_task_configure(orc_sim* s, const mi_task_params* tp);
void orc_task_pre_step(orc_sim* s, const float* actions, int64_t* reset_buf, int64_t* progress_buf,
                       float* potentials, float* prev_potentials, float* actions_out);
void orc_task_post_step(orc_sim* s, const float* actions, float* obs, float* rew, int64_t* reset_buf,
                        int64_t* progress_buf, float* potentials, float* prev_potentials);
void orc_env_step(orc_sim* s, const float* actions, int substeps, float* obs_out, float* obs_task,
                  float* rew, int64_t* reset_buf, int64_t* progress_buf, float* potentials,
                  float* prev_potentials, float* actions_out);
void orc_task_reset_idx(orc_sim* s, const int64_t* env_ids, int n, int64_t* reset_buf,
                        int64_t* progress_buf, float* potentials, float* prev_potentials);

/* observation / action noise DR (randomize.py:176-306, include/mi_dr.h) */
void orc_task_set_dr(orc_sim* s, const mi_dr_params* dr /*NULL = off*/);
void orc_dr_apply_actions(orc_sim* s, float* actions, const int64_t* reset_buf);
void orc_dr_apply_observations(orc_sim* s, float* obs, const int64_t* reset_buf);
void orc_get_dr_state(const orc_sim* s, uint32_t* out /*[N,6]*/);

/* stateless task math on caller-provided state (KAT + device task-kernel parity) */
void orc_loco_post_math(const mi_task_params* tp, int N, int D, int S, const float* root_pos,
                        const float* root_quat, const float* root_vel, const float* q,
                        const float* qd, const float* sensors, const float* actions,
                        const float* lower, const float* upper, float* obs, float* rew,
                        int64_t* reset_buf, int64_t* progress_buf, float* potentials,
                        float* prev_potentials);
void orc_cartpole_post_math(const mi_task_params* tp, int N, const float* q, const float* qd,
                            float* obs, float* rew, int64_t* reset_buf, int64_t* progress_buf);

/* physics cross-checks for one env (dense terms; n = 6*root_free + D) */
void orc_dynamics_terms(orc_sim* s, int env, float* M /*[n,n]*/, float* C /*[n]*/);
void orc_aba(orc_sim* s, int env, const float* tau /*[n]*/, float* udot /*[n]*/);
double orc_energy(orc_sim* s, int env);
void orc_momentum(orc_sim* s, int env, double* out6 /* angular about world origin, linear */);
int orc_contact_count(orc_sim* s, int env);
float orc_self_min_gap(orc_sim* s, int env);
void orc_decision_margin(const orc_sim* s, float* out /*[N]*/);
/* per env: how close any row's unprojected lambda came to a bound of its projection in the last
 * physics call, in row-velocity units (diagnostic for tools/parity_stats.py; not an exemption) */
void orc_projection_margin(const orc_sim* s, float* out /*[N]*/);

#ifdef __cplusplus
}
#endif
#endif
