/*
 * nav_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64 scalar) of the reference's hot path, used as the parity checker for
 * the HIP kernels in residual-td3-robot-navigation_amd/csrc and as the bench's `cpu_baseline` leg.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it. The product path
 * never links or calls this code.
 *
 * Parity pinning: every function below is checked against golden vectors produced by importing the
 * reference itself (tests/golden/make_golden.py, committed fixtures in tests/golden/ (*.npz)).
 *
 * Reference = benmcclusky/Residual-TD3-Robot-Navigation (environment.py, robot.py, robot-learning.py).
 * Third-party algorithm pinned here: numpy 2.2.6 legacy `RandomState` (MT19937, random_sample,
 * masked randint, legacy polar gauss, Fisher-Yates permutation) — the RNG every reference draw uses.
 */
#ifndef NAV_ORACLE_H
#define NAV_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- numpy legacy RandomState (MT19937) ---------------- */
typedef struct {
    uint32_t key[624];
    int pos;
    int has_gauss;
    double gauss;
} orc_mt_t;

void     orc_mt_seed(orc_mt_t* s, uint32_t seed);
uint32_t orc_mt_next32(orc_mt_t* s);
double   orc_mt_double(orc_mt_t* s);               /* random_sample() */
double   orc_mt_gauss(orc_mt_t* s);                /* legacy_gauss() */
int64_t  orc_mt_randint(orc_mt_t* s, int64_t low, int64_t high); /* randint(low, high) masked */
void     orc_mt_permutation(orc_mt_t* s, int64_t n, int64_t* out);
size_t   orc_mt_sizeof(void);

/* ---------------- Philox4x32-10 (the vectorised path's counter RNG) ---------------- */
void   orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_u01(uint32_t hi, uint32_t lo);         /* 53-bit double from two words, numpy formula */

/* ---------------- Environment (environment.py) ---------------- */
/* environment.py:98-119. fields are [100][100] float32, x-major (index cx*100+cy). */
void orc_dynamics(const float* speed, const float* angle, const double* s, const double* a,
                  double* out);
/* environment.py:122-127. returns 1 if the move was committed. */
int  orc_step(const float* speed, const float* angle, double* s, const double* a);
/* environment.py:135-137 with the two random_sample() draws given. */
void orc_reset_u(const double* region, double u0, double u1, double* out);
/* environment.py:28-56 drawn from a numpy legacy stream; returns the goal-draw count. */
int  orc_init_and_goal_mt(orc_mt_t* rs, double* region, double* goal, int* side);
/* environment.py:135-137 drawn from a numpy legacy stream. */
void orc_reset_mt(orc_mt_t* rs, const double* region, double* out);
/* np.linalg.norm of a 2-vector as numpy 2.2.6 + OpenBLAS ddot computes it (fma tail). */
double orc_norm2(double a0, double a1);

/* ---------------- Robot per-step math (robot.py) ---------------- */
/* robot.py:753 — min over the demo set of the scipy cdist euclidean distance (no fma). */
double orc_demo_min(const double* demo_xy, int64_t m, double x, double y);
/* robot.py:727-762 for a one-state path; *goal_reached set as the reference's side effect. */
double orc_compute_reward(const double* next_state, const double* goal, const double* demo_xy,
                          int64_t m, int demo_flag, int* goal_reached, double goal_thr,
                          double goal_reward, double demo_factor);
/* robot.py:509-538 on a 5-slot ring: hist [5][2], *count in 0..5, *head = oldest slot. */
int  orc_check_if_stuck(double* hist, int* count, int* head, const double* s, double thr);

/* ---------------- Vectorised path (same semantics the HIP kernels implement) ---------------- */
typedef struct {
    double world_size, max_action, init_region_size;
    double goal_threshold, goal_reward, stuck_threshold, stuck_penalty, demo_factor, noise_decay;
    int32_t path_length0, path_increase;
    uint32_t seed_lo, seed_hi;
    int32_t max_goal_draws;
} orc_params_t;

void orc_default_params(orc_params_t* p);

/* per-env Philox init: region/goal (environment.py:28-56 semantics). returns goal draws used
 * (0 = rejection cap hit, goal left at the last draw). */
int  orc_vec_init_one(const orc_params_t* p, uint32_t stream_id, double* region, double* goal);
/* per-env Philox reset draw for episode `ep` (environment.py:135-137 semantics). */
void orc_vec_reset_one(const orc_params_t* p, uint32_t env, uint32_t ep, const double* region,
                       double* out);
/* per-env Box-Muller pair for the exploration noise at vector step `step`. */
void orc_vec_noise_one(const orc_params_t* p, uint32_t env, uint32_t step, double* z);

/* One training tick of env e, fused the way nav_agent_step fuses it (robot.py:443-506, 509-538,
 * 645-675, 727-762; environment.py:130-137, 98-127). All per-env arrays are this env's slots.
 * meta: bit0 goal_reached, bit1 stuck, bit2 demo_flag, bits 8-10 hist count, bits 12-14 hist head.
 * Writes the replay row [8] float32 = s0 s1 a0 a1 r s'0 s'1 done; returns flags bit0 done,
 * bit1 goal, bit2 stuck, bit3 episode ended. */
int orc_vec_agent_tick(const orc_params_t* p, const float* speed, const float* angle,
                       const double* demo_xy, int64_t m, uint32_t env,
                       double* state, const double* goal, const double* region, double* hist,
                       uint32_t* meta, int32_t* plan_index, int32_t* path_length,
                       int32_t* episodes, double* noise_scale, const double* action,
                       double* next_state_out, float* replay_row, double* reward_out,
                       const double* reset_state /* NULL = Philox reset draw */);

/* Fused act epilogue restated: a = clip(b + residual + sigma*5*z, +-max) with b = s - g. */
void orc_act_epilogue(const double* s, const double* g, const float* residual, double sigma,
                      const double* z, double max_action, double* out);

/* Whole-batch helpers for the cpu_baseline leg (OpenMP over envs when built with -fopenmp). */
int  orc_threads(void);
void orc_set_threads(int n); /* OpenMP team size of the batched tick (cpu_baseline) */
void orc_vec_agent_step_batch(const orc_params_t* p, const float* speed, const float* angle,
                              const double* demo_xy, int64_t m, int64_t n, double* state,
                              const double* goal, const double* region, double* hist,
                              uint32_t* meta, int32_t* plan_index, int32_t* path_length,
                              int32_t* episodes, double* noise_scale, const double* action,
                              double* next_state_out, float* replay_rows, int64_t replay_cap,
                              int64_t replay_base, int64_t env0 /* global index of env 0 */,
                              const int64_t* idx_start, const int32_t* idx_cand /* nullable */);

/* Exact nearest-demo index (per index cell of width 1/ORC_DEMO_RES, the candidates that can be
 * nearest to any query in the cell; built from the 1 x 1 dynamics cells' lists):
 * cell_start [(100 ORC_DEMO_RES)^2 + 1], cand [returned total]; call with cand = NULL (cap 0) to
 * size. orc_demo_min_idx = orc_demo_min through it, the same f64 value.
 * ORC_DEMO_RES: index cells per dynamics cell side (= libnavenv's nav_demo_index_res) */
#ifndef ORC_DEMO_RES
#define ORC_DEMO_RES 4
#endif
int32_t orc_demo_index_res(void);
int64_t orc_demo_index_build(const double* demo_xy, int64_t m, int64_t* cell_start, int32_t* cand,
                             int64_t cap);
double orc_demo_min_idx(const double* demo_xy, int64_t m, const int64_t* cell_start,
                        const int32_t* cand, double x, double y);
/* K single-env steps on one core: Environment.step alone (tick 0) or the whole agent tick (1). */
double orc_single_env_run(const orc_params_t* p, const float* speed, const float* angle,
                          const double* demo_xy, int64_t m, const int64_t* idx_start,
                          const int32_t* idx_cand, const double* actions, int64_t n_act,
                          int64_t K, int tick);

#ifdef __cplusplus
}
#endif
#endif
