/*
 * navenv.h — C-ABI of libnavenv.so, the MI355X (gfx950) drop-in for the reference's hot path:
 * the Environment.step()/reset() simulator (environment.py) and the residual-TD3 agent's per-step
 * math and learner (robot.py) of benmcclusky/Residual-TD3-Robot-Navigation.
 *
 * Conventions (all entry points):
 *  - plain pointers and sizes only; every array pointer is DEVICE memory owned by the caller
 *    (torch tensors on the Python side), except `nav_params` / `nav_mlp` descriptors, which are
 *    host structs passed by pointer and copied into the launch;
 *  - asynchronous on the given stream (a hipStream_t passed as void*; NULL = default stream);
 *    no allocation, no synchronisation inside a launch function (graph-capturable);
 *  - return 0 on success, NAV_EINVAL for a bad argument (checked on the host before any launch),
 *    or -(hipError_t) when a launch fails; nothing aborts;
 *  - one caller thread per stream; the library keeps no global mutable state.
 *
 * Reference interface each entry replaces is cited as file:line of /root/reference.
 */
#ifndef NAVENV_H
#define NAVENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NAV_ABI_VERSION 11
#define NAV_EINVAL (-100000)

#define NAV_WORLD_CELLS 100 /* field = float32 [100][100][2] (speed, angle), x-major: cell cx*100+cy
                              (environment.py:20-21 dynamics_speed / dynamics_angle interleaved) */
#define NAV_HIST 5          /* STUCK_STEPS, robot.py:40 */
#define NAV_ROW 8           /* replay row: s0 s1 a0 a1 r s'0 s'1 done (float32) */

/* Philox4x32-10 stream tags (counter word 2). key = (seed_lo, seed_hi). */
#define NAV_TAG_INIT 1   /* ctr = (draw, stream_id, 1, 0)     set_init_and_goal draws   */
#define NAV_TAG_RESET 2  /* ctr = (0, env, 2, episode)        reset draw                */
#define NAV_TAG_NOISE 3  /* ctr = (0, env, 3, step)           exploration noise pair    */
#define NAV_TAG_SAMPLE 4 /* ctr = (i, 0, 4, update)           replay sample index       */
#define NAV_TAG_TNOISE 5 /* ctr = (row, 0, 5, update)         target-smoothing noise    */

/* Constants of constants.py / robot.py as a POD (defaults in nav_default_params). */
typedef struct nav_params {
    double world_size;       /* constants.py:6  WORLD_SIZE = 100 */
    double max_action;       /* constants.py:34 ROBOT_MAX_ACTION = 5 */
    double init_region_size; /* constants.py:25 INIT_REGION_SIZE = 25 */
    double goal_threshold;   /* constants.py:50 TEST_DISTANCE_THRESHOLD = 5 (robot.py:744) */
    double goal_reward;      /* robot.py:42 GOAL_REWARD = 50 */
    double stuck_threshold;  /* robot.py:39 STUCK_THRESHOLD = 2 */
    double stuck_penalty;    /* robot.py:41 STUCK_PENALTY = 50 */
    double demo_factor;      /* robot.py:43 DEMO_PROXIMITY_FACTOR = 10 */
    double noise_decay;      /* robot.py:33 NOISE_DECAY = 0.75 */
    int32_t path_length0;    /* robot.py:28 PATH_LENGTH = 50 */
    int32_t path_increase;   /* robot.py:29 PATH_INCREASE = 20 */
    uint32_t seed_lo, seed_hi; /* configuration.py:26 RANDOM_SEED by default */
    int32_t max_goal_draws;  /* cap on environment.py:52's rejection loop (default 65536) */
} nav_params;

/* Per-env state, structure-of-arrays, n envs (device). */
typedef struct nav_env_soa {
    int64_t n;
    double* state;        /* [n][2]  Environment.robot_state (environment.py:17)           */
    double* goal;         /* [n][2]  Environment.goal_state / Robot.goal_state              */
    double* region;       /* [n][4]  Environment.robot_init_region (left,right,bottom,top)  */
    double* hist;         /* [5][n][2] Robot.previous_states ring (robot.py:425, 509-538)   */
    uint32_t* meta;       /* [n] bit0 goal_reached, bit1 stuck_flag, bit2 demo_flag,
                             bits 8-10 history count, bits 12-14 history head              */
    int32_t* plan_index;  /* [n] Robot.plan_index (robot.py:424) — value at the NEXT step   */
    int32_t* path_length; /* [n] Robot.path_length (robot.py:423)                            */
    int32_t* episodes;    /* [n] Robot.num_episodes (robot.py:421)                           */
    double* noise_scale;  /* [n] Robot.current_noise_scale (robot.py:422)                    */
} nav_env_soa;

/* Per-step outputs of nav_agent_step (device, nullable fields noted). */
typedef struct nav_step_out {
    double* next_state;   /* [n][2] next state BEFORE any auto-reset (Environment.step return) */
    double* goal_term;    /* [n] -||s'-goal|| (robot.py:741), consumed by nav_demo_reward      */
    uint8_t* flags;       /* [n] bit0 done, bit1 goal, bit2 stuck, bit3 ended, bit4 demo term  */
    float* block_stats;   /* nullable: [ceil(n/64)][8], row k = envs [64k, 64k+64): sum of the
                             reward pushed to the replay rows, n_done, n_goal, n_stuck, n_ended,
                             0, 0, 0 (one wave's shuffle tree per row: deterministic). The sum
                             is of the final pushed rewards in every launch form: the demo pass
                             of nav_agent_step_indexed / nav_act_tick runs in the same launch;
                             after nav_agent_step with demo_pending, nav_demo_reward(_indexed)
                             given this pointer rewrites the rows of flagged envs             */
} nav_step_out;

/* Replay ring (device): rows [capacity][8] float32 (robot.py:58-124 ReplayBuffer). */
typedef struct nav_replay {
    float* rows;
    int64_t capacity;
} nav_replay;

/* ReLU MLP (robot.py:128-206) in the device layout: one flat fp32 buffer per network,
 * hidden width padded to a multiple of 32 with zeros (exact: relu(0)=0, zero rows/cols add 0):
 *   W0 [hp][d_in], b0 [hp], {Wl [hp][hp], bl [hp]} x (n_hidden-1), Wo [d_out][hp], bo [d_out]
 * plus `packed` = per hidden->hidden layer the fp16 MFMA B-operand images of the forward
 * (B[k][n] = W[n][k]) then of the backward (B[k][n] = W[k][n]; for d_out = 1 the top hidden
 * layer's backward image holds B[k][n] = fl32(Wo[0][k] W[k][n]), the operand of the row
 * backward's bit-operand product, ABI 11) product: per column n an exponent
 * e_n (B's column max |B| 2^e_n in [2^13, 2^14)) and each entry as two fp16 planes hi =
 * fp16(B 2^e_n), lo = fp16(B 2^e_n - hi) (22 significant bits), laid out [plane 2][hp/16][2][hp][8]
 * (entry (p, k/16, (k/8)&1, n, k&7)) followed by int32 e[hp]: hp^2 + hp floats per image; rebuilt
 * after every writer by nav_adam(_multi) / nav_polyak(_multi) / nav_grad_reduce_adam(_polyak) /
 * nav_mlp_pack (one extra launch on the same stream). ABI 10: the image format (ABI 9: three
 * bf16 planes, 1.5 hp^2 floats). */
typedef struct nav_mlp {
    int32_t d_in;       /* 2 actor (robot.py:145), 4 critic (robot.py:185) */
    int32_t d_out;      /* 2 actor, 1 critic */
    int32_t hidden;     /* logical width: 200 reference, 256 perf config */
    int32_t hidden_pad; /* multiple of 32, <= 256 */
    int32_t n_hidden;   /* hidden layers: 3 reference, 2 perf config */
    float* params;      /* flat, nav_mlp_param_count floats */
    float* packed;      /* nav_mlp_packed_count floats (may be NULL only for n_hidden == 1) */
} nav_mlp;

/* ---- version / descriptors ---- */
int nav_abi_version(void);
void nav_default_params(nav_params* p);
int64_t nav_mlp_param_count(int32_t d_in, int32_t d_out, int32_t hidden_pad, int32_t n_hidden);
int64_t nav_mlp_packed_count(int32_t hidden_pad, int32_t n_hidden);
/* float offset of layer l's W and b inside the flat buffer (l = 0 .. n_hidden) */
int nav_mlp_layer_offsets(const nav_mlp* net, int32_t layer, int64_t* w_off, int64_t* b_off);

/* ---- Environment (environment.py) ---- */
/* environment.py:28-56 set_init_and_goal per env, Philox stream_id = env / envs_per_group (so a
 * group shares region and goal); also initialises the Robot fields to their values at the first
 * training step after the demonstration phase (robot.py:443-489 trace: plan_index 5, path 50,
 * episodes 5, noise 1, demo_flag as given) and draws the first reset (environment.py:130-137).
 * draws_out (nullable) [n]: goal draws used, 0 = rejection cap hit. */
int nav_env_init(const nav_params* p, const nav_env_soa* env, int32_t envs_per_group,
                 int32_t demo_flag, int32_t* draws_out, void* stream);
/* environment.py:130-137 Environment.reset: state = low + (high-low)*u for envs with mask != 0
 * (mask NULL = all). u from `uniforms` [n][2] if given (e.g. the numpy stream of robot-learning.py:19,
 * for reference-stream parity) else Philox (NAV_TAG_RESET, episode = episodes[e]). */
int nav_env_reset(const nav_params* p, const nav_env_soa* env, const uint8_t* mask,
                  const double* uniforms, void* stream);
/* environment.py:122-127 Environment.step for n envs: state <- dynamics(state, action) when the
 * result is inside the world. action [n][2] f64. next_state (nullable) receives the result. */
int nav_env_step(const nav_params* p, const nav_env_soa* env, const float* field,
                 const double* action, double* next_state, void* stream);
/* environment.py:122-127 Environment.step applied K times in one launch (the pure-step loop of
 * robot-learning.py's tick without the agent): the state stays in registers; actions [K][n][2] f64;
 * next_states (nullable) [K][n][2] receives each step's committed state. */
int nav_env_step_k(const nav_params* p, const nav_env_soa* env, const float* field,
                   const double* actions, int32_t K, double* next_states, void* stream);
/* environment.py:98-119 Environment.dynamics, pure: out = f(state, action), n pairs. */
int nav_dynamics(const float* field, const double* state, const double* action, double* out,
                 int64_t n, void* stream);

/* ---- Robot per-step (robot.py) ---- */
/* One training tick for every env, fused: Environment.step (environment.py:122-127) ->
 * Robot.process_transition (robot.py:645-675: reward w/o demo term, check_if_stuck, done, push
 * to the replay row (replay_base + e) % capacity) -> next tick's end-of-episode check and
 * Robot.reset + Environment.reset (robot.py:479-506, environment.py:130-137).
 * demo_pending != 0: the caller runs nav_demo_reward(_indexed) next for the envs flagged
 * (flags bit4) — their demo-proximity term and stuck penalty are written then; 0: no demo set
 * exists, so (robot.py:749-751) the reward is the goal term and the stuck penalty is taken here.
 * replay->capacity must be >= n (one slot per env per launch). */
int nav_agent_step(const nav_params* p, const nav_env_soa* env, const float* field,
                   const double* action, const nav_replay* replay,
                   int64_t replay_base, const nav_step_out* out, int32_t demo_pending,
                   void* stream);
/* Robot.process_transition (robot.py:645-675) without the environment step, for callers that
 * step the Environment themselves (the N = 1 drop-in): reward w/o demo term, check_if_stuck,
 * done, replay push; meta/hist updated, plan_index/path_length read (not advanced).
 * demo_pending as nav_agent_step. */
int nav_transition(const nav_params* p, const nav_env_soa* env, const double* state,
                   const double* action, const double* next_state, const nav_replay* replay,
                   int64_t replay_base, const nav_step_out* out, int32_t demo_pending,
                   void* stream);
/* Robot.check_if_stuck (robot.py:509-538) alone: updates the history ring (hist, meta bits
 * 8-14) with `state` [n][2] and writes stuck [n] (0/1). */
int nav_check_if_stuck(const nav_params* p, const nav_env_soa* env, const double* state,
                       uint8_t* stuck, void* stream);
/* robot.py:741-762 demo-proximity term for envs flagged by nav_agent_step:
 * r = (goal_term + demo_factor * -min_j ||s' - d_j||) - stuck_penalty*stuck, written to the
 * replay row. demo_xy [m][2] f64 per group: group g = env / envs_per_group uses
 * demo_xy[demo_off[g] .. demo_off[g+1]) (demo_off NULL = one shared set of m points).
 * block_stats (nullable, nav_step_out's [ceil(n/64)][8] of the nav_agent_step this pass
 * completes): the reward column of every 64-env row holding a flagged env is summed again from
 * the final pushed rewards, so it equals the one-launch forms' column bit for bit. */
int nav_demo_reward(const nav_params* p, int64_t n, const double* next_state,
                    const double* goal_term, const uint8_t* flags, const double* demo_xy,
                    const int64_t* demo_off, int64_t m, int32_t envs_per_group,
                    const nav_replay* replay, int64_t replay_base, double* reward_out,
                    float* block_stats, void* stream);
/* Exact bucketed nearest-demo index (robot.py:753 made sublinear, result bit-identical to the
 * brute force), built in two levels.
 * Level 1, the 100 x 100 dynamics cells over all points of each group: for each (group, cell) the
 * bound U^2 = min_q maxdist^2(q, cell) and the candidate count (plan), an exclusive scan into
 * cell_start [n_groups*10000 + 1] (scan), then ascending group-relative point indices (fill).
 * cell_bound f64 / cell_count i32: [n_groups][10000]; cand: cell_start[last] int32 entries.
 * Level 2, the query index: every dynamics cell split into R x R index cells (R =
 * nav_demo_index_res(), a power of 2; index cell of s = ((int)(s.x*R), (int)(s.y*R)) on a
 * 100R x 100R grid, x-major), each cell's list taken from its level-1 parent's list (subplan),
 * scanned (subscan) and filled (subfill). sub_bound f64 / sub_count i32: [n_groups][(100R)^2];
 * sub_start [n_groups*(100R)^2 + 1]; sub_cand: sub_start[last] int32 entries. The reward entry
 * points below take (sub_start, sub_cand) as their (cell_start, cand). */
int nav_demo_index_plan(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                        int64_t m, double* cell_bound, int32_t* cell_count, void* stream);
int nav_demo_index_scan(const int32_t* cell_count, int32_t n_groups, int64_t* cell_start,
                        void* stream);
int nav_demo_index_fill(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                        int64_t m, const double* cell_bound, const int64_t* cell_start,
                        int32_t* cand, void* stream);
int32_t nav_demo_index_res(void);
int nav_demo_index_subplan(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                           const int64_t* cell_start, const int32_t* cand, double* sub_bound,
                           int32_t* sub_count, void* stream);
int nav_demo_index_subscan(const int32_t* sub_count, int32_t n_groups, int64_t* sub_start,
                           void* stream);
int nav_demo_index_subfill(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                           const int64_t* cell_start, const int32_t* cand,
                           const double* sub_bound, const int64_t* sub_start, int32_t* sub_cand,
                           void* stream);
/* nav_demo_reward through the level-2 index (same result, a few instead of 11 355 points per
 * env; block_stats as there). */
int nav_demo_reward_indexed(const nav_params* p, int64_t n, const double* next_state,
                            const double* goal_term, const uint8_t* flags, const double* demo_xy,
                            const int64_t* demo_off, int32_t envs_per_group,
                            const int64_t* cell_start, const int32_t* cand,
                            const nav_replay* replay, int64_t replay_base, double* reward_out,
                            float* block_stats, void* stream);
/* nav_agent_step + nav_demo_reward_indexed in one launch (same results bit for bit): flagged envs
 * get their demo-proximity reward through the index before the replay row is written, so the row
 * is stored once with the final reward. reward_out (nullable) [n] receives the reward of the
 * flagged envs only, as nav_demo_reward_indexed writes it. Replaces the pair of calls the
 * reference makes per step: robot.py:661-675 process_transition -> compute_reward (727-762). */
int nav_agent_step_indexed(const nav_params* p, const nav_env_soa* env, const float* field,
                           const double* action, const nav_replay* replay, int64_t replay_base,
                           const nav_step_out* out, const double* demo_xy,
                           const int64_t* demo_off, int32_t envs_per_group,
                           const int64_t* cell_start, const int32_t* cand, double* reward_out,
                           void* stream);
/* robot.py:753 min_j ||p_i - d_j|| (scipy cdist euclidean, f64) for n points [n][2]. */
int nav_demo_min(const double* points, int64_t n, const double* demo_xy, int64_t m,
                 double* out, void* stream);
/* Pure robot.py:727-762 compute_reward for n next-states, f64 out; goal_hit (nullable) [n]
 * receives the goal_reached side effect (robot.py:745). */
int nav_compute_reward(const nav_params* p, int64_t n, const double* next_state,
                       const double* goal, const double* demo_xy, int64_t m, int32_t demo_flag,
                       double* reward, uint8_t* goal_hit, void* stream);

/* Batched open-loop rollouts of Environment.dynamics (the CEM demonstrator's inner loop,
 * environment.py:151-165): P paths x T steps; start [P][2], actions [P][T][2] f64 ->
 * paths [P][T+1][2] f64; reward (nullable) [P] = -||f32(s_T) - goal|| (environment.py:182-183). */
int nav_rollout(const float* field, int64_t P, int32_t T, const double* start,
                const double* actions, double* paths, const double* goal, double* reward,
                void* stream);
/* The CEM demonstrator batched over n_prob independent problems (environment.py:140-179; one per
 * (group, demonstration)), P paths x T steps each. nav_cem_rollout runs CEM iteration `iter` for
 * every path of every problem: start = region_sample(region[prob], uniforms[prob]) (environment.py:
 * 150, 136), actions a0 [n][P][T][2] (iteration 0, the +-5 np.random.choice draws) or
 * mean[prob][t] + std[prob][t] * z [n][P][T][2] in f64 (np.random.normal's loc + scale * gauss),
 * written as float32 to actions [n][P][T][2] (planning_actions); paths (nullable) [n][P][T+1][2]
 * float32 (planning_paths); reward [n][P] = -||f32(s_T) - goal|| (environment.py:164, 182-183).
 * nav_cem_elite: per problem the E best paths (ascending reward order, ties by path index), their
 * float32 action mean / std [n][T][2] (numpy float32 reductions over the elites in that order);
 * best (nullable) [n] = first argmax of the rewards (environment.py:166-175). P <= 256. */
int nav_cem_rollout(const float* field, int32_t n_prob, int32_t P, int32_t T, int32_t iter,
                    const double* region, const double* uniforms, const double* goal,
                    const double* a0, const double* z, const float* mean, const float* stdv,
                    float* actions, float* paths, double* reward, void* stream);
int nav_cem_elite(int32_t n_prob, int32_t P, int32_t T, int32_t E, const double* reward,
                  const float* actions, float* mean, float* stdv, int32_t* best, void* stream);
/* environment.py:59-95 set_dynamics as nav.fields restates it (perlin_noise is absent: the field
 * values are parity unpinned against the reference): unit gradient tables g5 [6][6][2],
 * g10 [11][11][2], g20 [21][21][2], f64, from the host's seeded draws. The speed cells mix the
 * three octaves (environment.py:72-74); the angle cells are the SAME octave-5 noise (:85 is the
 * function of :62), min-max normalised. field out [100][100][2] float32 (speed, angle) x-major,
 * the table every dynamics kernel reads. Same f32 values as nav.fields.make_fields (angle bit
 * for bit, speed within 4 ulp: numpy's f32 exp). */
int nav_fields_generate(const double* g5, const double* g10, const double* g20, float* field,
                        void* stream);
/* Robot.process_demonstration's demonstration set for n_demo demonstrations (robot.py:694-698,
 * 771-824): per demo its T states [T][2] (f32, the CEM output) followed by n_aug augmentations
 * of (T-1)*(steps+1) + 1 states each, f64 out [n_demo][T + n_aug*((T-1)(steps+1)+1)][2];
 * noise [n_demo][n_aug][(T-1)(steps+1)*4 + 4] = each augmentation's np.random.normal draws in the
 * reference's order. Bit-identical to the numpy restatement nav.demos.demo_set_from. */
int nav_demo_augment(int32_t n_demo, int32_t T, int32_t steps, int32_t n_aug,
                     const float* states, const double* noise, double* out, void* stream);
/* ReplayBuffer.push (robot.py:79-96) of n transitions (f64 in, float32 rows), slots
 * (base + i) % capacity. */
int nav_replay_push(const nav_replay* replay, int64_t base, int64_t n, const double* state,
                    const double* action, const double* reward, const double* next_state,
                    const uint8_t* done, void* stream);

/* ---- Actor / critic MLPs on MFMA (robot.py:128-206) ---- */
/* Action selection, fused: residual = actor(f32(state - goal)) (robot.py:598-624) and the
 * epilogue a = clip(b + residual + noise, +-max_action) (robot.py:541-569). mode 0 = training
 * (noise = noise_scale*max_action*z; z from `noise_z` [n][2] f64 if given, else Philox
 * NAV_TAG_NOISE at `step`), mode 1 = testing (robot.py:572-595, no noise). action_out [n][2] f64;
 * residual_out (nullable) [n][2] f32. */
int nav_act(const nav_params* p, const nav_mlp* actor, int64_t n, const double* state,
            const double* goal, const double* noise_scale, const double* noise_z,
            uint32_t step, int32_t mode, double* action_out, float* residual_out, void* stream);

/* nav_act (training or testing mode, noise from noise_z or Philox) and nav_agent_step_indexed
 * (demo_xy given) / nav_agent_step with demo_pending 0 (demo_xy NULL) in ONE launch: the actor's
 * action epilogue hands each env's action to that env's training tick in the same workgroup, so
 * the action never round-trips through memory (action_out nullable). Same results as the two
 * launches, bit for bit (robot.py:541-569 then the tick of nav_agent_step; the robot-learning.py
 * 'step' tick, robot-learning.py:95-101). */
int nav_act_tick(const nav_params* p, const nav_mlp* actor, const nav_env_soa* env,
                 const float* field, const double* noise_z, uint32_t step, int32_t mode,
                 const nav_replay* replay, int64_t replay_base, const nav_step_out* out,
                 const double* demo_xy, const int64_t* demo_off, int32_t envs_per_group,
                 const int64_t* cell_start, const int32_t* cand, double* action_out,
                 double* reward_out, void* stream);
/* Generic forward of up to 2 networks sharing one input (twin critics), rows [M]:
 * x = in[m*ld_in + in_col + 0..d_in) (f32). out_mode 0: out[m*ld_out + out_col + j] = y;
 * out_mode 1 (target policy smoothing, robot.py:336-339): out = clamp(y + clamp(policy_noise*eps,
 * +-noise_clip), +-max_action) with eps from `eps` [M][2] f32 if given else Philox
 * (NAV_TAG_TNOISE, counter). acts (nullable, per net): [n_hidden][M][hp] post-ReLU activations,
 * layer L written when bit L of save_mask is set; masks (nullable, per net): nav_mlp_mask_count
 * u16 words of ReLU-derivative bits (for nav_mlp_backward / nav_mlp_wgrad). */
int nav_mlp_forward(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                    int32_t ld_in, int32_t in_col, float* const* out, int32_t ld_out,
                    int32_t out_col, int32_t out_mode, const float* eps, float policy_noise,
                    float noise_clip, float max_action, uint32_t seed_lo, uint32_t seed_hi,
                    uint32_t counter, float* const* acts, uint32_t save_mask,
                    uint16_t* const* masks, void* stream);
/* train_critic's row-local part (robot.py:329-353) in one launch: per batch row b, sample
 * rows[k] of the replay ring (k = idx[b] if given, else Philox NAV_TAG_SAMPLE at 2*counter, with
 * replacement over [0, size)) into batch [B][8]; a' = clamp(target_actor(s') + clamp(policy_noise
 * * eps, +-noise_clip), +-max_action) with eps from `eps` [B][2] if given else Philox
 * NAV_TAG_TNOISE at counter; y = r + gamma*min(target_critics[0](s', a'), target_critics[1](s',
 * a'))*(1 - done); then both online critics on (s, a) as nav_td3_critic_forward (dq, loss_part,
 * edge_slabs, acts/save_mask, masks). With row_backward != 0 each online critic's row backward
 * (robot.py:361) follows its forward in the same launch, as nav_mlp_backward of dq with the
 * batch's (s, a) columns as input: W0 / bias partials into edge_slabs, dz rows of dz_save_mask
 * layers into dz[i] — the caller then skips nav_mlp_backward. split_twins: 1 = the twin online
 * critics in separate workgroups (grid.y = 2, each repeating the target passes: the small-batch
 * form), 0 = both in one workgroup, < 0 = the library's choice (split for B <= 2048); the
 * results are bit-identical either way. */
int nav_td3_critic_rows(const nav_mlp* target_actor, const nav_mlp* target_critics,
                        const nav_mlp* critics, const nav_replay* replay, int64_t size,
                        int64_t B, const int64_t* idx, uint32_t seed_lo, uint32_t seed_hi,
                        uint32_t counter, const float* eps, float policy_noise,
                        float noise_clip, float max_action, float gamma, float* batch,
                        float* const* dq, float* const* loss_part, float* const* edge_slabs,
                        float* const* acts, uint32_t save_mask, uint16_t* const* masks,
                        int32_t row_backward, float* const* dz, uint32_t dz_save_mask,
                        int32_t split_twins, void* stream);
/* train_actor's row-local part (robot.py:382-390) in one launch: sample rows (Philox
 * NAV_TAG_SAMPLE at 2*counter + 1, or idx) into batch [B][8]; actor forward on s (ReLU bits to
 * masks_actor, activations to acts for save_mask bits; the top layer's dWo partials come
 * from registers, so it need not be saved);
 * q [B] (nullable) = critic(s, actor(s)); dL/da of L = -mean(q) through the critic (masks_critic)
 * into da [B][2]; the actor's row backward with dz_save_mask rows to dz and its edge partials. */
int nav_td3_actor_rows(const nav_mlp* actor, const nav_mlp* critic, const nav_replay* replay,
                       int64_t size, int64_t B, const int64_t* idx, uint32_t seed_lo,
                       uint32_t seed_hi, uint32_t counter, float* batch, float* q, float* da,
                       float* acts, uint32_t save_mask, float* dz, uint32_t dz_save_mask,
                       uint16_t* masks_actor, uint16_t* masks_critic, float* edge_slabs,
                       void* stream);
/* u16 words of the ReLU mask image for M rows (layout: [n_hidden][row tiles][hp/32][64]). */
int64_t nav_mlp_mask_count(int32_t hidden_pad, int32_t n_hidden, int64_t M);
/* Parameter gradients are produced in two parts that nav_grad_reduce combines:
 *  - edge slabs [row blocks][nav_mlp_edge_count]: per row block of the forward/backward launches
 *    (nav_mlp_row_blocks(M) blocks), partial sums of every parameter except the hidden x hidden
 *    weights, in the flat order with those segments cut out (W0 | b0 .. b_{n_hidden-1} | Wo | bo);
 *  - hidden slabs [splits][nav_mlp_hidden_count]: nav_mlp_wgrad's split-M partials of
 *    W_1 .. W_{n_hidden-1}. */
int64_t nav_mlp_row_blocks(int64_t M);
int64_t nav_mlp_edge_count(int32_t d_in, int32_t d_out, int32_t hidden_pad, int32_t n_hidden);
int64_t nav_mlp_hidden_count(int32_t hidden_pad, int32_t n_hidden);
/* train_critic's online twin forward (robot.py:341-361), nets[2] critics (d_out 1) on
 * x = in[b*ld_in + in_col + 0..4): y = r + gamma*min(q1t, q2t)*(1 - done) from the replay batch
 * [B][8] (r at column 4, done at 7); dq[i] [B] = 2*(q_i - y)/B (mse_loss backward);
 * loss_part[i] [row blocks] = block sums of (q_i - y)^2; edge_slabs[i] (nullable) receive the
 * output layer's Wo / bo partials; acts/save_mask as nav_mlp_forward; masks[i] required. */
int nav_td3_critic_forward(const nav_mlp* nets, int64_t B, const float* in, int32_t ld_in,
                           int32_t in_col, const float* batch, const float* q1t, const float* q2t,
                           float gamma, float* const* dq, float* const* loss_part,
                           float* const* edge_slabs, float* const* acts, uint32_t save_mask,
                           uint16_t* const* masks, void* stream);
/* Row-local backward (autograd of robot.py:355-395) of 1 or 2 networks of the same shape that
 * share the input rows (the twin critics: one launch): per net i, dL/dy rows
 * dy[i][m*ld_dy + 0..d_out) (ld_dy 0: one row for all) and the forward's ReLU masks[i] give dL/dz
 * of every hidden layer, dz_L written to dz[i] [n_hidden][M][hp] for bits L of save_mask;
 * dx[i] (nullable) [M][d_in] = dL/dx. edge_slabs[i] (nullable): per-block W0 / bias partials
 * (input rows from `in`), plus Wo / bo when h_top[i] [M][hp] (top hidden activations) is given.
 * Pointer arrays themselves may be NULL where every entry would be. */
int nav_mlp_backward(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* const* dy,
                     int32_t ld_dy, const uint16_t* const* masks, const float* in, int32_t ld_in,
                     int32_t in_col, const float* const* h_top, float* const* dz,
                     uint32_t save_mask, float* const* dx, float* const* edge_slabs,
                     void* stream);
/* Hidden x hidden weight gradients dW_L = dz_L^T h_{L-1} of 1 or 2 networks (one launch) as
 * `splits` partial slabs slabs[i] [splits][nav_mlp_hidden_count] (rows of split s =
 * [s*P, (s+1)*P), P = ceil(M/splits) rounded up to 64). h_0 is recomputed from `in`,
 * dz_{n_hidden-1} from dy[i] and masks[i]; acts[i] / dz[i] (saved layers 1 .. n_hidden-2) are
 * read only for n_hidden > 2. Any splits >= 1 is valid; nav_mlp_wgrad_splits gives the count
 * that fills the chip (one tile workgroup per CU; the tile is 128 x 64 for d_out = 1 at
 * n_hidden = 2 and hidden_pad % 128 == 0, else 64 x 64). */
int32_t nav_mlp_wgrad_splits(int32_t n_nets, int32_t d_out, int32_t hidden_pad, int32_t n_hidden,
                             int64_t M);
int nav_mlp_wgrad(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                  int32_t ld_in, int32_t in_col, const float* const* acts,
                  const float* const* dz, const float* const* dy, int32_t ld_dy,
                  const uint16_t* const* masks, float* const* slabs, int32_t splits,
                  void* stream);
/* grad [param_count] = sum of the hidden slabs (hidden weights) and of the edge slabs (the rest),
 * in a fixed order. */
int nav_grad_reduce(const nav_mlp* net, const float* hidden_slabs, int32_t splits,
                    const float* edge_slabs, int64_t edge_blocks, float* grad, void* stream);
/* nav_grad_reduce fused with the Adam step (robot.py:236-239, as nav_adam) of 1 or 2 networks in
 * one launch: per net i the reduced gradient (also stored to grads[i] when grads and grads[i]
 * are non-NULL) updates nets[i].params with moments m[i], v[i], step_size[i] =
 * lr/(1-b1^t), bc2_sqrt[i] = sqrt(1-b2^t) (host arrays); refreshes packed. */
int nav_grad_reduce_adam(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                         int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                         float* const* grads, float* const* m, float* const* v, float beta1,
                         float beta2, float eps, const float* step_size, const float* bc2_sqrt,
                         void* stream);
/* nav_grad_reduce_adam plus the soft updates of robot.py:283-285 in the same launch: each net's
 * target net_targets[i] <- target*(1-tau) + p_new*tau right after p's Adam step (same thread), and
 * n_pairs (<= 4) further (target, source) pairs whose sources are final (the critics on a policy
 * epoch) by extra blocks; bit-identical to nav_grad_reduce_adam followed by nav_polyak_multi. */
int nav_grad_reduce_adam_polyak(const nav_mlp* nets, int32_t n_nets,
                                const float* const* hidden_slabs, int32_t splits,
                                const float* const* edge_slabs, int64_t edge_blocks,
                                float* const* grads, float* const* m, float* const* v,
                                float beta1, float beta2, float eps, const float* step_size,
                                const float* bc2_sqrt, const nav_mlp* net_targets,
                                const nav_mlp* targets, const nav_mlp* sources, int32_t n_pairs,
                                float tau, void* stream);
/* nav_grad_reduce of 1 or 2 same-shape networks in one launch (the twin critics' gradients into
 * one contiguous bucket for the shared-policy all-reduce). */
int nav_grad_reduce_multi(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                          int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                          float* const* grads, void* stream);
/* nav_adam of 1 or 2 networks in one launch on gradients g / grad_div (shared policy, BASELINE
 * config 5: the bucket holds the SUM over ranks after the all-reduce, grad_div = world size, as
 * torch DDP's averaging; grad_div 1 = the plain step, bit-identical to nav_adam). step_size and
 * bc2_sqrt are host arrays [n_nets]. */
int nav_adam_multi(const nav_mlp* nets, int32_t n_nets, const float* const* grads,
                   float* const* m, float* const* v, float beta1, float beta2, float eps,
                   const float* step_size, const float* bc2_sqrt, float grad_div, void* stream);
/* nav_adam_multi + a policy epoch's soft updates (robot.py:283-285) in the same launch: each net's
 * own target net_targets[i] follows its stepped parameters, and the n_pairs (targets[i],
 * sources[i]) pairs (sources not stepped by this call) run beside them — the shared-policy
 * counterpart of nav_grad_reduce_adam_polyak; every written `packed` is rebuilt. */
int nav_adam_polyak_multi(const nav_mlp* nets, int32_t n_nets, const float* const* grads,
                          float* const* m, float* const* v, float beta1, float beta2, float eps,
                          const float* step_size, const float* bc2_sqrt, float grad_div,
                          const nav_mlp* net_targets, const nav_mlp* targets,
                          const nav_mlp* sources, int32_t n_pairs, float tau, void* stream);
/* torch.optim.Adam step (robot.py:236-239; torch 2.10 single-tensor semantics) on a flat buffer,
 * step_size = lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t) precomputed by the caller; refreshes `packed`
 * of `net` (net->params must equal params). */
int nav_adam(const nav_mlp* net, const float* grad, float* m, float* v, float beta1, float beta2,
             float eps, float step_size, float bc2_sqrt, void* stream);
/* robot.py:293-310 soft update target <- target*(1-tau) + source*tau, refreshing target packed. */
int nav_polyak(const nav_mlp* target, const nav_mlp* source, float tau, void* stream);
/* The same for n <= 4 (target, source) pairs in one launch (TD3.soft_update x 3, robot.py:283-285). */
int nav_polyak_multi(const nav_mlp* targets, const nav_mlp* sources, int32_t n, float tau,
                     void* stream);
/* rebuild `packed` from `params` (after a host-side weight load). */
int nav_mlp_pack(const nav_mlp* net, void* stream);

/* ---- TD3 glue (robot.py:312-398) ---- */
/* ReplayBuffer.sample (robot.py:98-115): batch[b] = rows[idx[b]] with idx from `idx` if given,
 * else uniform with replacement over [0, size) from Philox (NAV_TAG_SAMPLE, counter). */
int nav_replay_sample(const nav_replay* replay, int64_t size, int64_t B, const int64_t* idx,
                      uint32_t seed_lo, uint32_t seed_hi, uint32_t counter, float* batch,
                      void* stream);
/* Fill / strided copy helpers of the TD3 glue (robot.py:329-339, 386-390). */
int nav_fill(float* x, int64_t n, float value, void* stream);
int nav_strided_copy(const float* src, int32_t ld_src, int32_t col_src, float* dst, int32_t ld_dst,
                     int32_t col_dst, int64_t rows, int32_t cols, void* stream);

/* ---- kernel timing (measurement only, not on the reference's interface) ----
 * Timing events recorded with a device-scope release (hipEventReleaseToDevice): bracketing a
 * launch costs no system-scope L2 writeback, so timing the bench's timed region does not stretch
 * it (a default torch/HIP event costs ~6 us of GPU time per record on MI355X). */
int nav_event_create(void** event);
int nav_event_destroy(void* event);
int nav_event_record(void* event, void* stream);
/* waits for `end`, then *ms = end - start */
int nav_event_elapsed_ms(void* start, void* end, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* NAVENV_H */
