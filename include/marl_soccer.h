/*
 * marl_soccer.h — C-ABI of the MI355X-native batched 2v2 soccer environment.
 *
 * This is the drop-in boundary for the reference's env.step() hot path.
 * Every entry point below replaces a piece of the reference's Python/FFI stack:
 *
 *   ms_create / ms_destroy   <- SoccerEnv.__init__ x N + SyncMultiAgentVecEnv.__init__
 *                               (soccer_simulation/soccer_env.py:19-73, marl_vecenv.py:8-16,
 *                                game/game.py:11-43 incl. pymunk.Space() construction)
 *   ms_reset                 <- SyncMultiAgentVecEnv.reset (marl_vecenv.py:18-28)
 *                               -> SoccerEnv.reset (soccer_env.py:81-98)
 *                               -> Game.reset (game/game.py:76-118)
 *   ms_step                  <- SyncMultiAgentVecEnv.step (marl_vecenv.py:30-68)
 *                               -> SoccerEnv.step (soccer_env.py:100-154)
 *                               -> Game.step (game/game.py:378-437)
 *                               -> pymunk.Space.step(1/60) -> cpSpaceStep (Chipmunk2D, cffi)
 *                                  with the entities.py:19-28 / :69-77 velocity callbacks
 *   ms_step_ring /           <- the same step / reset with the stacked observation kept as a
 *   ms_reset_ring               window into a per-agent frame ring (opt-in; the frame-stack
 *                               deque of soccer_env.py:130-140 without re-writing old frames)
 *   ms_observe               <- Game._get_observations (game/game.py:258-322)
 *   ms_seed_pcg64            <- np.random.default_rng(seed) (game/game.py:81-85): numpy
 *                               SeedSequence -> PCG64 state, restated so a C caller can seed
 *                               exactly like the reference
 *   ms_export/import_state   <- (no reference equivalent: the reference has no env
 *                               save/restore; used for parity tests and checkpointing)
 *   ms_debug_rewards         <- Game._update_reward_state + Game._calculate_rewards
 *                               (game/game.py:251-256, 324-375) evaluated on given states;
 *                               a test hook for the golden reward vectors
 *   ms_last_error            <- the ValueError messages of soccer_env.py:101-117
 *
 * Conventions
 *   - Every bulk array argument is a DEVICE pointer (hipMalloc'd or a torch tensor's
 *     data_ptr()), owned by the caller. The library owns the per-env state.
 *   - All calls are asynchronous on the handle's HIP stream (ms_create's `stream`,
 *     NULL = the device's null stream); synchronise that stream before reading outputs
 *     on the host. Calls on one handle must be serialised by the caller.
 *   - Return value: MS_OK (0) or a non-zero ms_status; ms_last_error() gives a
 *     thread-local message.
 *   - Agents are ordered agent_0..agent_3 (blue, blue, red, red), as
 *     SoccerEnv.possible_agents (soccer_env.py:29). The ball is body index 4.
 *
 * Layouts (row-major, C order)
 *   actions  float32 [N][4][3]   normalised in [-1,1]: (force_x, force_y, torque) in the
 *                                agent's local frame (soccer_env.py:119-125, game.py:390-397)
 *   obs      float32 [N][4][66]  3 stacked 22-float frames, oldest first (soccer_env.py:130-140)
 *   rew      float32 [N][4]      agents 2,3 always 0 (soccer_env.py:141-146)
 *   term     uint8   [N][4]      always 0 (soccer_env.py:147)
 *   trunc    uint8   [N][4]      1 on the episode's last step (soccer_env.py:148)
 *   goal     int8    [N]         0 none, 1 blue scored, 2 red scored (game.py:407-418)
 *   score    int32   [N][2]      (blue, red) after this step (game.py:415)
 */
#ifndef MARL_SOCCER_H
#define MARL_SOCCER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MS_ABI_VERSION 5

#define MS_N_AGENTS 4
#define MS_N_BODIES 5 /* 4 agents + ball */
#define MS_ACTION_DIM 3
#define MS_FRAME_SIZE 22
#define MS_STACK 3
#define MS_OBS_DIM (MS_FRAME_SIZE * MS_STACK) /* 66 */

/* Capacity of the per-env arbiter (contact-pair) cache and of the per-step active
 * arbiter list. 48 shape pairs exist (6 agent-agent, 4 agent-ball, 32 agent-static,
 * 6 ball-wall); geometry bounds the simultaneously touching ones far below this.
 * Overflow is counted in ms_stats.arbiter_overflow (tests assert it stays 0). */
#define MS_MAX_ARBITERS 32
#define MS_N_PAIRS 48

typedef enum ms_status {
  MS_OK = 0,
  MS_ERR_INVALID_ARGUMENT = 1,
  MS_ERR_HIP = 2,
  MS_ERR_OUT_OF_MEMORY = 3,
  MS_ERR_NONFINITE_ACTION = 4,
  MS_ERR_NO_DEVICE = 5
} ms_status;

/* Spawn modes of Game.reset / Game._reset_positions (game.py:109-127). */
typedef enum ms_spawn_mode {
  MS_SPAWN_RANDOM = 0,      /* _apply_random_positions      game.py:154-190 (default) */
  MS_SPAWN_FULL_RANDOM = 1, /* _apply_full_random_positions game.py:192-249 */
  MS_SPAWN_FIXED = 2        /* _apply_fixed_positions       game.py:129-152 */
} ms_spawn_mode;

/* Mirrors config.json (soccer_simulation/config.json:2-21) plus the code defaults the
 * reference reads with .get(...) (soccer_env.py:63-64, game.py:262-264, 330, 430) and the
 * constants hard-coded in entities.py:11,31-32,62,80-81. Values are converted to fp32
 * by ms_create. */
typedef struct ms_config {
  /* physics */
  double max_velocity;         /* 200      config.json:3 */
  double agent_mass;           /* 10       config.json:4 */
  double ball_mass;            /* 1        config.json:5 */
  double agent_moment;         /* 100      entities.py:11 */
  double ball_moment;          /* 10       entities.py:62 */
  double agent_friction;       /* 0.99     config.json:6 (per-tick velocity damping) */
  double ball_friction;        /* 0.97     config.json:7 */
  double agent_elasticity;     /* 0.2      entities.py:31 */
  double agent_surface_friction; /* 0.8    entities.py:32 */
  double ball_elasticity;      /* 0.95     entities.py:80 */
  double ball_surface_friction;  /* 0.2    entities.py:81 */
  double action_force_max;     /* 150000   soccer_env.py:63 default */
  double action_torque_max;    /* 1000     config.json:8 */
  double max_angular_velocity; /* torque_max/100  game.py:264 (obs scaling only) */
  /* rewards (config.json:10-18) */
  double ball_proximity_multiplier;   /* 0.002 */
  double move_ball_to_goal_multiplier;/* 0.1 */
  double alive_penalty;               /* 1e-5 */
  double goal_scored_reward;          /* 4.0 */
  double goal_conceded_penalty;       /* 0.0 */
  double score_difference_multiplier; /* 0.0 (code default 5.0, game.py:430) */
  /* simulation */
  int32_t max_steps; /* 1000  config.json:20; <=0 disables truncation (game.py:426) */
  /* 1: SyncMultiAgentVecEnv semantics — a finished env is reset inside ms_step with
   *    the full-random spawn and its returned obs is the reset obs (marl_vecenv.py:45-53).
   * 0: SoccerEnv semantics — the caller resets (soccer_env.py:151-152). */
  int32_t autoreset;
} ms_config;

/* Per-env state record (host/device exchange format, fp32 like the device state). */
typedef struct ms_body_state {
  float px, py;   /* position */
  float vx, vy;   /* velocity */
  float angle;    /* agents only; the ball's angle is unobservable and kept at 0 */
  float w;        /* angular velocity */
  float vbx, vby; /* Chipmunk bias velocity (penetration recovery), consumed next tick */
  float wb;       /* bias angular velocity */
} ms_body_state;

typedef struct ms_arbiter_state {
  uint8_t pair;    /* shape-pair id, 0..47 (DESIGN.md "pair table") */
  uint8_t count;   /* contacts 0..2 */
  uint8_t idle;    /* steps since last touched (0 = touched this step); dropped at 3 */
  uint8_t pad0;
  uint8_t hash[2]; /* contact feature ids used to carry impulses across steps */
  uint8_t pad1[2];
  float jn[2];     /* accumulated normal impulse */
  float jt[2];     /* accumulated tangent impulse */
} ms_arbiter_state;

/* Obs history is kept as state snapshots: the 22-float frame of every agent is a pure
 * function of these 26 values (Game._get_observations, game.py:258-322), so the frames of
 * t-2 and t-1 are recomputed bit-identically instead of being stored. */
#define MS_SNAP_SIZE 26 /* px[5], py[5], vx[4], vy[4], angle[4], w[4] (agents 0..3, ball 4) */

typedef struct ms_env_state {
  ms_body_state body[MS_N_BODIES];
  float snap[2][MS_SNAP_SIZE]; /* obs history snapshots: [0] = t-2, [1] = t-1 */
  int32_t steps;
  int32_t score_blue;
  int32_t score_red;
  uint8_t mode;       /* ms_spawn_mode used by goal soft-resets */
  uint8_t hist_empty; /* 1 until the first reset: next step stacks 3 copies (soccer_env.py:134-135) */
  uint8_t n_arb;
  uint8_t has_uint32; /* numpy PCG64 buffered 32-bit half */
  uint32_t uinteger;
  uint32_t pad;
  uint64_t pcg_state_hi, pcg_state_lo; /* numpy PCG64 128-bit LCG state */
  uint64_t pcg_inc_hi, pcg_inc_lo;     /* numpy PCG64 128-bit increment */
  ms_arbiter_state arb[MS_MAX_ARBITERS];
} ms_env_state;

typedef struct ms_stats {
  uint64_t arbiter_overflow;  /* arbiters dropped because MS_MAX_ARBITERS was full */
  uint64_t nonfinite_envs;    /* env-steps skipped because an action was not finite */
  int64_t first_nonfinite_env;/* lowest env index with a non-finite action, -1 if none */
  /* Since the last ms_reset_stats, counted inside ms_step, ms_step_n and ms_step_ring (ABI 2): env-steps
   * taken, and the arbiter-cache entries they read (the previous step's cache) and wrote (this
   * step's), i.e. the warm-start cache traffic of the algorithmic byte count (20 B per entry).
   * Kept as 64-bit counts per 64-env block on the device: they do not wrap within a run. */
  uint64_t env_steps;
  uint64_t cache_entries_read;
  uint64_t cache_entries_written;
} ms_stats;

typedef struct ms_env ms_env;

/* Fill `cfg` with the reference defaults (config.json + code defaults). */
void ms_config_default(ms_config *cfg);

/* Which step-kernel specialisation `cfg` selects: 1 = the reference's default physics and
 * rewards as compile-time constants (config.json; only max_steps and autoreset may differ),
 * 2 = the default physics as constants with the reward multipliers from the kernel arguments
 * (lane-pair and lane-group kernels; the one-lane and frame-ring kernels run generic for it),
 * 0 = the generic kernel (every parameter from the kernel arguments); negative on error.
 * Every kernel computes the same results. Host-only, no device needed. */
int ms_config_specialised(const ms_config *cfg);

/* Allocate device state for `n_envs` environments on HIP device `device`; launches
 * go to `stream` (a hipStream_t; NULL = null stream). The envs start reset with
 * OS-entropy seeds and the default random spawn, as Game.__init__ -> reset() does
 * (game.py:17, 74); their next step stacks three copies of its frame. */
int ms_create(const ms_config *cfg, int64_t n_envs, int device, void *stream, ms_env **out);
int ms_destroy(ms_env *env);
int ms_set_stream(ms_env *env, void *stream);
int64_t ms_num_envs(const ms_env *env);

/* numpy SeedSequence(entropy) -> PCG64: writes {state_hi, state_lo, inc_hi, inc_lo}.
 * `entropy` holds the seed as little-endian 32-bit words (numpy's
 * _coerce_to_uint32_array), n_words >= 1. Host-only, no device needed. */
int ms_seed_pcg64(const uint32_t *entropy, int n_words, uint64_t out[4]);
/* Same for seeds seed0 + i, i < n (SyncMultiAgentVecEnv seeds env i with seed+i,
 * marl_vecenv.py:23); seed0 + i must be >= 0. Writes out[i*4 .. i*4+3]. Host memory. */
int ms_seed_pcg64_range(uint64_t seed0, int64_t n, uint64_t *out);

/* Episode reset (Game.reset). `pcg`: device uint64 [N][4] new RNG states or NULL to
 * continue each env's stream (reset(seed=None)). `env_mask`: device uint8 [N], non-zero
 * = reset this env, or NULL = all. `mode`: ms_spawn_mode, also stored for later goal
 * soft-resets. `obs`: device float [N][4][66] receives 3 stacked copies of the reset
 * frame for reset envs (others untouched), or NULL. */
int ms_reset(ms_env *env, const uint64_t *pcg, const uint8_t *env_mask, int mode, float *obs);

/* One env.step for every env (see layouts above). obs must be non-NULL; rew, term,
 * trunc, goal, score may be NULL (not written). An env whose actions contain a
 * non-finite value is not stepped (SoccerEnv.step raises ValueError there, soccer_env.py:116-117);
 * it is counted in ms_stats (read with ms_get_stats, which synchronises) and its outputs get
 * defined values (ABI 5): obs all NaN, rew (NaN, NaN, 0, 0), term / trunc / goal 0, score the
 * env's current score. */
int ms_step(ms_env *env, const float *actions, float *obs, float *rew, uint8_t *term,
            uint8_t *trunc, int8_t *goal, int32_t *score);

/* K consecutive ms_step calls with actions given up front (open loop: a random-action or
 * scripted rollout, the workload of marl_vecenv.py:30-68 driven by pre-drawn actions) (ABI 4).
 * actions [K][N][4][3]; every output with a leading K dimension: obs [K][N][4][66],
 * rew [K][N][4], term / trunc [K][N][4], goal [K][N], score [K][N][2] (NULL: not written; obs
 * required). Results are those of K ms_step calls, bit for bit. With the lane-pair and the
 * lane-group kernels (ms_set_lane_group 2, 8, 16: the defaults) the K steps run in ONE launch,
 * each wave stepping its envs K times back to back (a wave slowed by a pile-up in one step no
 * longer holds the whole grid at every step boundary); the one-lane-per-env kernel (lanes 0)
 * issues K ms_step launches. An env whose actions at step k are not all finite is skipped for
 * that step exactly as ms_step skips it: counted in ms_stats, and its step-k outputs take
 * ms_step's defined values for a skipped env-step (NaN obs and rewards, term / trunc / goal 0, the
 * current score).
 * 1 <= K, alignment as ms_step; MS_ERR_INVALID_ARGUMENT otherwise. */
int ms_step_n(ms_env *env, int K, const float *actions, float *obs, float *rew, uint8_t *term,
              uint8_t *trunc, int8_t *goal, int32_t *score);

/* ms_step's kernel by lanes per env (replaces the serial per-env loop of marl_vecenv.py:39).
 * lanes = 8 or 16: a group of that many lanes steps each env (a wave holds 64 / lanes envs),
 * spreading loads, per-body work, the broadphase, the narrowphase, prestep, cache writes and the
 * observation frames over the group (small batches that leave most SIMDs idle at one lane per
 * env). lanes = 2: a lane pair per env (32 envs per wave), each lane holding half of the env's
 * working set, so the kernel fits 256 registers and two waves share each SIMD (batches that fill
 * the SIMDs). lanes = 0: one lane per env. Same results bit for bit. lanes < 0: automatic, which
 * is ms_create's default (ms_step_kernel_name names the kernel it picked). Host-only. */
int ms_set_lane_group(ms_env *env, int lanes);
int ms_get_lane_group(const ms_env *env);

/* The lane-group kernel's contact-solve schedule (Chipmunk's 10 Gauss-Seidel passes of
 * cpSpaceStep, cpSpaceStep.c's solver loop, restated by oracle/soccer_oracle.c): mode 0
 * (ms_create's default) picks per wave, 1 always solves each env's contacts in canonical order on
 * two lanes (velocity and bias halves), 2 solves them in rounds by dependency level wherever the
 * level schedule covers every env of the wave. Same results bit for bit in every mode; modes 1 and
 * 2 exist so each path can be tested on its own. Host-only. */
int ms_set_group_solve(ms_env *env, int mode);
int ms_get_group_solve(const ms_env *env);

/* Name of the kernel the next ms_step launches for this handle's batch size and launch shape
 * ("ms_step_kernel", "ms_step_group_kernel" or "ms_step_pair_kernel"; ms_step_n runs the
 * matching "_n" kernel), as rocprofv3 lists it
 * (without template arguments): what bench.py's roofline line and its PMC lookup are keyed on.
 * Host-only; "" for a null handle. */
const char *ms_step_kernel_name(const ms_env *env);

/* Frame-ring observations (opt-in; replaces the deque of 3 frames of soccer_env.py:130-140
 * and marl_vecenv.py:30-68 with a window into a longer per-agent ring, so a step writes one
 * frame instead of three). `frames`: device float [N][4][R][22], 16-B aligned, R even >= 4.
 * The step's stacked observation of env e, agent a is frames[e][a][pos .. pos+2] (t-2, t-1,
 * t): 66 contiguous floats, row stride R*22. ms_step_ring writes frame t at pos+2; with
 * wrap = 1 it also writes t-2 and t-1 at pos, pos+1 (use when the window moves back to the
 * start of the ring); with wrap = 0 the caller guarantees slots pos, pos+1 hold the previous
 * two steps' frames t (window advanced by one). Envs that are reset (auto-reset, or the
 * first step after ms_create) get 3 copies of the reset frame, as ms_step. Otherwise as
 * ms_step (obs replaced by the ring). 0 <= pos <= R-3, else MS_ERR_INVALID_ARGUMENT. */
int ms_step_ring(ms_env *env, const float *actions, float *frames, int R, int pos, int wrap,
                 float *rew, uint8_t *term, uint8_t *trunc, int8_t *goal, int32_t *score);

/* ms_reset writing the 3 stacked copies of the reset frame into ring slots pos..pos+2. */
int ms_reset_ring(ms_env *env, const uint64_t *pcg, const uint8_t *env_mask, int mode,
                  float *frames, int R, int pos);

/* Current frame of every agent (Game._get_observations), device float [N][4][22]. */
int ms_observe(ms_env *env, float *frames);

/* State exchange: device ms_env_state [N]. */
int ms_export_state(ms_env *env, ms_env_state *dst);
int ms_import_state(ms_env *env, const ms_env_state *src);

/* Reward shaping on given states, device arrays: prev_pos/cur_pos float [N][5][2]
 * (bodies 0..4), goal int8 [N], terminal uint8 [N], score int32 [N][2]; writes
 * rew float [N][2] (agent_0, agent_1). Same device code as ms_step. */
int ms_debug_rewards(ms_env *env, const float *prev_pos, const float *cur_pos,
                     const int8_t *goal, const uint8_t *terminal, const int32_t *score,
                     float *rew);

/* ---- policy forward (the env's immediate caller: SURVEY.md §8(f) rank 1) -------------------
 * ms_policy_forward <- the reference rollout's per-step policy evaluation (marl-soccer.ipynb
 * train cell L299-313; eval.py:69-81): RunningMeanStd normalisation of the blue agents' obs
 * (clip((x - mean) / (sqrt(var) + 1e-8), -10, 10) in float64, then float32) followed by the
 * notebook Agent's two tanh MLPs 66-512-256-128-64-{3, 1} (actor mean, critic value;
 * eval.py:17-47), fused in one gfx950 kernel (f32-input MFMA, activations in registers).
 *   x: device float rows of 66; row r at x + (r / group_rows) * group_stride +
 *      (r % group_rows) * row_stride floats (the blue agents of an (N, 4, 66) obs buffer:
 *      rows 2N, group_rows 2, group_stride 264, row_stride 66).
 *   mean, den: device float64 [66]: the normaliser's mean and sqrt(var) + 1e-8, or both NULL
 *      for rows that are normalised already.
 *   actor, critic: device packed nets (MS_POLICY_NET_FLOATS floats each, 16-B aligned; the
 *      layout is marlsoccer/policy.py pack_net's; either may be NULL to skip that net).
 *   act_mean: device float [rows][3]; value: device float [rows]. Asynchronous on `stream`. */
#define MS_POLICY_NET_FLOATS 211936
int ms_policy_forward(const float *x, int64_t rows, int group_rows, int64_t group_stride, int64_t row_stride,
                      const double *mean, const double *den, const float *actor, const float *critic,
                      float *act_mean, float *value, void *stream);
const char *ms_policy_last_error(void);

/* The same kernel with every output of one rollout step (marlsoccer.rollout.DeviceRollout;
 * the notebook's rollout L299-313): NULL pointers are not written. Row r as above; outputs
 * per row: act_mean [rows][3], value [rows]; action [rows][3] = eps * exp(logstd) + mean when
 * eps (device standard-normal draws [rows][3]) is given (Agent.sample), else the mean;
 * logprob [rows] = its Normal log-prob summed over the 3 components (0 without eps);
 * obs_copy [rows][66] the raw input rows; env_actions [rows / 2][4][3]: row r's action at
 * env r / 2, agent r % 2 (the blue agents of the env's action buffer; rows even), and with
 * red_uniform (device uniform [0, 1) draws [rows][3]) 2u - 1 at env r / 2, agent 2 + r % 2. */
typedef struct ms_policy_io {
  const float *obs;
  int64_t rows;
  int32_t group_rows;
  int32_t pad0;
  int64_t group_stride, row_stride;
  const double *mean, *den;
  const float *actor, *critic;
  const float *logstd, *eps;
  float *act_mean, *action, *logprob, *value, *obs_copy, *env_actions;
  const float *red_uniform;
} ms_policy_io;
int ms_policy_run(const ms_policy_io *io, void *stream);

/* A rollout step's bookkeeping from ms_step's outputs in one launch (marlsoccer.rollout.
 * DeviceRollout; the notebook's rollout L313-336, PPO storage of the two blue agents): for env
 * i < n_envs and agent a < 2, rewards[i][a] = rew[i][a] and next_done[i][a] = 1.0f if
 * term[i][a] | trunc[i][a] else 0.0f (also into dones_next[i][a] when non-NULL: the next
 * step's row of the dones storage); every env with trunc[i][0] adds 1 to *episodes and
 * score[i][0..1] to score_sum[0..1] (int64, device). All pointers device memory. */
int ms_rollout_record(int64_t n_envs, const float *rew, const uint8_t *term, const uint8_t *trunc,
                      const int32_t *score, float *rewards, float *next_done, float *dones_next,
                      int64_t *episodes, int64_t *score_sum, void *stream);

/* Synchronises the stream and reads the device counters. */
int ms_get_stats(ms_env *env, ms_stats *out);
int ms_reset_stats(ms_env *env);

const char *ms_last_error(void);
int ms_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MARL_SOCCER_H */
