/* g2048.h -- C ABI of the MI355X-native batched 2048 environment + replay ring.
 *
 * The drop-in boundary for the reference's hot path (ribal-aladeeb/reinforcement-learning-2048).
 * The reference has no FFI: its seams are Python callables operating on ONE Board2048 at a
 * time.  Each entry point below cites the reference interface it replaces; the Python mirror
 * (reinforcement-learning-2048_amd/g2048/dqn_lib.py) binds these through ctypes with the
 * reference's own function names.  See INTEGRATION.md for the bindings.
 *
 * Conventions
 *  - Boards are 16 log2 exponents (u8, 0 = empty), row-major: cell(r, c) = 4r + c.  This is
 *    exactly Board2048.log_scale() (src/board.py:224-231) of the reference's int64 values.
 *  - Actions: 0 = up, 1 = down, 2 = left, 3 = right (src/board.py:191, :129).
 *  - Legal masks: bit a set iff move a changes the board (src/board.py:128-135).
 *  - Every call returns 0 (G2048_OK) or a negative g2048_status; nothing throws across the ABI;
 *    g2048_last_error() returns a thread-local message for the last failure.
 *  - Every pointer named *dev* / every buffer argument is DEVICE memory on the env's device,
 *    owned by the caller unless the object was made by *_create (library-owned).
 *  - All step / sample calls are stream-ordered and asynchronous (no host sync, no allocation),
 *    so they may be captured into a hipGraph.  `stream` is a hipStream_t (NULL = default).
 *  - One env per stream; distinct envs are thread-safe, concurrent calls on one env are not.
 *  - Randomness is counter-based Philox4x32-10.  Board g (global id = board_offset + i) owns
 *    rocRAND philox4x32_10 subsequence g: its step draw at step t is the 4-word block
 *    rocrand_init(seed, g, 4t) would return first (domain bits 30-31 of the subsequence word
 *    select step / random-policy / explicit-reset / sampler draws).  No per-lane RNG state in
 *    HBM: the counter t is the env's step clock (one u64 per 64 boards).
 *  - The random policy (actions == NULL, g2048_env_rollout), ABI v3: step t takes ONE word
 *    w = word (t & 3) of block t >> 2 of the random-policy domain (a block per four steps).
 *    Action w >> 30; a 4 spawns iff bit 29 is set (p = 0.5, src/board.py:12,49); the spawn cell
 *    is the k-th empty cell of the slid board, k = floor((w << 3) * n / 2^32), in move-space
 *    line-major order (up/down: column j = 0..3, then rows from the top / bottom; left/right:
 *    row j, then columns from the left / right) -- uniform over the empty cells like the
 *    reference's np.random.choice.  A terminal step's auto-reset: a tile at cell (w >> 26) & 15
 *    (a 4 iff bit 25), one at the k2-th of the other 15 cells in row-major order,
 *    k2 = floor((w << 8) * 15 / 2^32) (a 4 iff bit 24).  With G2048_P4_10 the values come from
 *    word t & 3 of the blocks at counters (t >> 2) | 2^63 (spawn, first reset tile) and
 *    (t >> 2) | 2^62 (second reset tile): a 4 iff the word < round(0.1 * 2^32).
 *    (ABI v2 drew half a block per step and spawned in row-major order.)
 */
#ifndef G2048_H
#define G2048_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define G2048_ABI_VERSION 5

#ifndef G2048_API
#define G2048_API __attribute__((visibility("default")))
#endif

typedef enum {
    G2048_OK = 0,
    G2048_EINVAL = -1,   /* bad argument (size, null, dtype) */
    G2048_EHIP = -2,     /* HIP runtime error */
    G2048_ENOMEM = -3,
    G2048_EBADINPUT = -4 /* device-side input errors were counted (see g2048_env_error_count) */
} g2048_status;

typedef enum {
    G2048_P4_10 = 1u,         /* spawn a 4 with p = 0.1 (default: p = 0.5, src/board.py:12,49) */
    G2048_EGREEDY_FIXED = 2u, /* greedy over legal moves only / explore among legal moves;
                                 default reproduces src/dqn_lib.py:25-29 bit-for-bit (F5) */
    G2048_NO_AUTORESET = 4u   /* leave terminal boards in place (tests) */
} g2048_flags;

typedef enum { G2048_F32 = 0, G2048_F64 = 1 } g2048_dtype;

typedef struct g2048_env g2048_env;
typedef struct g2048_replay g2048_replay;

/* One finished episode (the Experiment.add_episode fields, src/experiments.py:112-122).  40 B.
 * mean reward = score / moves (the rewards of an episode sum to its merge score);
 * q_value = q_sum / moves (max_a Q per step, 0 on explore / non-greedy steps, src/dqn_lib.py:19,29);
 * epsilon follows from `episode` and the schedule. */
typedef struct {
    uint64_t step;     /* the board's step counter at its terminal step */
    double q_sum;      /* sum over the episode's steps of max_a Q(s) */
    uint32_t board;    /* global board id (board_offset + i) */
    uint32_t episode;  /* the board's episode index (0-based) */
    uint32_t score;    /* Board2048.merge_score() */
    uint32_t moves;    /* len(_action_history), including the terminal self-transition */
    uint32_t max_exp;  /* log2 of max(state) */
    uint32_t reserved;
} g2048_episode;

/* ---- environment -------------------------------------------------------------------------
 * State per board i: board u8[16]; meta u32[2][n] (two rows): meta[0][i] = score
 * (Board2048._mergescore), meta[1][i] = start = the step clock (low 32 bits) at which the running
 * episode began, so moves = len(_action_history) = (uint32_t)(clock - start) is derived, not
 * stored (ABI v5; v4 held {score, moves} per board, a read-modify-write of both every step --
 * g2048_env_score_moves writes that pair layout); ep u32[4] = {episodes finished, last score,
 * last moves, last max exponent} (the Experiment.add_episode fields, src/experiments.py:112-122).  Per group of 64 boards (boards 64g .. 64g+63): clock u64[g] =
 * the number of steps taken, i.e. the Philox counter of the next step and the replay row it
 * appends to.  Every step call advances every board, so all clocks of an env hold the same
 * value; each group is read and advanced only by the wavefront that steps its boards, so no
 * kernel needs a grid-wide barrier to advance it. */
#define G2048_CLOCK_GROUP 64
#define G2048_CLOCK_WORDS(n) (((n) + G2048_CLOCK_GROUP - 1) / G2048_CLOCK_GROUP)
/* Largest env: 2^31 - 256 boards (80 GB of board / meta / episode state).  A dispatch's grid is
 * at most 2^32 - 1 work-items per dimension, and the dense-64 fused step gives a board two
 * threads (the warp-specialised rollout does too, but its < 4 GiB ring window caps it lower). */
#define G2048_MAX_BOARDS ((int64_t)2147483392)

/* Replaces `Board2048()` x n_boards (src/board.py:10-20): allocates and resets n boards. */
G2048_API int g2048_env_create(g2048_env** out, int64_t n_boards, uint64_t seed, uint64_t board_offset,
                     int device_id, uint32_t flags, void* stream);
/* Same, over caller-owned device buffers board u8[n][16], meta u32[2][n], ep u32[n][4],
 * clock u64[G2048_CLOCK_WORDS(n)] (board/ep 16-byte, meta/clock 8-byte aligned).  If reset != 0
 * the boards are reset (2 spawns each), else left as given; the clock is used as given (all
 * words equal: zero for a fresh env). */
G2048_API int g2048_env_wrap(g2048_env** out, int64_t n_boards, uint64_t seed, uint64_t board_offset,
                   int device_id, uint32_t flags, uint8_t* board_dev, uint32_t* meta_dev,
                   uint32_t* ep_dev, uint64_t* clock_dev, int reset, void* stream);
G2048_API void g2048_env_destroy(g2048_env* env);
/* Device views of the env state (library-owned or wrapped); any out-pointer may be NULL. */
G2048_API int g2048_env_views(g2048_env* env, uint8_t** board_dev, uint32_t** meta_dev,
                              uint32_t** ep_dev, uint64_t** clock_dev);
G2048_API int64_t g2048_env_size(const g2048_env* env);

/* {score, moves} of every board as u32[n][2] (out_dev 8-byte aligned): Board2048.merge_score()
 * (src/board.py:207) and len(_action_history) (src/experiments.py:112-122 number_moves), from meta
 * and the clock -- the v4 meta layout, for hosts that read it. */
G2048_API int g2048_env_score_moves(g2048_env* env, uint32_t* out_dev, void* stream);

/* Re-deal fresh boards (2 spawns, src/board.py:18-20) where reset_mask_dev[i] != 0 (all if NULL). */
G2048_API int g2048_env_reset(g2048_env* env, const uint8_t* reset_mask_dev, void* stream);

/* Explicit-reset epoch (host state of the env: the Philox counter of the next g2048_env_reset),
 * for checkpoint / resume. */
G2048_API int g2048_env_get_epoch(const g2048_env* env, uint32_t* epoch_out);
G2048_API int g2048_env_set_epoch(g2048_env* env, uint32_t epoch);

/* Attach (log_dev != NULL) or detach an episode log: on every later terminal step of any step /
 * rollout call, board i writes its episode e as a g2048_episode into slot i*S + (e % S) of
 * log_dev [n][S] (S = slots_per_board; no atomics, so the layout is deterministic).  A reader
 * that remembers each board's episode count (ep[i][0]) at its last read finds the new records
 * in those slots, as long as no board finished more than S episodes in between.
 * qsum_dev f64[n] holds each board's running max-Q sum (zero it before attaching).  With
 * G2048_NO_AUTORESET a board that stays terminal logs again on every step.  Replaces the
 * per-episode bookkeeping of training_loop (src/dqn_lib.py:184-213). */
G2048_API int g2048_env_set_episode_log(g2048_env* env, g2048_episode* log_dev,
                                        int64_t slots_per_board, double* qsum_dev);

/* Legal-move mask of every current board: available_moves_as_torch_unit_vector
 * (src/board.py:128-135) as bits (bit a = move a changes the board). */
G2048_API int g2048_env_legal_mask(g2048_env* env, uint8_t* legal_dev, void* stream);

/* One env step of every board.  Replaces Board2048.peek_action (src/board.py:185-202) +
 * available_moves_as_torch_unit_vector (:128-135) + reward_func_merge_score
 * (src/dqn_lib.py:87-88) + the done test (src/dqn_lib.py:17-18).
 *  actions_dev  u8[n] (0..3) or NULL = uniform random action per board (np.random.randint(4)).
 *  reward_dev   i32[n] merge-score gain (0 for invalid / terminal moves), or NULL
 *  done_dev     u8[n]  1 iff the board had no legal move BEFORE this step, or NULL
 *  legal_dev    u8[n]  legal mask of the board before this step, or NULL
 *  rb           replay ring to append (s, a, r, s', done) to, or NULL (src/dqn_lib.py:106)
 * A terminal board records the self-transition (s, a, 0, s, 1) (F6) and is then re-dealt unless
 * G2048_NO_AUTORESET.  An action > 3 is counted as a device-side input error and is a no-op. */
G2048_API int g2048_env_step(g2048_env* env, const uint8_t* actions_dev, int32_t* reward_dev,
                   uint8_t* done_dev, uint8_t* legal_dev, g2048_replay* rb, void* stream);

/* Fused epsilon-greedy select + step + replay append: replaces play_one_step
 * (src/dqn_lib.py:91-107) with epsilon_greedy_policy (:16-30) for every board at once.
 *  q_dev      Q-values [n][4] of the current boards, dtype q_dtype (f32 or f64)
 *  eps_dev    f64 scalar on device (read at kernel time, graph-safe), or NULL -> use eps
 *  action_dev u8[n] chosen actions out, or NULL */
G2048_API int g2048_env_step_egreedy(g2048_env* env, const void* q_dev, int q_dtype, const double* eps_dev,
                           double eps, int32_t* reward_dev, uint8_t* done_dev,
                           uint8_t* action_dev, g2048_replay* rb, void* stream);

/* The same with the reference's per-episode schedule applied per board (src/dqn_lib.py:184-188):
 * eps_b = max((eps_decay_episodes - episodes_b) / eps_decay_episodes, eps_min), episodes_b = the
 * board's finished-episode count (ep[i][0]); graph-safe, no host input per step. */
G2048_API int g2048_env_step_egreedy_schedule(g2048_env* env, const void* q_dev, int q_dtype,
                                              double eps_decay_episodes, double eps_min,
                                              int32_t* reward_dev, uint8_t* done_dev,
                                              uint8_t* action_dev, g2048_replay* rb, void* stream);

/* Test entry: actions + injected spawns (cell index -1..15, exponent) instead of Philox draws,
 * so trajectories recorded from the reference replay bit-for-bit. */
G2048_API int g2048_env_step_inject(g2048_env* env, const uint8_t* actions_dev, const int8_t* spawn_idx_dev,
                          const uint8_t* spawn_exp_dev, int32_t* reward_dev, uint8_t* done_dev,
                          uint8_t* legal_dev, void* stream);

/* k_steps random-policy env steps per launch with the board held in registers (replay pre-fill,
 * env-only throughput).  Identical results to k_steps calls of g2048_env_step(actions=NULL).
 * reward_sum_dev (i64[n], accumulated, or NULL).  A step's transition is appended with five
 * stores whose per-step offset is a scalar (row * n), the board never leaves the VGPRs, and the
 * Philox block of a 4-step quad is drawn once. */
G2048_API int g2048_env_rollout(g2048_env* env, int32_t k_steps, g2048_replay* rb, int64_t* reward_sum_dev,
                      void* stream);

/* Device-side input errors counted since the last call (synchronises `stream`). */
G2048_API int g2048_env_error_count(g2048_env* env, int64_t* count_out, void* stream);

/* ---- replay ring (replaces the deque of (Board, a, r, Board, done), src/dqn_lib.py:172) ----
 * SoA in HBM: s u8[C][16], s2 u8[C][16], a u8[C], r i32[C], d u8[C], count u64 (valid rows).
 * The env appends board i of step t at row (t mod (C/n)) * n + i, so C must be a multiple of the
 * appending env's n.
 * g2048_replay_create carves the sections from one allocation in the order s | s2 | r | a | d |
 * count, each starting G2048_REPLAY_SECTION_PAD bytes past the 256-byte-aligned end of the one
 * before: without the pad, power-of-two capacities put the five concurrently written streams at
 * power-of-two distances, and the HBM channel hash served them from the same channels (4M boards
 * x 16 steps: 500-610 us per rollout launch against 436-450 us with the pad). */
#define G2048_REPLAY_SECTION_PAD 4352
G2048_API int g2048_replay_create(g2048_replay** out, int64_t capacity, int device_id, void* stream);
G2048_API int g2048_replay_wrap(g2048_replay** out, int64_t capacity, int device_id, uint8_t* s_dev,
                      uint8_t* s2_dev, uint8_t* a_dev, int32_t* r_dev, uint8_t* d_dev,
                      uint64_t* count_dev);
G2048_API void g2048_replay_destroy(g2048_replay* rb);
G2048_API int g2048_replay_views(g2048_replay* rb, uint8_t** s_dev, uint8_t** s2_dev, uint8_t** a_dev,
                       int32_t** r_dev, uint8_t** d_dev, uint64_t** count_dev);

/* sample_experiences + extract_samples_conv/_dense (src/dqn_lib.py:33-84) for a whole batch:
 * gather rows idx_dev[b] (i64[B]; NULL -> uniform with replacement over [0, count) from Philox
 * (seed, epoch, b)) and encode them.  s_out/s2_out: [B][16] of `dtype` (f32/f64; the conv view
 * [B,1,4,4] is the same memory), a_out i64[B], r_out/d_out [B] of `dtype`, idx_out i64[B] or
 * NULL.  Any of the outputs may be NULL. */
G2048_API int g2048_replay_sample_encode(g2048_replay* rb, const int64_t* idx_dev, int64_t batch,
                               uint64_t seed, uint64_t epoch, int dtype, void* s_out,
                               void* s2_out, int64_t* a_out, void* r_out, void* d_out,
                               int64_t* idx_out, void* stream);

/* ---- fused Q-network (learner fast path) -------------------------------------------------
 * Forward of the reference conv Q-net (src/configs/double_dqn_conv.py:19-28) for n boards in
 * one launch, fp32 on MFMA: Q[b] = net(log2 exponents of rows[idx ? idx[b] : b]).  Replaces
 * board_as_4d_tensor / extract_samples_conv + model(state) (src/dqn_lib.py:8-9,23-24,126-130).
 * Parameter pointers are device fp32 tensors in torch's layouts (Conv2d [out,in,kh,kw], Linear
 * [out,in]); rows u8[*][16]; q_out f32[n][4]. */
typedef struct {
    const float *w1, *b1;       /* Conv2d(1, 64, 2)   */
    const float *w2, *b2;       /* Conv2d(64, 64, 2)  */
    const float *fc1_w, *fc1_b; /* Linear(256, 64)    */
    const float *fc2_w, *fc2_b; /* Linear(64, 4)      */
} g2048_convnet_params;

G2048_API int g2048_convnet_forward(const g2048_convnet_params* params, const uint8_t* rows_dev,
                                    const int64_t* idx_dev, int64_t n, float* q_out_dev,
                                    void* stream);

/* The rollout forward restricted to the greedy branch: epsilon_greedy_policy evaluates the model
 * only when it does not explore (src/dqn_lib.py:20-24).  For every board of env the explore draw
 * of its next g2048_env_step_egreedy / _schedule step is repeated (same Philox block; eps as in
 * g2048_env_step_egreedy_dense64: eps_decay_episodes > 0 selects the per-board schedule, else
 * eps_dev (device f64) or eps), and q_out[b] (f32[n][4]) is written only for the boards that
 * will take the greedy branch -- bitwise the rows g2048_convnet_forward writes.  The other rows
 * are left as they are: the step does not read them.  Call it between the same two steps as
 * the forward it replaces, with the same eps arguments as the step. */
G2048_API int g2048_convnet_forward_greedy(const g2048_convnet_params* params, g2048_env* env,
                                           const double* eps_dev, double eps,
                                           double eps_decay_episodes, double eps_min,
                                           float* q_out_dev, void* stream);

/* Gradient of the graded half of train_step (src/dqn_lib.py:146-161) for the conv net, fp32:
 * q_b = Q(rows[idx[b]])[actions[idx[b]]], loss = sum_b (q_b - y_b)^2 (MSELoss(reduction='sum'))
 * and d loss / d params written to grad_out (f32[33476], torch parameter order and layouts --
 * the layout of a flat bucket of model.parameters()), loss to loss_out (f32 scalar, nullable).
 * workspace: f32[g2048_convnet_train_workspace(batch)] device scratch (partial-gradient slabs;
 * the final reduction is in a fixed order, so results are run-to-run deterministic).
 * step_dev (u64, nullable) is incremented once: the update counter that g2048_convnet_targets
 * (sampler epoch) and g2048_adam_step (bias correction) read -- graph-replay safe. */
G2048_API int64_t g2048_convnet_train_workspace(int64_t batch);
G2048_API int g2048_convnet_train_grad(const g2048_convnet_params* params,
                                       const uint8_t* rows_dev, const uint8_t* actions_dev,
                                       const int64_t* idx_dev, const float* y_dev, int64_t batch,
                                       float* workspace_dev, float* grad_out_dev,
                                       float* loss_out_dev, uint64_t* step_dev, void* stream);

/* g2048_convnet_train_grad with optimizer.step() folded into the gradient reduction (single
 * process; src/dqn_lib.py:146-163 in the intended zero_grad -> backward -> step order): the
 * same sums as train_grad, then Adam exactly as g2048_adam_step_sync (t = *step_dev after the
 * train launch's increment), applied in place to `params`; when sync_every > 0 and t is a
 * multiple of it, the updated parameters are also written to `target` (src/dqn_lib.py:227-228).
 * grad_out may be NULL (then only the parameters change).  2 launches per update. */
G2048_API int g2048_convnet_train_adam(const g2048_convnet_params* params,
                                       const uint8_t* rows_dev, const uint8_t* actions_dev,
                                       const int64_t* idx_dev, const float* y_dev, int64_t batch,
                                       float* workspace_dev, float* grad_out_dev,
                                       float* loss_out_dev, uint64_t* step_dev,
                                       float* exp_avg_dev, float* exp_avg_sq_dev, double lr,
                                       double beta1, double beta2, double eps,
                                       const g2048_convnet_params* target, uint64_t sync_every,
                                       void* stream);

/* Double-DQN targets for a minibatch in one launch (src/dqn_lib.py:67-68,125-132): indices
 * idx_out[b] = idx_in[b], or uniform over the ring's filled rows from Philox (seed, *epoch_dev)
 * -- the same draw as g2048_replay_sample_encode's; then y[b] = r + ((1 - d) * float32(gamma)) *
 * Q_target(s', argmax_a Q_online(s', a)) (vanilla DQN when double_dqn == 0: max_a Q_target). */
G2048_API int g2048_convnet_targets(const g2048_convnet_params* online,
                                    const g2048_convnet_params* target, g2048_replay* rb,
                                    const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                    const uint64_t* epoch_dev, float gamma, int double_dqn,
                                    int64_t* idx_out_dev, float* y_out_dev, void* stream);

/* One whole conv train_step (src/dqn_lib.py:119-164; + the target sync of :227-228): the
 * targets of g2048_convnet_targets and the gradient of g2048_convnet_train_grad on the sampled
 * rows, then -- when exp_avg / exp_avg_sq are given -- Adam applied in place as in
 * g2048_convnet_train_adam (grad_out may then be NULL); without them the summed gradient goes to
 * grad_out (a data-parallel all-reduce and g2048_adam_step follow).  step_dev is the sampler
 * epoch and Adam's t (incremented once).  y_out receives the Bellman targets.  For Double DQN
 * the targets launch splits its grid into an online-net half (a*) and a target-net half
 * (Q_target, r, discount), each staging one net, and the train launch forms y from them (the
 * same float as g2048_convnet_targets).  workspace: f32[g2048_convnet_train_workspace(batch)].
 * 4 launches per update. */
G2048_API int g2048_convnet_update(const g2048_convnet_params* online,
                                   const g2048_convnet_params* target, g2048_replay* rb,
                                   const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                   uint64_t* step_dev, float gamma, int double_dqn,
                                   int64_t* idx_out_dev, float* y_out_dev, float* workspace_dev,
                                   float* grad_out_dev, float* loss_out_dev, float* exp_avg_dev,
                                   float* exp_avg_sq_dev, double lr, double beta1, double beta2,
                                   double eps, uint64_t sync_every, void* stream);

/* One-launch Adam (torch.optim.Adam semantics, amsgrad off, no weight decay) over n_tensors
 * (<= 16) fp32 parameter tensors whose gradients are packed back to back in grad_dev; exp_avg /
 * exp_avg_sq are flat state buffers of the same length; the step t is read from *step_dev. */
G2048_API int g2048_adam_step(float* const* params_dev, const int64_t* numels, int n_tensors,
                              const float* grad_dev, float* exp_avg_dev, float* exp_avg_sq_dev,
                              const uint64_t* step_dev, double lr, double beta1, double beta2,
                              double eps, void* stream);
/* The same, plus the target-network sync of training_loop (src/dqn_lib.py:227-228) decided on
 * the device: when t % sync_every == 0, each updated parameter is also written to
 * target_params (same tensor shapes/order), so graph replays need no host decision. */
G2048_API int g2048_adam_step_sync(float* const* params_dev, const int64_t* numels, int n_tensors,
                                   const float* grad_dev, float* exp_avg_dev,
                                   float* exp_avg_sq_dev, const uint64_t* step_dev, double lr,
                                   double beta1, double beta2, double eps,
                                   float* const* target_params_dev, uint64_t sync_every,
                                   void* stream);
/* The same with the gradient read as g * grad_scale (> 0): the data-parallel step after a SUM
 * all-reduce of the gradient bucket (grad_scale = 1 / world), so the collective can sit inside the
 * same captured graph as the update with no divide launch between them (since ABI v4). */
G2048_API int g2048_adam_step_scaled(float* const* params_dev, const int64_t* numels, int n_tensors,
                                     const float* grad_dev, float* exp_avg_dev,
                                     float* exp_avg_sq_dev, const uint64_t* step_dev, double lr,
                                     double beta1, double beta2, double eps,
                                     float* const* target_params_dev, uint64_t sync_every,
                                     double grad_scale, void* stream);

/* ---- dense 16 -> 64 -> 4 Q-net (BASELINE configs[2]): the same four entry points ---------- */
typedef struct {
    const float *w1, *b1; /* Linear(16, 64) */
    const float *w2, *b2; /* Linear(64, 4)  */
} g2048_dense64_params;

/* play_one_step of every board with the dense 16-64-4 Q-network (BASELINE configs[2]) fused in:
 * each board's Q(s) is computed inside the step kernel (same fp32 summation order as
 * g2048_dense64_forward, so the actions are bitwise those of forward + g2048_env_step_egreedy),
 * then the eps-greedy step / replay append.  eps_decay_episodes > 0 selects the per-board
 * schedule (as g2048_env_step_egreedy_schedule); else eps_dev (device f64) or eps.
 * q_out f32[n][4] (16-byte aligned) receives Q, or NULL.  */
G2048_API int g2048_env_step_egreedy_dense64(g2048_env* env, const g2048_dense64_params* params,
                                             const double* eps_dev, double eps,
                                             double eps_decay_episodes, double eps_min,
                                             int32_t* reward_dev, uint8_t* done_dev,
                                             uint8_t* action_dev, g2048_replay* rb,
                                             float* q_out_dev, void* stream);


G2048_API int g2048_dense64_forward(const g2048_dense64_params* params, const uint8_t* rows_dev,
                                    const int64_t* idx_dev, int64_t n, float* q_out_dev,
                                    void* stream);
G2048_API int g2048_dense64_targets(const g2048_dense64_params* online,
                                    const g2048_dense64_params* target, g2048_replay* rb,
                                    const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                    const uint64_t* epoch_dev, float gamma, int double_dqn,
                                    int64_t* idx_out_dev, float* y_out_dev, void* stream);
G2048_API int64_t g2048_dense64_train_workspace(int64_t batch);
G2048_API int g2048_dense64_train_grad(const g2048_dense64_params* params,
                                       const uint8_t* rows_dev, const uint8_t* actions_dev,
                                       const int64_t* idx_dev, const float* y_dev, int64_t batch,
                                       float* workspace_dev, float* grad_out_dev,
                                       float* loss_out_dev, uint64_t* step_dev, void* stream);

/* One whole Double-DQN update of the dense net in two launches (train_step, src/dqn_lib.py:116-165,
 * intended zero_grad -> backward -> step order): per 32-row tile the sampler (idx_in, or the
 * Philox draw of g2048_dense64_targets with epoch *step_dev), Q_target(s') / Q_online(s') -> y,
 * Q_online(s) -> MSE(sum) -> gradient slab; then the fixed-order slab reduction, which with
 * exp_avg / exp_avg_sq non-NULL applies torch Adam (lr, betas, eps; t = *step_dev + 1) to the
 * ONLINE parameters in place.  *step_dev is incremented once.  grad_out (f32[1348], nullable with
 * Adam) receives the summed gradient -- for a data-parallel all-reduce, pass NULL Adam state here
 * and call g2048_adam_step afterwards.  idx_out / y_out receive the rows and targets; loss_out the
 * loss (nullable).  With Adam and sync_every > 0, the updated parameters are also written to the
 * TARGET net when t % sync_every == 0 (the target sync of training_loop, decided on the device).
 * G2048_DENSE64_ONE_LAUNCH=1 in the environment selects a one-launch form, bitwise the same
 * update (the last workgroups to finish their tiles reduce, synchronised through arrival counters
 * at the workspace's tail, which every update leaves at zero); measured slower, not the default.
 * workspace: f32[g2048_dense64_update_workspace(batch)], zero-filled before its first use. */
G2048_API int64_t g2048_dense64_update_workspace(int64_t batch);
G2048_API int g2048_dense64_update(const g2048_dense64_params* online,
                                   const g2048_dense64_params* target, g2048_replay* rb,
                                   const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                   uint64_t* step_dev, float gamma, int double_dqn,
                                   int64_t* idx_out_dev, float* y_out_dev, float* workspace_dev,
                                   float* grad_out_dev, float* loss_out_dev, float* exp_avg_dev,
                                   float* exp_avg_sq_dev, double lr, double beta1, double beta2,
                                   double eps, uint64_t sync_every, void* stream);

/* ---- float64 (the reference's precision, src/configs/double_dqn_dense.py:15) -------------
 * One whole Double-DQN update of the dense 16-64-4 net in float64, fused: per 64-row tile the
 * sampler (idx_in, or the Philox draw of g2048_replay_sample_encode with epoch *step_dev),
 * Q_target(s'), Q_online(s') -> y = r + double((1 - d) * gamma) * Q_target(s', a*) (gamma the
 * float32 torch uses), Q_online(s) -> MSELoss(sum) -> gradient slab; then a fixed-order slab
 * reduction that writes grad_out / loss_out and -- with exp_avg / exp_avg_sq -- applies torch's
 * Adam in float64 to the ONLINE parameters in place (+ the target sync when t % sync_every ==
 * 0).  Same step_dev protocol as g2048_dense64_update.  Parameters are device float64 tensors in
 * torch's layouts (Linear [out][in]).  G2048_DENSE64_ONE_LAUNCH as for g2048_dense64_update.
 * workspace: f64[g2048_dense64_update_f64_workspace(B)], zero-filled before its first use. */
typedef struct {
    double *w1, *b1; /* Linear(16, 64) */
    double *w2, *b2; /* Linear(64, 4)  */
} g2048_dense64_params_f64;

G2048_API int64_t g2048_dense64_update_f64_workspace(int64_t batch);
G2048_API int g2048_dense64_update_f64(const g2048_dense64_params_f64* online,
                                       const g2048_dense64_params_f64* target, g2048_replay* rb,
                                       const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                       uint64_t* step_dev, float gamma, int double_dqn,
                                       int64_t* idx_out_dev, double* y_out_dev,
                                       double* workspace_dev, double* grad_out_dev,
                                       double* loss_out_dev, double* exp_avg_dev,
                                       double* exp_avg_sq_dev, double lr, double beta1,
                                       double beta2, double eps, uint64_t sync_every,
                                       void* stream);

/* One whole Double-DQN update of the reference conv net (src/configs/double_dqn_conv.py:19-28)
 * in float64, the reference's precision (`.double()`, :28): the arguments, step_dev protocol,
 * sampler, Bellman target (gamma the float32 torch uses), MSELoss(sum), gradient order and
 * Adam / target-sync semantics of g2048_dense64_update_f64, for Conv2d(1,64,2) -> ReLU ->
 * Conv2d(64,64,2) -> ReLU -> Flatten -> Linear(256,64) -> ReLU -> Linear(64,4).  Four launches:
 * targets, two train launches, reduction + Adam.  grad_out: f64[33476] in torch parameter order.
 * workspace: f64[g2048_convnet_update_f64_workspace(B)]; it starts with both nets' weights packed
 * in f64-MFMA operand order.  With Adam folded in (exp_avg and exp_avg_sq given) the update reads
 * those packed operands and re-packs the weights it writes (the online net every update, the
 * target net on a sync), so the caller packs them with g2048_convnet_pack_f64 once after
 * allocating the workspace and again after changing either net's weights any other way (ABI v4:
 * an Adam-folded update on a workspace that was never packed for these two nets returns
 * G2048_EINVAL; the library remembers which workspaces it packed, host-side, by the workspace
 * and weight ADDRESSES -- a best-effort guard: a workspace freed and reallocated at the same
 * address for the same nets passes it without holding packed operands, so a caller that
 * reallocates a workspace packs it again, as after any other change of the weights).  A
 * gradient-only update (no Adam state: a data-parallel learner applies Adam after the
 * all-reduce) packs at its start. */
typedef struct {
    double *w1, *b1;       /* Conv2d(1, 64, 2)  */
    double *w2, *b2;       /* Conv2d(64, 64, 2) */
    double *fc1_w, *fc1_b; /* Linear(256, 64)   */
    double *fc2_w, *fc2_b; /* Linear(64, 4)     */
} g2048_convnet_params_f64;

G2048_API int64_t g2048_convnet_update_f64_workspace(int64_t batch);
/* Pack both nets' conv2 / fc1 weights into the head of an update workspace (one launch). */
G2048_API int g2048_convnet_pack_f64(const g2048_convnet_params_f64* online,
                                     const g2048_convnet_params_f64* target,
                                     double* workspace_dev, void* stream);
G2048_API int g2048_convnet_update_f64(const g2048_convnet_params_f64* online,
                                       const g2048_convnet_params_f64* target, g2048_replay* rb,
                                       const int64_t* idx_in_dev, int64_t batch, uint64_t seed,
                                       uint64_t* step_dev, float gamma, int double_dqn,
                                       int64_t* idx_out_dev, double* y_out_dev,
                                       double* workspace_dev, double* grad_out_dev,
                                       double* loss_out_dev, double* exp_avg_dev,
                                       double* exp_avg_sq_dev, double lr, double beta1,
                                       double beta2, double eps, uint64_t sync_every,
                                       void* stream);

/* The conv net's forward in float64 (the rollout's Q of a float64 learner): Q[b] (f64[n][4]) of
 * rows[idx ? idx[b] : b]; and the greedy-branch-only form, with the selection and arguments of
 * g2048_convnet_forward_greedy (rows of exploring boards are not written).  workspace: device
 * f64[G2048_CONVNET_F64_FWD_WORKSPACE] (the packed weight operands, rewritten by every call). */
#define G2048_CONVNET_F64_FWD_WORKSPACE 53248
G2048_API int g2048_convnet_forward_f64(const g2048_convnet_params_f64* params,
                                        const uint8_t* rows_dev, const int64_t* idx_dev, int64_t n,
                                        double* q_out_dev, double* workspace_dev, void* stream);
G2048_API int g2048_convnet_forward_greedy_f64(const g2048_convnet_params_f64* params,
                                               g2048_env* env, const double* eps_dev, double eps,
                                               double eps_decay_episodes, double eps_min,
                                               double* q_out_dev, double* workspace_dev,
                                               void* stream);

/* The forward of the reference's dense Q-net (src/configs/double_dqn_dense.py:7-15: Linear(16,
 * 512) ReLU Linear(512,512) ReLU Linear(512,256) ReLU Linear(256,4)) in float32 or float64
 * (dtype; every pointer below and q_out of that type): the rollout's `model(state)` of
 * epsilon_greedy_policy (src/dqn_lib.py:20-24) for a learner that trains this net on the torch
 * path.  g2048_densenet_forward: Q[b] (q_out[n][4]) of rows[idx ? idx[b] : b].
 * g2048_densenet_forward_greedy: Q of exactly the env's boards whose next eps-greedy step takes
 * the greedy branch (the step's own draw; eps forms of g2048_env_step_egreedy[_schedule]); rows
 * of exploring boards are not written.  A row's Q does not depend on the other rows: the greedy
 * rows are bitwise the all-rows forward's. */
typedef struct {
    const void *w1, *b1; /* Linear(16, 512)  */
    const void *w2, *b2; /* Linear(512, 512) */
    const void *w3, *b3; /* Linear(512, 256) */
    const void *w4, *b4; /* Linear(256, 4)   */
} g2048_densenet_params;
G2048_API int g2048_densenet_forward(const g2048_densenet_params* params, int dtype,
                                     const uint8_t* rows_dev, const int64_t* idx_dev, int64_t n,
                                     void* q_out_dev, void* stream);
G2048_API int g2048_densenet_forward_greedy(const g2048_densenet_params* params, int dtype,
                                            g2048_env* env, const double* eps_dev, double eps,
                                            double eps_decay_episodes, double eps_min,
                                            void* q_out_dev, void* stream);

/* One whole Double-DQN update of the reference dense net (train_step, src/dqn_lib.py:119-164, +
 * the target sync of :227-228) in float32 or float64 (dtype; y_out, workspace, grad_out,
 * loss_out, exp_avg, exp_avg_sq and both nets' tensors of that type): the arguments, step_dev
 * protocol, Philox sampler (idx_in NULL) or given rows, Bellman target (gamma the float32 torch
 * uses), MSELoss(sum), gradient order (torch parameter order, grad_out[403716]) and Adam /
 * target-sync semantics of g2048_convnet_update_f64.  With exp_avg / exp_avg_sq the update
 * writes the online net's tensors (and the target's on a sync) through the params' pointers.
 * Six launches: sampler, the two target-side forwards, the row tiles (forward with stored
 * activations, MSE, the input-gradient GEMMs, dW1 / dW4 / bias terms), the dW2 / dW3 GEMMs
 * (K = batch, split in row ranges), the fixed-order reduction with Adam.  workspace: dtype
 * elements, g2048_densenet_update_workspace(batch, dtype) of them (since ABI v4). */
G2048_API int64_t g2048_densenet_update_workspace(int64_t batch, int dtype);
G2048_API int g2048_densenet_update(const g2048_densenet_params* online,
                                    const g2048_densenet_params* target, int dtype,
                                    g2048_replay* rb, const int64_t* idx_in_dev, int64_t batch,
                                    uint64_t seed, uint64_t* step_dev, float gamma, int double_dqn,
                                    int64_t* idx_out_dev, void* y_out_dev, void* workspace_dev,
                                    void* grad_out_dev, void* loss_out_dev, void* exp_avg_dev,
                                    void* exp_avg_sq_dev, double lr, double beta1, double beta2,
                                    double eps, uint64_t sync_every, void* stream);

/* g2048_adam_step_sync in float64: the Adam update of the float64 fused reductions (torch's Adam
 * with its scalars in double) over n_tensors (<= 16) float64 parameter tensors, for a
 * data-parallel float64 learner (gradient -> all-reduce -> this step). */
G2048_API int g2048_adam_step_sync_f64(double* const* params_dev, const int64_t* numels,
                                       int n_tensors, const double* grad_dev, double* exp_avg_dev,
                                       double* exp_avg_sq_dev, const uint64_t* step_dev, double lr,
                                       double beta1, double beta2, double eps,
                                       double* const* target_params_dev, uint64_t sync_every,
                                       void* stream);
/* g2048_adam_step_scaled in float64 (gradient read as g * grad_scale). */
G2048_API int g2048_adam_step_scaled_f64(double* const* params_dev, const int64_t* numels,
                                         int n_tensors, const double* grad_dev,
                                         double* exp_avg_dev, double* exp_avg_sq_dev,
                                         const uint64_t* step_dev, double lr, double beta1,
                                         double beta2, double eps,
                                         double* const* target_params_dev, uint64_t sync_every,
                                         double grad_scale, void* stream);

/* g2048_env_step_egreedy_dense64 for a float64 dense 16-64-4 net: Q(s) computed in the step
 * kernel in double, the step as g2048_env_step_egreedy with f64 Q (q_out: f64[n][4] or NULL). */
G2048_API int g2048_env_step_egreedy_dense64_f64(g2048_env* env,
                                                 const g2048_dense64_params_f64* params,
                                                 const double* eps_dev, double eps,
                                                 double eps_decay_episodes, double eps_min,
                                                 int32_t* reward_dev, uint8_t* done_dev,
                                                 uint8_t* action_out_dev, g2048_replay* rb,
                                                 double* q_out_dev, void* stream);

/* ---- A* replay pre-fill (src/state_space_search.py:46-131), host code -------------------
 * Best-first search from one board (exponents start[16], merge score start_score) until a
 * popped board holds a tile of exponent goal_exp: priority -score // 2, ties in insertion
 * order, the reference's closed-list rule and child order (up, down, left, right), one spawn
 * per child -- Philox4x32-10 keyed (seed, game, expansion counter), or (tests, parity with
 * reference runs) a 2 in the first empty cell.  Writes the path root .. returned node:
 * path_boards [len + 1][16], path_moves [len], path_scores [len + 1]; *success = 0 when the
 * open list empties or max_expansions (> 0) is reached -- the last popped node is returned,
 * as in the reference.  G2048_EINVAL if the path is longer than max_path.  No GPU needed. */
#define G2048_ASTAR_SPAWN_PHILOX 0
#define G2048_ASTAR_SPAWN_FIRST_EMPTY 1
G2048_API int g2048_astar_search(const uint8_t* start, int64_t start_score, int goal_exp,
                                 uint64_t seed, uint64_t game, int spawn_mode,
                                 int64_t max_expansions, int64_t max_path, uint8_t* path_boards,
                                 uint8_t* path_moves, int64_t* path_scores, int64_t* path_len,
                                 int64_t* visited, int64_t* expanded, int* success);

/* ---- misc ---- */
G2048_API const char* g2048_last_error(void);
G2048_API int g2048_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* G2048_H */
