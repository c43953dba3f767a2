/* oracle2048.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference hot path (ribal-aladeeb/reinforcement-learning-2048,
 * src/board.py + src/dqn_lib.py) and of this build's env-step contract (include/g2048.h).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the CPU baseline -- never as the product path.
 *
 * Parity pinning: the slide/score restatement is checked against every reference golden
 * vector in tests/golden/ (row KATs, exhaustive 65 536-row LUT, injected-spawn trajectories,
 * epsilon-greedy rows), all produced by running the Python reference in the build container
 * (tests/golden/gen_goldens.py).
 *
 * Boards are 16 log2 exponents (0 = empty), row-major: cell(r,c) = 4r + c.
 */
#ifndef ORACLE2048_H
#define ORACLE2048_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/board.py:92-126 _apply_action_to_vector on exponents; returns the merge-score gain. */
uint32_t o2048_slide_row(const uint8_t in[4], uint8_t out[4]);
/* src/board.py:147-183 up/down/left/right WITHOUT the spawn; action 0=up 1=down 2=left 3=right. */
uint32_t o2048_move(const uint8_t in[16], int action, uint8_t out[16]);
/* src/board.py:128-135 available_moves_as_torch_unit_vector as a bit mask (bit a = move a legal). */
uint8_t o2048_legal_mask(const uint8_t b[16]);
/* Philox4x32-10 (Salmon et al. 2011; rocRAND philox4x32_10 constants and round order). */
void o2048_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* src/dqn_lib.py:25-29 greedy branch (compat formula) / fixed (legal-only argmax). */
int o2048_greedy_f64(const double q[4], uint8_t legal, int fixed);
int o2048_greedy_f32(const float q[4], uint8_t legal, int fixed);

/* Batched env step, mirroring g2048_env_step* exactly (see include/g2048.h for the contract).
 * mode: 0 = actions in, 1 = random, 2 = eps-greedy over q_f32, 3 = eps-greedy over q_f64,
 *       4 = actions in + injected spawns.
 * meta: uint32[N][2] = {score, moves}; ep: uint32[N][4] = {episodes, last_score, last_moves,
 * last_max_exp}; clock: uint64[ceil(N/64)] step counters (board i uses clock[i/64]).  Replay
 * pointers may be NULL (no append). */
/* One finished episode, the layout of include/g2048.h g2048_episode (40 B). */
typedef struct {
    uint64_t step;
    double q_sum;
    uint32_t board, episode, score, moves, max_exp, reserved;
} o2048_episode;

typedef struct {
    int64_t n;               /* boards in this shard */
    uint64_t board_offset;   /* global id of board 0 (rank * n for sharded envs) */
    uint64_t seed;
    uint32_t flags;
    uint8_t* board;          /* [n][16] */
    uint32_t* meta;          /* [n][2]  */
    uint32_t* ep;            /* [n][4]  */
    uint64_t* clock;         /* [ceil(n/64)] */
    double* qsum;            /* [n] running max-Q sum, or NULL (episode log off) */
    o2048_episode* log;      /* [n][log_slots]: board i's episode e at i*S + e%S, or NULL */
    int64_t log_slots;
} o2048_env;

typedef struct {
    int64_t capacity;
    uint8_t* s;   /* [C][16] */
    uint8_t* s2;  /* [C][16] */
    uint8_t* a;   /* [C] */
    int32_t* r;   /* [C] */
    uint8_t* d;   /* [C] */
    uint64_t* count;
} o2048_replay;

void o2048_env_reset(o2048_env* e, const uint8_t* mask_or_null, uint32_t epoch);
/* returns number of invalid inputs seen (bad action / occupied injected cell) */
int64_t o2048_env_step(o2048_env* e, int mode, const uint8_t* actions, const void* q, double eps,
                       double eps_decay, double eps_min,
                       const int8_t* spawn_idx, const uint8_t* spawn_exp,
                       int32_t* reward, uint8_t* done, uint8_t* legal_out,
                       uint8_t* action_out, o2048_replay* rb);
/* src/dqn_lib.py:33-84 sample_experiences + extract_samples_*: gather + exponent encode.
 * idx may be NULL: then idx[b] = mulhi(philox(seed, b, epoch).x, count). */
void o2048_replay_sample_f64(const o2048_replay* rb, const int64_t* idx, int64_t B,
                             uint64_t seed, uint64_t epoch, int64_t* idx_out,
                             double* s, double* s2, int64_t* a, double* r, double* d);

#ifdef __cplusplus
}
#endif
#endif
