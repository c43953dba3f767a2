// g2048.hip -- batched 2048 env step / rollout / reset and replay sample-encode kernels for
// gfx950, plus the extern "C" ABI declared in include/g2048.h.
//
// HBM layout (one env = one shard of boards, SoA):
//   board u8[N][16]   exponents                       (one uint4 per board)
//   meta  u32[2][N]   row 0: score; row 1: start = the step clock (low word) at which the running
//                     episode began, so moves = clock - start (mod 2^32) is derived, never
//                     stored: a one-launch step reads and writes 4 B of meta per board, and the
//                     start row is written only when an episode ends (ABI v5; v4 held {score,
//                     moves} per board and moved 16 B per step)
//   ep    u32[N][4]   {episodes, last score, last moves, last max exponent} (read with the board
//                     only where the step needs it; written on done)
//   clock u64[N/64]   the step counter of each 64-board group (all equal: every call steps every
//                     board).  The wavefront that steps group g is the only reader-writer of
//                     clock[g], so the counter needs no grid-wide ordering, and it reaches the
//                     kernel as a scalar: Philox counters, ring rows and ring offsets of a step
//                     are SALU work.
// Replay ring (capacity C): s u8[C][16], s2 u8[C][16], a u8[C], r i32[C], d u8[C], count u64.
// Optional episode log (g2048_env_set_episode_log): g2048_episode records [N][S], board i's
// episode e in slot i*S + e%S, written on its terminal step + qsum f64[N] (running sum of
// max_a Q over the board's episode).
//
// One lane owns one board for the whole launch: load board + meta, do the legal-mask / select /
// slide / spawn / reset arithmetic in VGPRs (g2048_board.hpp), store them back.  Consecutive
// blocks own consecutive board ranges, so a board's lines stay in the same XCD L2 from one step
// to the next (blocks are dealt round-robin over the 8 XCDs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"
#include "g2048_roll.hpp"

using namespace g2048;

namespace {

constexpr int kBlock = 256;
// k_step's workgroup below kStepSmallMaxBoards: one wave per workgroup.  At 64k boards the step
// is bound by its launch floor, and 1 024 one-wave workgroups finish sooner than 256 four-wave
// ones (tools/blockbench.py, cold process: 2.75 us vs 2.96 us per step; 128: 3.36, 512: 3.24,
// 1 024: 4.22).  HBM-bound sizes keep 256.
constexpr int kStepBlockSmall = 64;
constexpr int64_t kStepSmallMaxBoards = 1 << 20;
static_assert(kBlock % G2048_CLOCK_GROUP == 0 && kStepBlockSmall % G2048_CLOCK_GROUP == 0,
              "a wavefront must own whole clock groups");
enum : int {
    MODE_ACTIONS = 0,
    MODE_RANDOM = 1,
    MODE_EG_F32 = 2,
    MODE_EG_F64 = 3,
    MODE_INJECT = 4,
    MODE_EG_REG = 5,   // eps-greedy over f32 Q computed in-kernel (passed in registers)
    MODE_EG_REG64 = 6  // eps-greedy over f64 Q computed in-kernel (passed in registers)
};

struct ReplayDev {
    uint4* s;
    uint4* s2;
    uint8_t* a;
    int32_t* r;
    uint8_t* d;
    unsigned long long* count;
    int64_t capacity;
    int64_t rows;  // capacity / n  (0 = no replay)
    // one buffer-resource window over every section (k_rollout's buffer stores): base, size and
    // the byte offset of each section in it; win_bytes = 0 when the sections do not fit 4 GiB
    uint8_t* win;
    uint32_t win_bytes;
    uint32_t o_s, o_s2, o_a, o_r, o_d;
};

struct StepArgs {
    uint4* board;
    uint32_t* score;  // meta row 0
    uint32_t* start;  // meta row 1
    uint4* ep;
    uint64_t* clock;
    int64_t n;
    uint64_t board_offset;
    uint32_t seed_lo, seed_hi;
    uint32_t p4_thresh;
    uint32_t flags;
    const uint8_t* actions;
    const void* q;
    const double* eps_dev;
    double eps;
    double eps_decay;  // > 0: per-board schedule eps_b = max((D - episodes_b) / D, eps_min)
    double eps_min;
    const int8_t* spawn_idx;
    const uint8_t* spawn_exp;
    int32_t* reward;
    uint8_t* done;
    uint8_t* legal_out;
    uint8_t* action_out;
    unsigned long long* err;
    ReplayDev rb;
    int k_steps;
    long long* reward_sum;
    g2048_episode* log;  // per-board episode slot rings [n][log_slots] (NULL = off)
    int64_t log_slots;
    double* qsum;        // per-board running sum of max Q (NULL = off)
};

__device__ __forceinline__ Board load_board(const uint4 v) { return Board{v.x, v.y, v.z, v.w}; }

// {score, moves} of board i at clock t (the rollouts carry both in registers)
__device__ __forceinline__ uint2 load_meta(const StepArgs& A, int64_t i, uint64_t t) {
    return make_uint2(A.score[i], (uint32_t)t - A.start[i]);
}
// ... and back at clock t1: the start row only if an episode ended in the launch (otherwise
// t1 - moves is the start it was loaded with)
__device__ __forceinline__ void store_meta(const StepArgs& A, int64_t i, uint64_t t1, uint2 m,
                                           bool ended) {
    A.score[i] = m.x;
    if (ended) A.start[i] = (uint32_t)t1 - m.y;
}

// The step counter of board i's 64-board group as a wave-uniform (SGPR) value.  Every lane of the
// wave loads the same word; the wave's first lane is always live (groups start at 64-aligned
// board indices and a wave never straddles two groups).
// A 64-bit value as the wave's first lane holds it, in SGPRs.  readfirstlane returns an int: each
// half goes through uint32_t before widening, or a low word >= 2^31 would sign-extend into the
// high word (the rollout kernels' clocks past 2^31 steps were wrong that way until round 5).
__device__ __forceinline__ uint64_t first_lane_u64(uint64_t c) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)c);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(c >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint64_t load_clock(const uint64_t* clock, int64_t i) {
    return first_lane_u64(clock[i >> 6]);
}

// k_step's form: the group index is wave-uniform by construction (a wave never straddles two
// groups and its first live lane is 64-aligned), so the address is an SGPR value and the load is a
// scalar one -- a shorter round trip than a vector load + readfirstlane, and the first one on the
// step's critical path (the Philox counter needs t).
template <int BS>
__device__ __forceinline__ uint64_t load_clock_s(const uint64_t* clock) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
    return clock[(int64_t)blockIdx.x * (BS / 64) + wave];
}

// Ring row of step t (t mod rows) -- wave-uniform.
__device__ __forceinline__ uint64_t ring_row(uint64_t t, int64_t rows) {
    return (t >> 32) ? (t % (uint64_t)rows) : (uint64_t)((uint32_t)t % (uint32_t)rows);
}

// End of board i's episode on its terminal step t: the Experiment.add_episode fields
// (src/experiments.py:112-122) into ep[i] and, with a log attached, one record in the board's own
// slot ring (no atomics, fixed order).  The caller re-deals the board.
template <bool kGreedy>
__device__ __forceinline__ void end_episode(const StepArgs& A, int64_t i, uint64_t gid, uint64_t t,
                                            const Board& b, const uint2& m, uint4& ep, double& qs) {
    const uint32_t mx = max_exp(b);
    const uint32_t ep_idx = ep.x;
    ep = make_uint4(ep.x + 1u, m.x, m.y, mx);
    A.ep[i] = ep;
    if (A.log) {
        g2048_episode rec;
        rec.step = t;
        rec.q_sum = qs;
        rec.board = (uint32_t)gid;
        rec.episode = ep_idx;
        rec.score = m.x;
        rec.moves = m.y;
        rec.max_exp = mx;
        rec.reserved = 0u;
        A.log[i * A.log_slots + (int64_t)(ep_idx % (uint32_t)A.log_slots)] = rec;
    }
    qs = 0.0;
    if constexpr (!kGreedy) {  // non-greedy steps add 0 to the sum: reset it on done
        if (A.qsum) A.qsum[i] = 0.0;
    }
}

// One transition of board i (global id gid) at step t (the group clock).  Mirrors o2048_env_step
// (oracle/oracle2048.c), which restates src/dqn_lib.py:91-107 + src/board.py.
// m.x is the score; the episode's moves (clock - start) are needed only on a terminal step, and a
// re-dealt board's start row is written there -- a one-launch step moves 4 B of meta, not 16.
// kPre: the caller loaded ep, the start row (in m.y) and qs (when a q-sum buffer is attached)
// together with the board; otherwise ep and start are read on a terminal step only.
// Otherwise they are loaded here on done only -- 16 B less traffic per board, at the price of a
// dependent memory round trip for every wave that holds a terminal board.
template <int MODE, bool kPre = true>
__device__ __forceinline__ void step_one(const StepArgs& A, int64_t i, uint64_t gid, uint64_t t,
                                         Board& b, uint2& m, double eps, double& qs,
                                         int32_t& rew_out, uint32_t& done_out, uint32_t& legal_out,
                                         uint32_t& act_out, uint4& ep,
                                         float4 qreg = float4{0, 0, 0, 0},
                                         double4 qreg64 = double4{0, 0, 0, 0}) {
    constexpr bool kGreedy = MODE == MODE_EG_F32 || MODE == MODE_EG_F64 || MODE == MODE_EG_REG ||
                             MODE == MODE_EG_REG64;
    const Board s_old = b;
    uint32_t legal = 0u, act, r = 0u;
    bool done;
    uint4 u;
    RandWords rw{0u, 0u, 0u};
    if constexpr (MODE == MODE_RANDOM) {  // the random-policy contract of g2048_roll.hpp
        const bool p410 = (A.flags & G2048_P4_10) != 0u;
        rw = random_words(A.seed_lo, A.seed_hi, gid, t, p410);
        act = rw.w >> 30;
        if (A.legal_out) legal = legal_mask(b);
        uint4 F, I;
        dir_sel_reg(act, F, I);
        r = lean_step(b, rw.w, p410 ? spawn_exp<true>(rw.w, rw.v, A.p4_thresh)
                                   : spawn_exp<false>(rw.w, rw.v, A.p4_thresh), F, I, done);
    } else {
        u = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_STEP, t);
        legal = legal_mask(b);
        done = legal == 0u;
        if constexpr (MODE == MODE_ACTIONS || MODE == MODE_INJECT) {
            act = A.actions[i];
        } else {
            const bool explore = explores(u.y, eps);
            const bool fixed = (A.flags & G2048_EGREEDY_FIXED) != 0u;
            if (explore) {
                const uint32_t nl = __popc(legal);
                act = (fixed && nl) ? kth_bit4(legal, __umulhi(u.x, nl)) : (u.x >> 30);
            } else if constexpr (MODE == MODE_EG_F32 || MODE == MODE_EG_REG) {
                float4 q;
                if constexpr (MODE == MODE_EG_REG) q = qreg;
                else q = reinterpret_cast<const float4*>(A.q)[i];
                act = fixed ? greedy_fixed(q.x, q.y, q.z, q.w, legal)
                            : greedy_compat(q.x, q.y, q.z, q.w, legal);
                qs += (double)qmax4_torch(q.x, q.y, q.z, q.w);  // torch.max(Q) (:29)
            } else if constexpr (MODE == MODE_EG_REG64) {
                const double4 q = qreg64;
                act = fixed ? greedy_fixed(q.x, q.y, q.z, q.w, legal)
                            : greedy_compat(q.x, q.y, q.z, q.w, legal);
                qs += qmax4_torch(q.x, q.y, q.z, q.w);
            } else {
                const double2 q01 = reinterpret_cast<const double2*>(A.q)[2 * i];
                const double2 q23 = reinterpret_cast<const double2*>(A.q)[2 * i + 1];
                act = fixed ? greedy_fixed(q01.x, q01.y, q23.x, q23.y, legal)
                            : greedy_compat(q01.x, q01.y, q23.x, q23.y, legal);
                qs += qmax4_torch(q01.x, q01.y, q23.x, q23.y);
            }
        }
        if (act > 3u) {
            atomicAdd(A.err, 1ull);  // src/board.py:192 IndexError -> counted, no-op here
        } else if (!done && ((legal >> act) & 1u)) {
            r = apply_move(b, act);
            if constexpr (MODE == MODE_INJECT) {
                const int si = A.spawn_idx[i];
                if (si >= 0 && si < 16 && cell_empty(b, (uint32_t)si))
                    set_cell(b, (uint32_t)si, A.spawn_exp[i]);
                else
                    atomicAdd(A.err, 1ull);
            } else {
                spawn(b, u.z, u.w, A.p4_thresh);
            }
        }
    }
    m.x += r;

    if (A.rb.rows) {
        const int64_t slot = (int64_t)ring_row(t, A.rb.rows) * A.n + i;
        A.rb.s[slot] = make_uint4(s_old.r0, s_old.r1, s_old.r2, s_old.r3);
        A.rb.s2[slot] = make_uint4(b.r0, b.r1, b.r2, b.r3);  // terminal: s' = s (F6)
        A.rb.a[slot] = (uint8_t)act;
        A.rb.r[slot] = (int32_t)r;
        A.rb.d[slot] = (uint8_t)done;
    }

    if (done) {
        if constexpr (!kPre) {
            ep = A.ep[i];
            if constexpr (!kGreedy) {  // non-greedy steps add 0 to the sum: read it on done
                if (A.qsum) qs = A.qsum[i];
            }
        }
        m.y = (uint32_t)(t + 1u) - (kPre ? m.y : A.start[i]);  // this terminal step included
        end_episode<kGreedy>(A, i, gid, t, b, m, ep, qs);
        if (!(A.flags & G2048_NO_AUTORESET)) {
            if constexpr (MODE == MODE_RANDOM)
                b = (A.flags & G2048_P4_10) ? fresh_board_w<true>(rw.w, rw.v, rw.v2, A.p4_thresh)
                                            : fresh_board_w<false>(rw.w, rw.v, rw.v2, A.p4_thresh);
            else
                b = fresh_board(u, A.p4_thresh);  // the step's own block (see fresh_board)
            m = make_uint2(0u, 0u);
            A.start[i] = (uint32_t)(t + 1u);
        }
    }
    rew_out = (int32_t)r;
    done_out = done;
    legal_out = legal;
    act_out = act;
}

// count = min(t_next * n, capacity), without the product overflowing at any clock
__device__ __forceinline__ void bump_count(const StepArgs& A, uint64_t t_next) {
    const uint64_t c = t_next >= (uint64_t)A.rb.rows ? (uint64_t)A.rb.capacity
                                                     : t_next * (uint64_t)A.n;
    atomicMax(A.rb.count, (unsigned long long)c);
}

// kFull: every block is full (n % BS == 0), so there is no bounds test and every kernel argument
// load can be issued at once (with the test, the pointer loads wait for n's round trip).
// The four per-board pointers and the scalars the Philox draw needs first (board offset, seed,
// p(4) threshold, flags) are leading scalar arguments (copies of A's): the library is built with
// kernel-argument preloading (16 SGPRs), so they arrive in SGPRs and neither the board loads nor
// the draw wait for a scalar load of the argument block.
template <int MODE, bool kFull, bool kPre, int BS>
__global__ __launch_bounds__(BS) void k_step(uint4* __restrict__ board_p, uint32_t* __restrict__ score_p,
                                             uint4* ep_p, uint64_t* clock_p, uint64_t board_offset,
                                             uint32_t seed_lo, uint32_t seed_hi,
                                             uint32_t p4_thresh, uint32_t flags, StepArgs A) {
    const int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    if (!kFull && i >= A.n) return;
    A.board_offset = board_offset;
    A.seed_lo = seed_lo;
    A.seed_hi = seed_hi;
    A.p4_thresh = p4_thresh;
    A.flags = flags;
    const uint64_t t = load_clock_s<BS>(clock_p);
    Board b = load_board(board_p[i]);
    uint2 m = make_uint2(score_p[i], kPre ? A.start[i] : 0u);
    uint4 ep = kPre ? ep_p[i] : make_uint4(0u, 0u, 0u, 0u);
    double eps = 0.0;
    if constexpr (MODE == MODE_EG_F32 || MODE == MODE_EG_F64) {
        // src/dqn_lib.py:184-188 per board: ep.x = its episode count
        const uint32_t e = A.eps_decay > 0.0
                               ? (kPre ? ep.x : reinterpret_cast<const uint32_t*>(A.ep)[4 * i])
                               : 0u;
        eps = step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, e);
    }
    int32_t rew;
    uint32_t done, legal, act;
    constexpr bool kGreedy = MODE == MODE_EG_F32 || MODE == MODE_EG_F64;
    double qs = ((kPre || kGreedy) && A.qsum) ? A.qsum[i] : 0.0;
    step_one<MODE, kPre>(A, i, board_offset + (uint64_t)i, t, b, m, eps, qs, rew, done, legal,
                         act, ep);
    board_p[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    score_p[i] = m.x;
    if ((i & 63) == 0) clock_p[i >> 6] = t + 1u;
    if (kGreedy && A.qsum) A.qsum[i] = qs;
    if (A.reward) A.reward[i] = rew;
    if (A.done) A.done[i] = (uint8_t)done;
    if (A.legal_out) A.legal_out[i] = (uint8_t)legal;
    if (A.action_out) A.action_out[i] = (uint8_t)act;
    if (A.rb.rows && i == 0) bump_count(A, t + 1u);
}

// The fused rollout step of the dense 16-64-4 net (BASELINE configs[2]): Q(s) of each board
// (h = relu(W1 x + b1), Q = W2 h + b2 in the summation order of k_mlp_forward, so Q and the
// chosen actions are bitwise those of forward + g2048_env_step_egreedy), then the eps-greedy
// step.  Weights are SGPR operands (uniform loads -> s_load): with one wave doing all 64 units
// per board at 64k boards (1 wave per SIMD) the MLP phase was bound by exposed scalar-load
// latency (~12k cycles; an LDS-staged variant hit the same time, bound by LDS broadcast
// bandwidth).
// The MLP is split over two waves per 64 boards (workgroup of 128): wave 0 evaluates the even
// hidden units (the e chains, bias included), wave 1 the odd units (the o chains); wave 1 hands
// its o over through LDS and wave 0 forms Q = e + o and takes the step.  The two waves per SIMD
// hide each other's scalar-load latency: 7.4 us per 64k-board step against 8.6 us with one wave
// doing all 64 units (tools/stepbench.py).
template <bool kFull>
__global__ __launch_bounds__(128) void k_step_dense64_split(StepArgs A, const float* __restrict__ w1,
                                                            const float* __restrict__ b1,
                                                            const float* __restrict__ w2,
                                                            const float* __restrict__ b2,
                                                            float* q_out) {
    __shared__ float4 so[64];
    const int lane = threadIdx.x & 63;
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const bool live = kFull || i < A.n;
    Board b{0u, 0u, 0u, 0u};
    uint2 m = make_uint2(0u, 0u);
    uint4 ep = make_uint4(0u, 0u, 0u, 0u);
    // both waves hold the same 64 boards (one clock group); lane 0 is live in every workgroup
    const uint64_t t = load_clock(A.clock, (int64_t)blockIdx.x * 64);
    if (live) {
        b = load_board(A.board[i]);
        if (half == 0 || !q_out) {
            m = make_uint2(A.score[i], A.start[i]);  // step_one's kPre form
            ep = A.ep[i];
        }
    }
    // epsilon_greedy_policy evaluates the model only on its greedy branch (src/dqn_lib.py:20-24):
    // when no board of the 64 takes it (early in the eps schedule) both waves skip the MLP --
    // unless q_out asks for every board's Q.  The two waves hold the same boards, so they agree.
    bool any_greedy = true;
    if (!q_out) {
        bool greedy = false;
        if (live) {
            const uint4 u = draw(A.seed_lo, A.seed_hi, A.board_offset + (uint64_t)i, DOMAIN_STEP, t);
            greedy = !explores(u.y, step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, ep.x));
        }
        any_greedy = __ballot(greedy) != 0ull;
    }
    float x[16];
    const uint32_t rw[4] = {b.r0, b.r1, b.r2, b.r3};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) x[4 * r + c] = (float)((rw[r] >> (8 * c)) & 0xFFu);
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2* w1p = reinterpret_cast<const f2*>(w1);  // [j][k/2]
    f2 xp[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xp[u] = f2{x[2 * u], x[2 * u + 1]};
    float acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a] = half == 0 ? b2[a] : 0.f;
#pragma unroll 4
    for (int jj = 0; jj < 32 && any_greedy; ++jj) {
        const int j = 2 * jj + half;
        f2 pa = f2{b1[j], 0.f}, pb = f2{0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pa = __builtin_elementwise_fma(w1p[j * 8 + 2 * u], xp[2 * u], pa);
            pb = __builtin_elementwise_fma(w1p[j * 8 + 2 * u + 1], xp[2 * u + 1], pb);
        }
        const float h = fmaxf((pa.x + pa.y) + (pb.x + pb.y), 0.f);
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a] = fmaf(w2[a * 64 + j], h, acc[a]);
    }
    if (half == 1) so[lane] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (half == 1 || !live) return;
    const float4 o = so[lane];
    const float4 q = make_float4(acc[0] + o.x, acc[1] + o.y, acc[2] + o.z, acc[3] + o.w);
    const double eps = step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, ep.x);
    if (q_out) reinterpret_cast<float4*>(q_out)[i] = q;
    int32_t rew;
    uint32_t done, legal, act;
    double qs = A.qsum ? A.qsum[i] : 0.0;
    step_one<MODE_EG_REG>(A, i, A.board_offset + (uint64_t)i, t, b, m, eps, qs, rew, done, legal,
                          act, ep, q);
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    A.score[i] = m.x;
    if (lane == 0) A.clock[blockIdx.x] = t + 1u;  // wave 1 read it before the barrier
    if (A.qsum) A.qsum[i] = qs;
    if (A.reward) A.reward[i] = rew;
    if (A.done) A.done[i] = (uint8_t)done;
    if (A.action_out) A.action_out[i] = (uint8_t)act;
    if (A.rb.rows && i == 0) bump_count(A, t + 1u);
}

// The float64 form (the reference's precision, src/configs/double_dqn_dense.py:15): the same
// two-wave split and selection as k_step_dense64_split, the MLP in double (SGPR weight operands)
// and Q (double) handed to the step in registers; Q = e + o with wave 0's chain holding b2.
template <bool kFull>
__global__ __launch_bounds__(128) void k_step_dense64_split64(StepArgs A, const double* __restrict__ w1,
                                                              const double* __restrict__ b1,
                                                              const double* __restrict__ w2,
                                                              const double* __restrict__ b2,
                                                              double* q_out) {
    __shared__ double4 so[64];
    const int lane = threadIdx.x & 63;
    const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const bool live = kFull || i < A.n;
    Board b{0u, 0u, 0u, 0u};
    uint2 m = make_uint2(0u, 0u);
    uint4 ep = make_uint4(0u, 0u, 0u, 0u);
    const uint64_t t = load_clock(A.clock, (int64_t)blockIdx.x * 64);
    if (live) {
        b = load_board(A.board[i]);
        if (half == 0 || !q_out) {
            m = make_uint2(A.score[i], A.start[i]);  // step_one's kPre form
            ep = A.ep[i];
        }
    }
    bool any_greedy = true;  // the model runs on the greedy branch only (src/dqn_lib.py:20-24)
    if (!q_out) {
        bool greedy = false;
        if (live) {
            const uint4 u = draw(A.seed_lo, A.seed_hi, A.board_offset + (uint64_t)i, DOMAIN_STEP, t);
            greedy = !explores(u.y, step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, ep.x));
        }
        any_greedy = __ballot(greedy) != 0ull;
    }
    double x[16];
    const uint32_t rw[4] = {b.r0, b.r1, b.r2, b.r3};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) x[4 * r + c] = (double)((rw[r] >> (8 * c)) & 0xFFu);
    double acc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a] = half == 0 ? b2[a] : 0.0;
#pragma unroll 2
    for (int jj = 0; jj < 32 && any_greedy; ++jj) {
        const int j = 2 * jj + half;
        double pa = b1[j], pb = 0.0;
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            pa = fma(w1[j * 16 + k], x[k], pa);
            pb = fma(w1[j * 16 + k + 1], x[k + 1], pb);
        }
        const double pre = pa + pb;
        const double h = pre > 0.0 ? pre : 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a] = fma(w2[a * 64 + j], h, acc[a]);
    }
    if (half == 1) so[lane] = double4{acc[0], acc[1], acc[2], acc[3]};
    __syncthreads();
    if (half == 1 || !live) return;
    const double4 o = so[lane];
    const double4 q = double4{acc[0] + o.x, acc[1] + o.y, acc[2] + o.z, acc[3] + o.w};
    const double eps = step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, ep.x);
    if (q_out) {
        reinterpret_cast<double2*>(q_out)[2 * i] = make_double2(q.x, q.y);
        reinterpret_cast<double2*>(q_out)[2 * i + 1] = make_double2(q.z, q.w);
    }
    int32_t rew;
    uint32_t done, legal, act;
    double qs = A.qsum ? A.qsum[i] : 0.0;
    step_one<MODE_EG_REG64>(A, i, A.board_offset + (uint64_t)i, t, b, m, eps, qs, rew, done,
                            legal, act, ep, float4{0, 0, 0, 0}, q);
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    A.score[i] = m.x;
    if (lane == 0) A.clock[blockIdx.x] = t + 1u;  // wave 1 read it before the barrier
    if (A.qsum) A.qsum[i] = qs;
    if (A.reward) A.reward[i] = rew;
    if (A.done) A.done[i] = (uint8_t)done;
    if (A.action_out) A.action_out[i] = (uint8_t)act;
    if (A.rb.rows && i == 0) bump_count(A, t + 1u);
}

// The ring as buffer resources: a step's five stores take the lane's constant byte offset
// (i * size) in voffset and the row's offset (row * n * size, wave-uniform) in soffset, so a
// step spends no VALU on addresses.  Used when every section of the ring is below 4 GiB.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A board's 16-byte buffer store whose data registers stay untouched for two wait states after
// it.  gfx950 reads a store's data VGPRs after issue when the store queue backs up, and a store of
// more than 8 bytes needs two wait states before a VALU rewrites them; hipcc does not always
// leave them (it scheduled the rollout's next v_perm into the board registers right behind the
// store: at 1M+ boards about one board in 1 600 of some ring rows was stored with the first word
// already overwritten).  The nop reads the four registers, so they stay live -- nothing is
// written into them -- until it has issued, two wait states after the store (both volatile:
// their order is kept).  tools/store_hazard_audit.py checks the compiled kernels.
template <int kAux = 0>
__device__ __forceinline__ void store_board(const Board& b, __amdgpu_buffer_rsrc_t rw,
                                            uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{b.r0, b.r1, b.r2, b.r3}, rw, voff, soff, kAux);
    asm volatile("s_nop 1" ::"v"(b.r0), "v"(b.r1), "v"(b.r2), "v"(b.r3));
}

// tools/prof_roll.hip: per-pair s_memtime ticks of a few waves (no-op in the library)
#ifndef G2048_ROLL_TICK
#define G2048_ROLL_TICK(np)
#define G2048_ROLL_MARK(k)
#endif

// g2048_env_rollout: k_steps random-policy steps of every board with the board, score, moves and
// episode counters held in registers; step t of the launch draws its word from the Philox block
// of its 4-step quad (ABI v3, g2048_roll.hpp random_words) and appends (s, a, r, s', d)
// to the ring.  Identical to k_steps g2048_env_step(actions = NULL) calls.  Issue-bound at 64k
// boards (one wave per SIMD, so SALU instructions cost issue turns like VALU ones): the loop
// keeps its scalar bookkeeping to a 32-bit ring row and a 64-bit pair counter, and the episode
// counters are stored once at the end (only the last finished episode's record survives in ep;
// the log, when attached, gets every one).  See DESIGN.md section 4.1.
//   kRing: a replay ring is attached; kBuf: its sections lie in one window below 4 GiB (buffer
//   stores through ONE resource, so the loop holds 4 SGPRs of descriptor, not 20);
//   kSum: per-board reward sums are accumulated.
template <bool kRing, bool kBuf, bool kSum>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kSum ? 5 : 6))) void k_rollout(StepArgs A) {
    __shared__ uint4 s_dir[8];  // the direction-selector table (g2048_roll.hpp kDirNet)
    if (threadIdx.x < 8)
        s_dir[threadIdx.x] = reinterpret_cast<const uint4*>(&kDirNet[0][0][0])[threadIdx.x];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= A.n) return;
    G2048_ROLL_MARK(0);
    const uint64_t t0 = load_clock(A.clock, i);
    Board b = load_board(A.board[i]);
    uint2 m = load_meta(A, i, t0);
    uint4 ep = A.ep[i];
    const uint64_t gid = A.board_offset + (uint64_t)i;
    const bool autoreset = !(A.flags & G2048_NO_AUTORESET);
    long long rsum = 0;
    double qs = A.qsum ? A.qsum[i] : 0.0;  // random policy: reset (0) on done only
    const uint32_t rows = kRing ? (uint32_t)A.rb.rows : 1u;
    uint32_t row = kRing ? (uint32_t)ring_row(t0, A.rb.rows) : 0u;
    // buffer path: the row's first slot (row * n) kept running, wrapped at the capacity
    const uint32_t cap32 = kBuf ? (uint32_t)A.rb.capacity : 0u;
    uint32_t soff = kBuf ? row * (uint32_t)A.n : 0u;
    const uint32_t n32 = (uint32_t)A.n;
    // (the global-store instance -- no 4 GiB window -- builds an empty descriptor)
    __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        A.rb.win, 0, (int)(kBuf ? A.rb.win_bytes : 0u), 0x00020000);
    const uint32_t lane = (uint32_t)i;
    // per-lane offsets of the five sections in the window (loop-invariant VGPRs)
    const uint32_t v_s = kBuf ? A.rb.o_s + 16u * lane : 0u, v_s2 = kBuf ? A.rb.o_s2 + 16u * lane : 0u;
    const uint32_t v_a = kBuf ? A.rb.o_a + lane : 0u, v_r = kBuf ? A.rb.o_r + 4u * lane : 0u;
    const uint32_t v_d = kBuf ? A.rb.o_d + lane : 0u;
    const uint32_t ep0 = ep.x;  // some episode of this board ended in the launch iff ep.x moved
    Board last = b;      // the final board of that episode (its max tile goes to ep.w at the end)
    const bool p410 = (A.flags & G2048_P4_10) != 0u;
    // one transition of step t with its draws rw (g2048_roll.hpp)
    // lean (std::true_type): no episode log and auto-reset on -- the loop then carries neither
    // uniform test
    const uint32_t k255 = opaque_255();
    auto one = [&](auto lean, const RandWords& rd, uint64_t t) {
        constexpr bool kLean = decltype(lean)::value;
        const uint32_t wa = rd.w;
        const Board so = b;
        bool done;
        const uint32_t a2 = (wa >> 30) * 2u;
        const uint32_t r = lean_step(b, wa,
                                     p410 ? spawn_exp<true>(wa, rd.v, A.p4_thresh)
                                          : spawn_exp<false>(wa, rd.v, A.p4_thresh),
                                     s_dir[a2], s_dir[a2 + 1u], done, k255);
        m.x += r;
        m.y += 1u;
        if constexpr (kSum) rsum += r;
        if constexpr (kRing) {
            if constexpr (kBuf) {
                store_board(so, rw, v_s, soff * 16u);
                store_board(b, rw, v_s2, soff * 16u);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(wa >> 30), rw, v_a, soff, 0);
                __builtin_amdgcn_raw_buffer_store_b32(r, rw, v_r, soff * 4u, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)done, rw, v_d, soff, 0);
            } else {
                const int64_t slot = (int64_t)row * A.n + i;
                A.rb.s[slot] = make_uint4(so.r0, so.r1, so.r2, so.r3);
                A.rb.s2[slot] = make_uint4(b.r0, b.r1, b.r2, b.r3);
                A.rb.a[slot] = (uint8_t)(wa >> 30);
                A.rb.r[slot] = (int32_t)r;
                A.rb.d[slot] = (uint8_t)done;
            }
            if constexpr (kBuf) soff = soff + n32 == cap32 ? 0u : soff + n32;
            else row = row + 1u == rows ? 0u : row + 1u;
        }
        if (done) {  // taken by some lane of the wave on roughly 40 % of the steps
            if (!kLean && A.log) {
                g2048_episode rec;
                rec.step = t;
                rec.q_sum = qs;
                rec.board = (uint32_t)gid;
                rec.episode = ep.x;
                rec.score = m.x;
                rec.moves = m.y;
                rec.max_exp = max_exp(b);
                rec.reserved = 0u;
                A.log[i * A.log_slots + (int64_t)(ep.x % (uint32_t)A.log_slots)] = rec;
            }
            ep = make_uint4(ep.x + 1u, m.x, m.y, 0u);
            last = b;
            qs = 0.0;
            if (kLean || autoreset) {
                b = p410 ? fresh_board_w<true>(wa, rd.v, rd.v2, A.p4_thresh)
                         : fresh_board_w<false>(wa, rd.v, rd.v2, A.p4_thresh);
                m = make_uint2(0u, 0u);
            }
        }
    };
    const int K = A.k_steps > 0 ? A.k_steps : 0;
    auto run = [&](auto lean) {
        // the quad's blocks are drawn when t enters it (a wave-uniform branch)
        uint4 blk = make_uint4(0, 0, 0, 0), vb = blk, vb2 = blk;
        G2048_ROLL_MARK(1);
        for (int s = 0; s < K; ++s) {
            const uint64_t t = t0 + (uint64_t)s;
            if (s == 0 || (t & 3u) == 0u) {
                if constexpr (kBuf) asm volatile("" : "+s"(rw));  // one SGPR quad for the descriptor
                blk = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, t >> 2);
                if (p410) value_blocks<true>(A.seed_lo, A.seed_hi, gid, t >> 2, vb, vb2);
            }
            const uint32_t k = (uint32_t)t & 3u;
            one(lean, RandWords{word_of(blk, k), word_of(vb, k), word_of(vb2, k)}, t);
        }
    };
    if (!A.log && autoreset) run(std::true_type{});
    else run(std::false_type{});
    G2048_ROLL_MARK(2);
    const uint64_t t1 = t0 + (uint64_t)K;
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    store_meta(A, i, t1, m, ep.x != ep0);
    if (ep.x != ep0) {
        ep.w = max_exp(last);
        A.ep[i] = ep;
        if (A.qsum) A.qsum[i] = 0.0;
    }
    if ((i & 63) == 0) A.clock[i >> 6] = t1;
    if constexpr (kSum) A.reward_sum[i] += rsum;
    if (kRing && i == 0) bump_count(A, t1);
    G2048_ROLL_MARK(3);
}

constexpr int kRingSc1 = 16;  // the sc1 bit of a gfx950 buffer store's cache policy

// The headline instance of g2048_env_rollout -- ring in one buffer window, auto-reset on, no
// episode log: four steps per iteration from one Philox block (one word per step), the next
// quad's block drawn at the top of a quad, and each step's direction selectors read from LDS one
// step ahead.  Each workgroup stages the selector table in LDS (64 B per action: F, I, 32 B
// unused, so a step's table offset is one v_and of its word's top byte).
//   kQR: the ring's rows (capacity / n) are a multiple of 4, so a quad never wraps: its four
//   steps take their row offsets from loop-invariant VGPRs (section offset + j * size * n) and
//   the quad's base from three SGPRs updated once per quad -- 1.25 SALU per step instead of 5
//   (at one wave per SIMD an SALU op costs an issue turn like a VALU op).
//   kStores: ring sections written (bits s, s2, a, r, d) -- all in the library; tools/rollexp.hip
//   times subsets to price the stores.
//   kWaves: the occupancy hint (the library uses 4; tools/rollexp.hip times others at large N).
//   kAux: the ring stores' cache-policy bits (the library uses kRingSc1; tools/rollexp.hip
//   times the others).
template <bool kSum, bool kP410, bool kQR, int kStores = 0x1F, int kWaves = 4, int kAux = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kWaves))) void k_rollout_lean(StepArgs A) {
    __shared__ uint4 s_dir[16];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < A.n;
    // the board state's loads go out before the table staging and its barrier, so their
    // latencies overlap (the prologue is a few steps' worth of a 64-step launch)
    uint64_t c0 = 0;
    uint4 bv = make_uint4(0, 0, 0, 0), ep = bv;
    uint2 m = make_uint2(0, 0);  // {score, start} until t0 is known, then {score, moves}
    if (live) {
        c0 = A.clock[i >> 6];
        bv = A.board[i];
        m = make_uint2(A.score[i], A.start[i]);
        ep = A.ep[i];
    }
    if (threadIdx.x < 16)
        s_dir[threadIdx.x] =
            (threadIdx.x & 2u) ? make_uint4(0, 0, 0, 0)
                               : reinterpret_cast<const uint4*>(
                                     &kDirNet[0][0][0])[(threadIdx.x >> 2) * 2u + (threadIdx.x & 1u)];
    __syncthreads();
    if (!live) return;
    const uint64_t t0 = first_lane_u64(c0);
    m.y = (uint32_t)t0 - m.y;
    Board b = load_board(bv);
    const uint64_t gid = A.board_offset + (uint64_t)i;
    const uint32_t p4 = A.p4_thresh;
    long long rsum = 0;
    const uint32_t row = (uint32_t)ring_row(t0, A.rb.rows);
    const uint32_t cap32 = (uint32_t)A.rb.capacity, n32 = (uint32_t)A.n;
    uint32_t soff = row * n32;
    __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(A.rb.win, 0, (int)A.rb.win_bytes, 0x00020000);
    const uint32_t lane = (uint32_t)i;
    const uint32_t v_s = A.rb.o_s + 16u * lane, v_s2 = A.rb.o_s2 + 16u * lane;
    const uint32_t v_a = A.rb.o_a + lane, v_r = A.rb.o_r + 4u * lane, v_d = A.rb.o_d + lane;
    const uint32_t ep0 = ep.x;
    Board last = b;
    const uint32_t k255 = opaque_255();
    // the ring offsets of one step: per-lane voffsets (section + lane) and the row's soffsets
    struct Off {
        uint32_t s, s2, a, r, d;  // VGPR
        uint32_t o16, o4, o1;     // SGPR: row * n * {16, 4, 1}
    };
    // one transition with the word w (+ value words v, v2 under G2048_P4_10), the action's
    // selector quads (F, I) and the ring offsets o
    auto one = [&](uint32_t w, uint32_t v, uint32_t v2, const uint4& F, const uint4& I,
                   const Off& o) {
        G2048_MARK(store_s, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
        if constexpr (kStores & 1)
            store_board<kAux>(b, rw, o.s, o.o16);
        bool done;
        const uint32_t r = lean_step(b, w, spawn_exp<kP410>(w, v, p4), F, I, done, k255);
        m.x += r;
        m.y += 1u;
        if constexpr (kSum) rsum += r;
        if constexpr ((kStores & 2) != 0)
            store_board<kAux>(b, rw, o.s2, o.o16);
        if constexpr ((kStores & 4) != 0)
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> 30), rw, o.a, o.o1, kAux);
        if constexpr ((kStores & 8) != 0) __builtin_amdgcn_raw_buffer_store_b32(r, rw, o.r, o.o4, kAux);
        if constexpr ((kStores & 16) != 0)
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)done, rw, o.d, o.o1, kAux);
        // a wave-uniform branch whose body is selects: every value keeps its registers (a
        // lane-masked `if (done)` made hipcc copy the board and counters through phi moves, and
        // a v_mov costs a full issue turn)
        G2048_MARK(reset, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
        const uint64_t dl = __builtin_amdgcn_ballot_w64(done);
        if (dl != 0u) {
            const Board f = fresh_board_w<kP410>(w, v, v2, p4);
            last.r0 = sel_lanes(dl, b.r0, last.r0);
            last.r1 = sel_lanes(dl, b.r1, last.r1);
            last.r2 = sel_lanes(dl, b.r2, last.r2);
            last.r3 = sel_lanes(dl, b.r3, last.r3);
            ep.x = sel_lanes(dl, ep.x + 1u, ep.x);
            ep.y = sel_lanes(dl, m.x, ep.y);
            ep.z = sel_lanes(dl, m.y, ep.z);
            b.r0 = sel_lanes(dl, f.r0, b.r0);
            b.r1 = sel_lanes(dl, f.r1, b.r1);
            b.r2 = sel_lanes(dl, f.r2, b.r2);
            b.r3 = sel_lanes(dl, f.r3, b.r3);
            m.x = sel_lanes(dl, 0u, m.x);
            m.y = sel_lanes(dl, 0u, m.y);
        }
    };
    // F, I of the action in w's top two bits: 64 B per action in s_dir
    auto sel = [&](uint32_t w, uint4& F, uint4& I) {
        const uint32_t off = (w >> 24) & 0xC0u;
        F = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s_dir) + off);
        I = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s_dir) + off + 16u);
    };
    // the running offsets of the one-at-a-time steps (wrap checked per step)
    auto step_off = [&]() {
        const Off o{v_s, v_s2, v_a, v_r, v_d, soff * 16u, soff * 4u, soff};
        soff = soff + n32 == cap32 ? 0u : soff + n32;
        return o;
    };
    const int K = A.k_steps > 0 ? A.k_steps : 0;
    // steps up to the first quad boundary, one at a time
    const int nh = min(K, (int)((4u - ((uint32_t)t0 & 3u)) & 3u));
    uint4 blk = make_uint4(0, 0, 0, 0), vb = blk, vb2 = blk;
    if (nh > 0) {
        blk = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, t0 >> 2);
        value_blocks<kP410>(A.seed_lo, A.seed_hi, gid, t0 >> 2, vb, vb2);
        for (int s = 0; s < nh; ++s) {
            const uint32_t k = ((uint32_t)t0 + (uint32_t)s) & 3u;
            uint4 F, I;
            const uint32_t w = word_of(blk, k);
            sel(w, F, I);
            one(w, word_of(vb, k), word_of(vb2, k), F, I, step_off());
        }
    }
    // whole quads: the block(s) of quad j + 1 are drawn at the top of quad j; each step issues
    // the selector reads of the next step before its own work (the last quad reads selectors
    // and draws blocks it does not use); two quads per iteration, so the blocks alternate
    // between two register sets
    uint64_t quad = (t0 + (uint64_t)nh) >> 2;
    blk = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, quad);
    value_blocks<kP410>(A.seed_lo, A.seed_hi, gid, quad, vb, vb2);
    // kQR: the quad's row offsets -- loop-invariant VGPRs for its four rows, SGPR quad base
    const uint32_t st16 = 16u * n32, st4 = 4u * n32;
    const uint32_t vq_s[4] = {v_s, v_s + st16, v_s + 2u * st16, v_s + 3u * st16};
    const uint32_t vq_s2[4] = {v_s2, v_s2 + st16, v_s2 + 2u * st16, v_s2 + 3u * st16};
    const uint32_t vq_a[4] = {v_a, v_a + n32, v_a + 2u * n32, v_a + 3u * n32};
    const uint32_t vq_r[4] = {v_r, v_r + st4, v_r + 2u * st4, v_r + 3u * st4};
    const uint32_t vq_d[4] = {v_d, v_d + n32, v_d + 2u * n32, v_d + 3u * n32};
    uint4 F, I;
    sel(blk.x, F, I);
    auto quad_of = [&](const uint4& cur, const uint4& cv, const uint4& cv2, uint4& nxt, uint4& nv,
                       uint4& nv2, uint64_t q_next) {
        G2048_MARK(philox, "+v"(F.x));
        nxt = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, q_next);
        value_blocks<kP410>(A.seed_lo, A.seed_hi, gid, q_next, nv, nv2);
        G2048_MARK(step, "+v"(nxt.x), "+v"(nxt.y), "+v"(nxt.z), "+v"(nxt.w));
        const uint32_t ws[5] = {cur.x, cur.y, cur.z, cur.w, nxt.x};
        const uint32_t vs[4] = {cv.x, cv.y, cv.z, cv.w}, v2s[4] = {cv2.x, cv2.y, cv2.z, cv2.w};
        const uint32_t q16 = soff * 16u, q4 = soff * 4u, q1 = soff;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint4 Fn, In;
            sel(ws[j + 1], Fn, In);  // the next step's selectors, in flight during this step
            asm volatile("" ::: "memory");
            if constexpr (kQR)
                one(ws[j], vs[j], v2s[j], F, I,
                    Off{vq_s[j], vq_s2[j], vq_a[j], vq_r[j], vq_d[j], q16, q4, q1});
            else
                one(ws[j], vs[j], v2s[j], F, I, step_off());
            F = Fn;
            I = In;
        }
        if constexpr (kQR) soff = soff + 4u * n32 == cap32 ? 0u : soff + 4u * n32;
    };
    int nq = (K - nh) >> 2;
    for (; nq >= 2; nq -= 2, quad += 2) {
        asm volatile("" : "+s"(rw));
        uint4 b1, v1, w1;
        quad_of(blk, vb, vb2, b1, v1, w1, quad + 1u);
        quad_of(b1, v1, w1, blk, vb, vb2, quad + 2u);
    }
    if (nq) {
        uint4 b1, v1, w1;
        quad_of(blk, vb, vb2, b1, v1, w1, quad + 1u);
        blk = b1;
        vb = v1;
        vb2 = w1;
        ++quad;
    }
    // the last K mod 4 steps (a partial quad): F, I already hold the first one's selectors
    for (int k = 0; k < ((K - nh) & 3); ++k) {
        const uint32_t w = word_of(blk, (uint32_t)k);
        if (k) sel(w, F, I);
        one(w, word_of(vb, (uint32_t)k), word_of(vb2, (uint32_t)k), F, I, step_off());
    }
    const uint64_t t1 = t0 + (uint64_t)K;
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    store_meta(A, i, t1, m, ep.x != ep0);
    if (ep.x != ep0) {
        ep.w = max_exp(last);
        A.ep[i] = ep;
        if (A.qsum) A.qsum[i] = 0.0;
    }
    if ((i & 63) == 0) A.clock[i >> 6] = t1;
    if constexpr (kSum) A.reward_sum[i] += rsum;
    if (i == 0) bump_count(A, t1);
}

__global__ __launch_bounds__(kBlock) void k_reset(uint4* board, uint32_t* meta, const uint64_t* clock,
                                                  int64_t n, uint64_t board_offset, uint32_t seed_lo,
                                                  uint32_t seed_hi, uint32_t p4_thresh,
                                                  uint32_t epoch, const uint8_t* mask) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (mask && !mask[i]) return;
    const Board b = fresh_board(
        draw(seed_lo, seed_hi, board_offset + (uint64_t)i, DOMAIN_RESET, epoch), p4_thresh);
    board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    meta[i] = 0u;                           // score
    meta[n + i] = (uint32_t)clock[i >> 6];  // a new episode starts at the running clock: 0 moves
}

// The {score, moves} pairs of ABI v4 (g2048_env_score_moves): out[i] = {score, clock - start}.
__global__ __launch_bounds__(kBlock) void k_score_moves(const uint32_t* meta, const uint64_t* clock,
                                                        int64_t n, uint2* out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    out[i] = make_uint2(meta[i], (uint32_t)clock[i >> 6] - meta[n + i]);
}

// available_moves_as_torch_unit_vector (src/board.py:128-135) of every board, as a bit mask.
__global__ __launch_bounds__(kBlock) void k_legal(const uint4* board, int64_t n, uint8_t* legal) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    legal[i] = (uint8_t)legal_mask(load_board(board[i]));
}

struct SampleArgs {
    const uint4* s;
    const uint4* s2;
    const uint8_t* a;
    const int32_t* r;
    const uint8_t* d;
    const unsigned long long* count;
    int64_t capacity;
    const int64_t* idx;
    int64_t batch;
    uint32_t seed_lo, seed_hi;
    uint64_t epoch;
    void* s_out;
    void* s2_out;
    int64_t* a_out;
    void* r_out;
    void* d_out;
    int64_t* idx_out;
    unsigned long long* err;
};

template <typename T>
__device__ __forceinline__ void store_exps(T* dst, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if constexpr (sizeof(T) == 4) {
        float4* o = reinterpret_cast<float4*>(dst);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = make_float4((float)(w[k] & 0xFFu), (float)((w[k] >> 8) & 0xFFu),
                               (float)((w[k] >> 16) & 0xFFu), (float)(w[k] >> 24));
    } else {
        double2* o = reinterpret_cast<double2*>(dst);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            o[2 * k] = make_double2((double)(w[k] & 0xFFu), (double)((w[k] >> 8) & 0xFFu));
            o[2 * k + 1] = make_double2((double)((w[k] >> 16) & 0xFFu), (double)(w[k] >> 24));
        }
    }
}

// sample_experiences + extract_samples_* (src/dqn_lib.py:33-84) for B rows at once.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sample(SampleArgs S) {
    const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (b >= S.batch) return;
    int64_t j;
    if (S.idx) {
        j = S.idx[b];
    } else {
        const uint4 u = philox10(make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32),
                                            (uint32_t)S.epoch,
                                            (uint32_t)(S.epoch >> 32) | (DOMAIN_SAMPLE << 30)),
                                 S.seed_lo, S.seed_hi);
        const unsigned long long x = ((unsigned long long)u.y << 32) | u.x;
        j = (int64_t)__umul64hi(x, *S.count);
    }
    if (j < 0 || j >= S.capacity) {  // np.random.randint never leaves range; a bad idx is counted
        atomicAdd(S.err, 1ull);
        j = 0;
    }
    if (S.idx_out) S.idx_out[b] = j;
    if (S.s_out) store_exps(reinterpret_cast<T*>(S.s_out) + 16 * b, S.s[j]);
    if (S.s2_out) store_exps(reinterpret_cast<T*>(S.s2_out) + 16 * b, S.s2[j]);
    if (S.a_out) S.a_out[b] = S.a[j];
    if (S.r_out) reinterpret_cast<T*>(S.r_out)[b] = (T)S.r[j];
    if (S.d_out) reinterpret_cast<T*>(S.d_out)[b] = (T)S.d[j];
}

// ------------------------------------------------------------------ host side
#define fail g2048_fail

#define G_HIP(expr)                                                                        \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(G2048_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                         \
    } while (0)

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

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

thread_local std::string g_err;

int g2048_fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

struct g2048_env {
    int64_t n = 0;
    uint64_t seed = 0, board_offset = 0;
    int device = 0;
    uint32_t flags = 0;
    uint8_t* board = nullptr;
    uint32_t* meta = nullptr;
    uint32_t* ep = nullptr;
    uint64_t* clock = nullptr;
    unsigned long long* err = nullptr;
    bool owns = false;
    uint32_t epoch = 0;
    g2048_episode* log = nullptr;
    int64_t log_slots = 0;
    double* qsum = nullptr;
};

struct g2048_replay {
    int64_t capacity = 0;
    int device = 0;
    uint8_t* s = nullptr;
    uint8_t* s2 = nullptr;
    uint8_t* a = nullptr;
    int32_t* r = nullptr;
    uint8_t* d = nullptr;
    unsigned long long* count = nullptr;
    unsigned long long* err = nullptr;
    bool owns = false;
};

namespace {

inline uint32_t p4_thresh(uint32_t flags) {
    return (flags & G2048_P4_10) ? 429496730u : 2147483648u;  // round(p * 2^32)
}

// The large-N instance of g2048_env_rollout: past ~1M boards the ring streams to HBM
// and the launch is store-bound; a kernel whose waves each compute AND store overlaps the two
// badly (with the store queue full, a SIMD's waves wait at their stores together: compute +
// stores ~ their sum).  Decoupled warp specialisation: workgroups of 512 threads, compute wave p
// (0-3) and store wave p + 4 own the same 64 boards and share a kD-step LDS ring of transitions.  No workgroup barrier
// inside the loop: the pair hands slots over through two LDS counters (produced / consumed steps,
// release / acquire at workgroup scope), so the compute wave runs up to kD steps ahead of its
// store wave and a store wave waiting on a full store queue stalls only itself.  Every wait is
// capped: a broken hand-over ends the loop and bumps the env's error counter (env.check_errors()
// raises) instead of hanging the GPU.
// kAux: the ring stores' cache-policy bits: 3 = sc0 | nt (4M x 16: 461 us against 478 with nt
// alone, 593 with sc0 alone).
// kD = 8: 78 KB of LDS, two workgroups per CU (4M x 16: 445 us against 694 for the five-wave
// k_rollout_lean; 4 or 12 steps: 622 / 652 us).  The same transitions, bit for bit.
struct alignas(16) PairSlot {
    uint4 s[64];
    uint4 s2[64];
    uint32_t r[64];
    uint8_t a[64];
    uint8_t d[64];
};

__device__ __forceinline__ bool wait_until(const uint32_t* c, uint32_t want) {
    // wave-uniform: every lane reads the same LDS word
    for (int spin = 0; spin < (1 << 20); ++spin) {
        if (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= want) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

template <bool kSum, bool kP410, int kD = 8, int kAux = 3>
__global__ __launch_bounds__(2 * kBlock) void k_rollout_ws(StepArgs A) {
    __shared__ uint4 s_dir[8];
    __shared__ PairSlot ring[4][kD];
    __shared__ uint32_t prod[4], cons[4];
    const bool storer = threadIdx.x >= kBlock;
    const int j = storer ? (int)threadIdx.x - kBlock : (int)threadIdx.x;
    const int pair = j >> 6, lane = j & 63;
    const int64_t i = (int64_t)blockIdx.x * kBlock + j;
    const bool live = i < A.n;
    uint64_t c0 = 0;
    if (live) c0 = A.clock[i >> 6];
    if (threadIdx.x < 8) s_dir[threadIdx.x] = reinterpret_cast<const uint4*>(&kDirNet[0][0][0])[threadIdx.x];
    if (threadIdx.x < 4) {
        prod[threadIdx.x] = 0u;
        cons[threadIdx.x] = 0u;
    }
    const uint64_t t0 = first_lane_u64(c0);
    const int K = A.k_steps > 0 ? A.k_steps : 0;
    __syncthreads();
    if (storer) {
        const uint32_t cap32 = (uint32_t)A.rb.capacity, n32 = (uint32_t)A.n;
        uint32_t soff = (uint32_t)ring_row(t0, A.rb.rows) * n32;
        __amdgpu_buffer_rsrc_t rw =
            __builtin_amdgcn_make_buffer_rsrc(A.rb.win, 0, (int)A.rb.win_bytes, 0x00020000);
        const uint32_t bl = (uint32_t)i;
        const uint32_t v_s = A.rb.o_s + 16u * bl, v_s2 = A.rb.o_s2 + 16u * bl;
        const uint32_t v_a = A.rb.o_a + bl, v_r = A.rb.o_r + 4u * bl, v_d = A.rb.o_d + bl;
        for (int s = 0; s < K; ++s) {
            if (!wait_until(&prod[pair], (uint32_t)s + 1u)) {
                if (lane == 0) atomicAdd(A.err, 1ull);  // never expected: surfaces as an env error
                break;
            }
            const PairSlot& B = ring[pair][s % kD];
            const uint4 sv = B.s[lane], s2v = B.s2[lane];
            const uint32_t rv = B.r[lane];
            const uint8_t av = B.a[lane], dv = B.d[lane];
            // the slot's reads are complete (the release below orders them) before it is freed
            if (lane == 0)
                __hip_atomic_store(&cons[pair], (uint32_t)s + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (live) {
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{sv.x, sv.y, sv.z, sv.w}, rw, v_s, soff * 16u, kAux);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{s2v.x, s2v.y, s2v.z, s2v.w}, rw, v_s2, soff * 16u, kAux);
                asm volatile("s_nop 1" ::"v"(sv.x), "v"(sv.y), "v"(sv.z), "v"(sv.w), "v"(s2v.x), "v"(s2v.y), "v"(s2v.z), "v"(s2v.w));
                __builtin_amdgcn_raw_buffer_store_b8(av, rw, v_a, soff, kAux);
                __builtin_amdgcn_raw_buffer_store_b32(rv, rw, v_r, soff * 4u, kAux);
                __builtin_amdgcn_raw_buffer_store_b8(dv, rw, v_d, soff, kAux);
            }
            soff = soff + n32 == cap32 ? 0u : soff + n32;
        }
        return;
    }
    Board b{0u, 0u, 0u, 0u};
    uint2 m = make_uint2(0, 0);
    uint4 ep = make_uint4(0, 0, 0, 0);
    if (live) {
        b = load_board(A.board[i]);
        m = load_meta(A, i, t0);
        ep = A.ep[i];
    }
    const uint64_t gid = A.board_offset + (uint64_t)i;
    const uint32_t p4 = A.p4_thresh;
    long long rsum = 0;
    const uint32_t ep0 = ep.x;
    Board last = b;
    const uint32_t k255 = opaque_255();
    uint4 blk = make_uint4(0, 0, 0, 0), vb = blk, vb2 = blk;
    bool ok = true;  // wave-uniform: false once a hand-over timed out
    for (int s = 0; s < K; ++s) {
        const uint64_t t = t0 + (uint64_t)s;
        if (s == 0 || (t & 3u) == 0u) {
            blk = draw(A.seed_lo, A.seed_hi, gid, DOMAIN_RANDOM, t >> 2);
            value_blocks<kP410>(A.seed_lo, A.seed_hi, gid, t >> 2, vb, vb2);
        }
        const uint32_t k = (uint32_t)t & 3u;
        const uint32_t w = word_of(blk, k), v = word_of(vb, k), v2 = word_of(vb2, k);
        const uint32_t a2 = (w >> 30) * 2u;
        // slot s % kD is free once the store wave has taken step s - kD
        if (s >= kD && !wait_until(&cons[pair], (uint32_t)(s - kD) + 1u)) {
            if (lane == 0) atomicAdd(A.err, 1ull);
            ok = false;
            break;
        }
        PairSlot& B = ring[pair][s % kD];
        B.s[lane] = make_uint4(b.r0, b.r1, b.r2, b.r3);
        bool done;
        const uint32_t r = lean_step(b, w, spawn_exp<kP410>(w, v, p4), s_dir[a2], s_dir[a2 + 1u], done, k255);
        m.x += r;
        m.y += 1u;
        if constexpr (kSum) rsum += r;
        B.s2[lane] = make_uint4(b.r0, b.r1, b.r2, b.r3);
        B.a[lane] = (uint8_t)(w >> 30);
        B.r[lane] = r;
        B.d[lane] = (uint8_t)done;
        if (lane == 0)
            __hip_atomic_store(&prod[pair], (uint32_t)s + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t dl = __builtin_amdgcn_ballot_w64(done);
        if (dl != 0u) {
            const Board f = fresh_board_w<kP410>(w, v, v2, p4);
            last.r0 = sel_lanes(dl, b.r0, last.r0);
            last.r1 = sel_lanes(dl, b.r1, last.r1);
            last.r2 = sel_lanes(dl, b.r2, last.r2);
            last.r3 = sel_lanes(dl, b.r3, last.r3);
            ep.x = sel_lanes(dl, ep.x + 1u, ep.x);
            ep.y = sel_lanes(dl, m.x, ep.y);
            ep.z = sel_lanes(dl, m.y, ep.z);
            b.r0 = sel_lanes(dl, f.r0, b.r0);
            b.r1 = sel_lanes(dl, f.r1, b.r1);
            b.r2 = sel_lanes(dl, f.r2, b.r2);
            b.r3 = sel_lanes(dl, f.r3, b.r3);
            m.x = sel_lanes(dl, 0u, m.x);
            m.y = sel_lanes(dl, 0u, m.y);
        }
    }
    // After a timed-out hand-over the wave leaves its boards, meta, episode counters and clock
    // at t0 (ring rows it handed over may be written; the env's error counter is set, so
    // check_errors() raises and the caller must reset the env).
    if (!live || !ok) return;
    const uint64_t t1 = t0 + (uint64_t)K;
    A.board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    store_meta(A, i, t1, m, ep.x != ep0);
    if (ep.x != ep0) {
        ep.w = max_exp(last);
        A.ep[i] = ep;
        if (A.qsum) A.qsum[i] = 0.0;
    }
    if ((i & 63) == 0) A.clock[i >> 6] = t1;
    if constexpr (kSum) A.reward_sum[i] += rsum;
    if (i == 0) bump_count(A, t1);
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int launch_reset(g2048_env* e, const uint8_t* mask, hipStream_t st) {
    DeviceGuard g(e->device);
    hipLaunchKernelGGL(k_reset, dim3(grid_for(e->n)), dim3(kBlock), 0, st,
                       reinterpret_cast<uint4*>(e->board), e->meta, e->clock, e->n,
                       e->board_offset, (uint32_t)e->seed, (uint32_t)(e->seed >> 32),
                       p4_thresh(e->flags), e->epoch, mask);
    G_HIP(hipGetLastError());
    e->epoch += 1;
    return G2048_OK;
}

int make_args(g2048_env* e, g2048_replay* rb, StepArgs& A) {
    std::memset(&A, 0, sizeof(A));
    A.board = reinterpret_cast<uint4*>(e->board);
    A.score = e->meta;
    A.start = e->meta + e->n;
    A.ep = reinterpret_cast<uint4*>(e->ep);
    A.clock = e->clock;
    A.n = e->n;
    A.board_offset = e->board_offset;
    A.seed_lo = (uint32_t)e->seed;
    A.seed_hi = (uint32_t)(e->seed >> 32);
    A.p4_thresh = p4_thresh(e->flags);
    A.flags = e->flags;
    A.err = e->err;
    A.log = e->log;
    A.log_slots = e->log_slots;
    A.qsum = e->qsum;
    if (rb) {
        if (rb->device != e->device)
            return fail(G2048_EINVAL, "replay on device %d, env on device %d", rb->device, e->device);
        if (rb->capacity < e->n || rb->capacity % e->n != 0)
            return fail(G2048_EINVAL, "replay capacity %lld must be a positive multiple of n=%lld",
                        (long long)rb->capacity, (long long)e->n);
        A.rb.s = reinterpret_cast<uint4*>(rb->s);
        A.rb.s2 = reinterpret_cast<uint4*>(rb->s2);
        A.rb.a = rb->a;
        A.rb.r = rb->r;
        A.rb.d = rb->d;
        A.rb.count = rb->count;
        A.rb.capacity = rb->capacity;
        A.rb.rows = rb->capacity / e->n;
        // the window: lowest section start to highest section end, when below 4 GiB
        const int64_t c = rb->capacity;
        const uintptr_t st[5] = {(uintptr_t)rb->s, (uintptr_t)rb->s2, (uintptr_t)rb->a,
                                 (uintptr_t)rb->r, (uintptr_t)rb->d};
        const uint64_t sz[5] = {16u * (uint64_t)c, 16u * (uint64_t)c, (uint64_t)c,
                                4u * (uint64_t)c, (uint64_t)c};
        uintptr_t lo = st[0], hi = st[0] + sz[0];
        for (int k = 1; k < 5; ++k) {
            lo = std::min(lo, st[k]);
            hi = std::max(hi, (uintptr_t)(st[k] + sz[k]));
        }
        if ((uint64_t)(hi - lo) < ((uint64_t)1 << 32)) {
            A.rb.win = reinterpret_cast<uint8_t*>(lo);
            A.rb.win_bytes = (uint32_t)(hi - lo);
            A.rb.o_s = (uint32_t)(st[0] - lo);
            A.rb.o_s2 = (uint32_t)(st[1] - lo);
            A.rb.o_a = (uint32_t)(st[2] - lo);
            A.rb.o_r = (uint32_t)(st[3] - lo);
            A.rb.o_d = (uint32_t)(st[4] - lo);
        }
    }
    return G2048_OK;
}

// Prefetch the episode counters with the board (k_step's kPre) when the extra 16 B are nearly
// free: the eps schedule reads the same 32 B sector anyway, a q-sum buffer is attached, or the
// batch is small enough to be latency-bound (measured: 64k boards -1 %; 4M boards, HBM-bound,
// +17 % per step with the prefetch).
constexpr int64_t kPrefetchMaxBoards = 1 << 18;

template <int MODE, bool kPre>
void launch_step_k(g2048_env* e, const StepArgs& A, hipStream_t st) {
    if (e->n <= kStepSmallMaxBoards) {
        constexpr int BS = kStepBlockSmall;
        const unsigned grid = (unsigned)((e->n + BS - 1) / BS);
        if (e->n % BS == 0)
            hipLaunchKernelGGL((k_step<MODE, true, kPre, BS>), dim3(grid), dim3(BS), 0, st, A.board,
                               A.score, A.ep, A.clock, A.board_offset, A.seed_lo, A.seed_hi,
                               A.p4_thresh, A.flags, A);
        else
            hipLaunchKernelGGL((k_step<MODE, false, kPre, BS>), dim3(grid), dim3(BS), 0, st, A.board,
                               A.score, A.ep, A.clock, A.board_offset, A.seed_lo, A.seed_hi,
                               A.p4_thresh, A.flags, A);
    } else if (e->n % kBlock == 0) {
        hipLaunchKernelGGL((k_step<MODE, true, kPre, kBlock>), dim3(grid_for(e->n)), dim3(kBlock), 0,
                           st, A.board, A.score, A.ep, A.clock, A.board_offset, A.seed_lo, A.seed_hi,
                           A.p4_thresh, A.flags, A);
    } else {
        hipLaunchKernelGGL((k_step<MODE, false, kPre, kBlock>), dim3(grid_for(e->n)), dim3(kBlock),
                           0, st, A.board, A.score, A.ep, A.clock, A.board_offset, A.seed_lo,
                           A.seed_hi, A.p4_thresh, A.flags, A);
    }
}

template <int MODE>
int launch_step(g2048_env* e, const StepArgs& A, void* stream) {
    DeviceGuard g(e->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (A.eps_decay > 0.0 || A.qsum || e->n <= kPrefetchMaxBoards)
        launch_step_k<MODE, true>(e, A, st);
    else
        launch_step_k<MODE, false>(e, A, st);
    G_HIP(hipGetLastError());
    return G2048_OK;
}

}  // namespace

// ------------------------------------------------------------------ extern "C" ABI
static int g2048_env_step_egreedy_impl(g2048_env* e, const void* q, int q_dtype,
                                       const double* eps_dev, double eps, double eps_decay,
                                       double eps_min, int32_t* reward, uint8_t* done,
                                       uint8_t* action_out, g2048_replay* rb, void* stream);

extern "C" {

const char* g2048_last_error(void) { return g_err.c_str(); }
int g2048_abi_version(void) { return G2048_ABI_VERSION; }

int g2048_env_wrap(g2048_env** out, int64_t n, uint64_t seed, uint64_t board_offset, int device_id,
                   uint32_t flags, uint8_t* board, uint32_t* meta, uint32_t* ep, uint64_t* clock,
                   int reset, void* stream) {
    if (!out || n <= 0) return fail(G2048_EINVAL, "env_wrap: need out != NULL and n > 0");
    if (n > G2048_MAX_BOARDS)
        return fail(G2048_EINVAL, "env_wrap: n = %lld boards exceeds G2048_MAX_BOARDS (%lld)",
                    (long long)n, (long long)G2048_MAX_BOARDS);
    if (!board || !meta || !ep || !clock || !aligned16(board) || !aligned16(ep) ||
        ((uintptr_t)meta & 7u) || ((uintptr_t)clock & 7u))
        return fail(G2048_EINVAL, "env_wrap: board/meta/ep/clock must be non-NULL, board/ep "
                                  "16-byte and meta/clock 8-byte aligned");
    if (flags & ~(uint32_t)(G2048_P4_10 | G2048_EGREEDY_FIXED | G2048_NO_AUTORESET))
        return fail(G2048_EINVAL, "env_wrap: unknown flags 0x%x", flags);
    DeviceGuard g(device_id);
    auto* e = new (std::nothrow) g2048_env;
    if (!e) return fail(G2048_ENOMEM, "env_wrap: host allocation failed");
    e->n = n;
    e->seed = seed;
    e->board_offset = board_offset;
    e->device = device_id;
    e->flags = flags;
    e->board = board;
    e->meta = meta;
    e->ep = ep;
    e->clock = clock;
    hipError_t he = hipMalloc(&e->err, sizeof(unsigned long long));
    if (he != hipSuccess) {
        delete e;
        return fail(G2048_ENOMEM, "env_wrap: hipMalloc(err): %s", hipGetErrorString(he));
    }
    he = hipMemsetAsync(e->err, 0, sizeof(unsigned long long), (hipStream_t)stream);
    if (he != hipSuccess) {
        g2048_env_destroy(e);
        return fail(G2048_EHIP, "env_wrap: %s", hipGetErrorString(he));
    }
    if (reset) {
        int rc = launch_reset(e, nullptr, (hipStream_t)stream);
        if (rc) {
            g2048_env_destroy(e);
            return rc;
        }
    }
    *out = e;
    return G2048_OK;
}

int g2048_env_create(g2048_env** out, int64_t n, uint64_t seed, uint64_t board_offset,
                     int device_id, uint32_t flags, void* stream) {
    if (!out || n <= 0) return fail(G2048_EINVAL, "env_create: need out != NULL and n > 0");
    if (n > G2048_MAX_BOARDS)
        return fail(G2048_EINVAL, "env_create: n = %lld boards exceeds G2048_MAX_BOARDS (%lld)",
                    (long long)n, (long long)G2048_MAX_BOARDS);
    DeviceGuard g(device_id);
    uint8_t* board = nullptr;
    uint32_t *meta = nullptr, *ep = nullptr;
    uint64_t* clock = nullptr;
    const int64_t groups = G2048_CLOCK_WORDS(n);
    auto release = [&]() {
        (void)hipFree(board);
        (void)hipFree(meta);
        (void)hipFree(ep);
        (void)hipFree(clock);
    };
    if (hipMalloc(&board, 16 * n) != hipSuccess || hipMalloc(&meta, 8 * n) != hipSuccess ||
        hipMalloc(&ep, 16 * n) != hipSuccess || hipMalloc(&clock, 8 * groups) != hipSuccess) {
        release();
        return fail(G2048_ENOMEM, "env_create: hipMalloc of %lld boards failed", (long long)n);
    }
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(meta, 0, 8 * n, st) != hipSuccess ||
        hipMemsetAsync(ep, 0, 16 * n, st) != hipSuccess ||
        hipMemsetAsync(clock, 0, 8 * groups, st) != hipSuccess) {
        release();
        return fail(G2048_EHIP, "env_create: hipMemsetAsync failed");
    }
    int rc = g2048_env_wrap(out, n, seed, board_offset, device_id, flags, board, meta, ep, clock,
                            1, stream);
    if (rc) {
        release();
        return rc;
    }
    (*out)->owns = true;
    return G2048_OK;
}

void g2048_env_destroy(g2048_env* e) {
    if (!e) return;
    DeviceGuard g(e->device);
    if (e->owns) {
        (void)hipFree(e->board);
        (void)hipFree(e->meta);
        (void)hipFree(e->ep);
        (void)hipFree(e->clock);
    }
    (void)hipFree(e->err);
    delete e;
}

int g2048_env_views(g2048_env* e, uint8_t** board, uint32_t** meta, uint32_t** ep,
                    uint64_t** clock) {
    if (!e) return fail(G2048_EINVAL, "env_views: NULL env");
    if (board) *board = e->board;
    if (meta) *meta = e->meta;
    if (ep) *ep = e->ep;
    if (clock) *clock = e->clock;
    return G2048_OK;
}

int64_t g2048_env_size(const g2048_env* e) { return e ? e->n : 0; }

int g2048_env_rng(const g2048_env* e, uint64_t* seed, uint64_t* board_offset) {
    if (!e || !seed || !board_offset) return fail(G2048_EINVAL, "env_rng: NULL argument");
    *seed = e->seed;
    *board_offset = e->board_offset;
    return G2048_OK;
}

int g2048_env_reset(g2048_env* e, const uint8_t* mask, void* stream) {
    if (!e) return fail(G2048_EINVAL, "env_reset: NULL env");
    return launch_reset(e, mask, (hipStream_t)stream);
}

int g2048_env_get_epoch(const g2048_env* e, uint32_t* epoch) {
    if (!e || !epoch) return fail(G2048_EINVAL, "env_get_epoch: NULL argument");
    *epoch = e->epoch;
    return G2048_OK;
}

int g2048_env_set_epoch(g2048_env* e, uint32_t epoch) {
    if (!e) return fail(G2048_EINVAL, "env_set_epoch: NULL env");
    e->epoch = epoch;
    return G2048_OK;
}

int g2048_env_set_episode_log(g2048_env* e, g2048_episode* log, int64_t slots_per_board,
                              double* qsum) {
    if (!e) return fail(G2048_EINVAL, "env_set_episode_log: NULL env");
    if (log && (slots_per_board <= 0 || slots_per_board > (1 << 20) || !qsum ||
                ((uintptr_t)log & 7u) || ((uintptr_t)qsum & 7u)))
        return fail(G2048_EINVAL,
                    "env_set_episode_log: need 0 < slots_per_board <= 2^20, qsum, 8-byte alignment");
    e->log = log;
    e->log_slots = log ? slots_per_board : 0;
    e->qsum = log ? qsum : nullptr;
    return G2048_OK;
}

int g2048_env_score_moves(g2048_env* e, uint32_t* out, void* stream) {
    if (!e || !out) return fail(G2048_EINVAL, "env_score_moves: NULL argument");
    if ((uintptr_t)out & 7u) return fail(G2048_EINVAL, "env_score_moves: out must be 8-byte aligned");
    DeviceGuard g(e->device);
    hipLaunchKernelGGL(k_score_moves, dim3(grid_for(e->n)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), e->meta, e->clock, e->n,
                       reinterpret_cast<uint2*>(out));
    G_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_env_legal_mask(g2048_env* e, uint8_t* legal, void* stream) {
    if (!e || !legal) return fail(G2048_EINVAL, "env_legal_mask: NULL argument");
    DeviceGuard g(e->device);
    hipLaunchKernelGGL(k_legal, dim3(grid_for(e->n)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint4*>(e->board), e->n, legal);
    G_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_env_step(g2048_env* e, const uint8_t* actions, int32_t* reward, uint8_t* done,
                   uint8_t* legal, g2048_replay* rb, void* stream) {
    if (!e) return fail(G2048_EINVAL, "env_step: NULL env");
    StepArgs A;
    int rc = make_args(e, rb, A);
    if (rc) return rc;
    A.actions = actions;
    A.reward = reward;
    A.done = done;
    A.legal_out = legal;
    return actions ? launch_step<MODE_ACTIONS>(e, A, stream) : launch_step<MODE_RANDOM>(e, A, stream);
}

int g2048_env_step_egreedy_schedule(g2048_env* e, const void* q, int q_dtype,
                                    double eps_decay_episodes, double eps_min, int32_t* reward,
                                    uint8_t* done, uint8_t* action_out, g2048_replay* rb,
                                    void* stream) {
    if (!(eps_decay_episodes > 0.0))
        return fail(G2048_EINVAL, "env_step_egreedy_schedule: eps_decay_episodes must be > 0");
    return g2048_env_step_egreedy_impl(e, q, q_dtype, nullptr, 0.0, eps_decay_episodes, eps_min,
                                       reward, done, action_out, rb, stream);
}

int g2048_env_step_egreedy(g2048_env* e, const void* q, int q_dtype, const double* eps_dev,
                           double eps, int32_t* reward, uint8_t* done, uint8_t* action_out,
                           g2048_replay* rb, void* stream) {
    return g2048_env_step_egreedy_impl(e, q, q_dtype, eps_dev, eps, 0.0, 0.0, reward, done,
                                       action_out, rb, stream);
}

static int g2048_env_step_egreedy_impl(g2048_env* e, const void* q, int q_dtype,
                                       const double* eps_dev, double eps, double eps_decay,
                                       double eps_min, int32_t* reward, uint8_t* done,
                                       uint8_t* action_out, g2048_replay* rb, void* stream) {
    if (!e || !q) return fail(G2048_EINVAL, "env_step_egreedy: NULL env or q");
    if (q_dtype != G2048_F32 && q_dtype != G2048_F64)
        return fail(G2048_EINVAL, "env_step_egreedy: q_dtype %d", q_dtype);
    if (!aligned16(q)) return fail(G2048_EINVAL, "env_step_egreedy: q must be 16-byte aligned");
    StepArgs A;
    int rc = make_args(e, rb, A);
    if (rc) return rc;
    A.q = q;
    A.eps_dev = eps_dev;
    A.eps = eps;
    A.eps_decay = eps_decay;
    A.eps_min = eps_min;
    A.reward = reward;
    A.done = done;
    A.action_out = action_out;
    return q_dtype == G2048_F32 ? launch_step<MODE_EG_F32>(e, A, stream)
                                : launch_step<MODE_EG_F64>(e, A, stream);
}

int g2048_env_step_egreedy_dense64(g2048_env* e, const g2048_dense64_params* p,
                                   const double* eps_dev, double eps, double eps_decay_episodes,
                                   double eps_min, int32_t* reward, uint8_t* done,
                                   uint8_t* action_out, g2048_replay* rb, float* q_out,
                                   void* stream) {
    if (!e || !p || !p->w1 || !p->b1 || !p->w2 || !p->b2)
        return fail(G2048_EINVAL, "env_step_egreedy_dense64: NULL env or parameter");
    if (q_out && !aligned16(q_out))
        return fail(G2048_EINVAL, "env_step_egreedy_dense64: q_out must be 16-byte aligned");
    StepArgs A;
    int rc = make_args(e, rb, A);
    if (rc) return rc;
    A.eps_dev = eps_dev;
    A.eps = eps;
    A.eps_decay = eps_decay_episodes > 0.0 ? eps_decay_episodes : 0.0;
    A.eps_min = eps_min;
    A.reward = reward;
    A.done = done;
    A.action_out = action_out;
    DeviceGuard g(e->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((e->n + 63) / 64);  // 64 boards per 2-wave workgroup
    if (e->n % 64 == 0)
        hipLaunchKernelGGL((k_step_dense64_split<true>), dim3(grid), dim3(128), 0, st, A, p->w1,
                           p->b1, p->w2, p->b2, q_out);
    else
        hipLaunchKernelGGL((k_step_dense64_split<false>), dim3(grid), dim3(128), 0, st, A, p->w1,
                           p->b1, p->w2, p->b2, q_out);
    G_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_env_step_egreedy_dense64_f64(g2048_env* e, const g2048_dense64_params_f64* p,
                                       const double* eps_dev, double eps,
                                       double eps_decay_episodes, double eps_min, int32_t* reward,
                                       uint8_t* done, uint8_t* action_out, g2048_replay* rb,
                                       double* q_out, void* stream) {
    if (!e || !p || !p->w1 || !p->b1 || !p->w2 || !p->b2)
        return fail(G2048_EINVAL, "env_step_egreedy_dense64_f64: NULL env or parameter");
    if (q_out && !aligned16(q_out))
        return fail(G2048_EINVAL, "env_step_egreedy_dense64_f64: q_out must be 16-byte aligned");
    StepArgs A;
    int rc = make_args(e, rb, A);
    if (rc) return rc;
    A.eps_dev = eps_dev;
    A.eps = eps;
    A.eps_decay = eps_decay_episodes > 0.0 ? eps_decay_episodes : 0.0;
    A.eps_min = eps_min;
    A.reward = reward;
    A.done = done;
    A.action_out = action_out;
    DeviceGuard g(e->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((e->n + 63) / 64);
    if (e->n % 64 == 0)
        hipLaunchKernelGGL((k_step_dense64_split64<true>), dim3(grid), dim3(128), 0, st, A, p->w1,
                           p->b1, p->w2, p->b2, q_out);
    else
        hipLaunchKernelGGL((k_step_dense64_split64<false>), dim3(grid), dim3(128), 0, st, A, p->w1,
                           p->b1, p->w2, p->b2, q_out);
    G_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_env_step_inject(g2048_env* e, const uint8_t* actions, const int8_t* spawn_idx,
                          const uint8_t* spawn_exp, int32_t* reward, uint8_t* done,
                          uint8_t* legal, void* stream) {
    if (!e || !actions || !spawn_idx || !spawn_exp)
        return fail(G2048_EINVAL, "env_step_inject: NULL argument");
    StepArgs A;
    int rc = make_args(e, nullptr, A);
    if (rc) return rc;
    A.actions = actions;
    A.spawn_idx = spawn_idx;
    A.spawn_exp = spawn_exp;
    A.reward = reward;
    A.done = done;
    A.legal_out = legal;
    return launch_step<MODE_INJECT>(e, A, stream);
}

int g2048_env_rollout(g2048_env* e, int32_t k_steps, g2048_replay* rb, int64_t* reward_sum,
                      void* stream) {
    if (!e || k_steps < 0) return fail(G2048_EINVAL, "env_rollout: NULL env or k_steps < 0");
    if (k_steps == 0) return G2048_OK;
    StepArgs A;
    int rc = make_args(e, rb, A);
    if (rc) return rc;
    A.k_steps = k_steps;
    A.reward_sum = reinterpret_cast<long long*>(reward_sum);
    DeviceGuard g(e->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // buffer-resource stores while the ring's sections fit one 4 GiB window
    const dim3 grid(grid_for(e->n)), block(kBlock);
    if (!rb) {
        if (reward_sum) hipLaunchKernelGGL((k_rollout<false, false, true>), grid, block, 0, st, A);
        else hipLaunchKernelGGL((k_rollout<false, false, false>), grid, block, 0, st, A);
    } else if (A.rb.win_bytes && !A.log && !(A.flags & G2048_NO_AUTORESET)) {
        // the headline case
        const bool p410 = (A.flags & G2048_P4_10) != 0u, qr = A.rb.rows % 4 == 0;
        // from 256k boards on the launch is store-bound: the warp-specialised
        // k_rollout_ws (compute and store waves decoupled by an LDS ring) runs 4M x 16 in 445 us
        // against 694 for the five-wave k_rollout_lean, 1M x 64 in 524 against 674, 256k x 64 in
        // 124 against 147; at 64k it loses (42 us against 28: one compute wave per SIMD there)
        const bool big = A.n >= (1 << 18);
        // (the p(4) = 0.1 instances carry two more Philox blocks per quad: under the four-wave
        // register cap they spilled, so they take a three-wave cap -- at 64k boards the kernel
        // runs one wave per SIMD anyway)
// (ring stores with the sc1 cache-policy bit: 64k x 64 25.1 us against 28.1 with none, 27.5
// with sc0, 28.3-30.0 with nt; tools/rollexp.hip, profiles/r03/rollexp_cachepolicy_*)
#define G2048_LEAN(S, P, Q) hipLaunchKernelGGL((k_rollout_lean<S, P, Q, 0x1F, (P) ? 3 : 4, kRingSc1>), grid, block, 0, st, A)
#define G2048_WS(S, P) hipLaunchKernelGGL((k_rollout_ws<S, P>), grid, dim3(2 * kBlock), 0, st, A)
        if (big) {
            if (reward_sum) { if (p410) G2048_WS(true, true); else G2048_WS(true, false); }
            else { if (p410) G2048_WS(false, true); else G2048_WS(false, false); }
        } else if (reward_sum) {
            if (p410) { if (qr) G2048_LEAN(true, true, true); else G2048_LEAN(true, true, false); }
            else { if (qr) G2048_LEAN(true, false, true); else G2048_LEAN(true, false, false); }
        } else {
            if (p410) { if (qr) G2048_LEAN(false, true, true); else G2048_LEAN(false, true, false); }
            else { if (qr) G2048_LEAN(false, false, true); else G2048_LEAN(false, false, false); }
        }
#undef G2048_WS
#undef G2048_LEAN
    } else if (A.rb.win_bytes) {
        if (reward_sum) hipLaunchKernelGGL((k_rollout<true, true, true>), grid, block, 0, st, A);
        else hipLaunchKernelGGL((k_rollout<true, true, false>), grid, block, 0, st, A);
    } else {
        if (reward_sum) hipLaunchKernelGGL((k_rollout<true, false, true>), grid, block, 0, st, A);
        else hipLaunchKernelGGL((k_rollout<true, false, false>), grid, block, 0, st, A);
    }
    G_HIP(hipGetLastError());
    return G2048_OK;
}

int g2048_env_error_count(g2048_env* e, int64_t* count, void* stream) {
    if (!e || !count) return fail(G2048_EINVAL, "env_error_count: NULL argument");
    DeviceGuard g(e->device);
    hipStream_t st = (hipStream_t)stream;
    unsigned long long h = 0;
    G_HIP(hipMemcpyAsync(&h, e->err, sizeof(h), hipMemcpyDeviceToHost, st));
    G_HIP(hipStreamSynchronize(st));
    G_HIP(hipMemsetAsync(e->err, 0, sizeof(h), st));
    *count = (int64_t)h;
    return G2048_OK;
}

int g2048_replay_wrap(g2048_replay** out, int64_t capacity, int device_id, uint8_t* s,
                      uint8_t* s2, uint8_t* a, int32_t* r, uint8_t* d, uint64_t* count) {
    if (!out || capacity <= 0) return fail(G2048_EINVAL, "replay_wrap: need capacity > 0");
    if (!s || !s2 || !a || !r || !d || !count || !aligned16(s) || !aligned16(s2))
        return fail(G2048_EINVAL, "replay_wrap: NULL buffer or s/s2 not 16-byte aligned");
    DeviceGuard g(device_id);
    auto* rb = new (std::nothrow) g2048_replay;
    if (!rb) return fail(G2048_ENOMEM, "replay_wrap: host allocation failed");
    rb->capacity = capacity;
    rb->device = device_id;
    rb->s = s;
    rb->s2 = s2;
    rb->a = a;
    rb->r = r;
    rb->d = d;
    rb->count = reinterpret_cast<unsigned long long*>(count);
    if (hipMalloc(&rb->err, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(rb->err, 0, sizeof(unsigned long long)) != hipSuccess) {
        delete rb;
        return fail(G2048_ENOMEM, "replay_wrap: hipMalloc(err) failed");
    }
    *out = rb;
    return G2048_OK;
}

int g2048_replay_create(g2048_replay** out, int64_t capacity, int device_id, void* stream) {
    if (!out || capacity <= 0) return fail(G2048_EINVAL, "replay_create: need capacity > 0");
    DeviceGuard g(device_id);
    // one allocation, 256-byte aligned sections: s | s2 | r | a | d | count, each one
    // G2048_REPLAY_SECTION_PAD bytes further (include/g2048.h: the HBM channel spread of the
    // five store streams)
    auto up = [](int64_t x) { return ((x + 255) & ~(int64_t)255) + G2048_REPLAY_SECTION_PAD; };
    const int64_t o_s2 = up(16 * capacity), o_r = o_s2 + up(16 * capacity);
    const int64_t o_a = o_r + up(4 * capacity), o_d = o_a + up(capacity);
    const int64_t o_c = o_d + up(capacity), total = o_c + 256;
    uint8_t* base = nullptr;
    if (hipMalloc(&base, total) != hipSuccess)
        return fail(G2048_ENOMEM, "replay_create: hipMalloc(%lld) failed", (long long)total);
    if (hipMemsetAsync(base, 0, total, (hipStream_t)stream) != hipSuccess) {
        (void)hipFree(base);
        return fail(G2048_EHIP, "replay_create: hipMemsetAsync failed");
    }
    int rc = g2048_replay_wrap(out, capacity, device_id, base, base + o_s2, base + o_a,
                               reinterpret_cast<int32_t*>(base + o_r), base + o_d,
                               reinterpret_cast<uint64_t*>(base + o_c));
    if (rc) {
        (void)hipFree(base);
        return rc;
    }
    (*out)->owns = true;
    return G2048_OK;
}

void g2048_replay_destroy(g2048_replay* rb) {
    if (!rb) return;
    DeviceGuard g(rb->device);
    if (rb->owns) (void)hipFree(rb->s);
    (void)hipFree(rb->err);
    delete rb;
}

int g2048_replay_views(g2048_replay* rb, uint8_t** s, uint8_t** s2, uint8_t** a, int32_t** r,
                       uint8_t** d, uint64_t** count) {
    if (!rb) return fail(G2048_EINVAL, "replay_views: NULL replay");
    if (s) *s = rb->s;
    if (s2) *s2 = rb->s2;
    if (a) *a = rb->a;
    if (r) *r = rb->r;
    if (d) *d = rb->d;
    if (count) *count = reinterpret_cast<uint64_t*>(rb->count);
    return G2048_OK;
}

int g2048_replay_sample_encode(g2048_replay* rb, const int64_t* idx, int64_t batch, uint64_t seed,
                               uint64_t epoch, int dtype, void* s_out, void* s2_out,
                               int64_t* a_out, void* r_out, void* d_out, int64_t* idx_out,
                               void* stream) {
    if (!rb || batch <= 0) return fail(G2048_EINVAL, "replay_sample_encode: NULL rb or batch <= 0");
    if (dtype != G2048_F32 && dtype != G2048_F64)
        return fail(G2048_EINVAL, "replay_sample_encode: dtype %d", dtype);
    if ((s_out && !aligned16(s_out)) || (s2_out && !aligned16(s2_out)))
        return fail(G2048_EINVAL, "replay_sample_encode: s/s2 outputs must be 16-byte aligned");
    SampleArgs S;
    std::memset(&S, 0, sizeof(S));
    S.s = reinterpret_cast<const uint4*>(rb->s);
    S.s2 = reinterpret_cast<const uint4*>(rb->s2);
    S.a = rb->a;
    S.r = rb->r;
    S.d = rb->d;
    S.count = rb->count;
    S.capacity = rb->capacity;
    S.idx = idx;
    S.batch = batch;
    S.seed_lo = (uint32_t)seed;
    S.seed_hi = (uint32_t)(seed >> 32);
    S.epoch = epoch;
    S.s_out = s_out;
    S.s2_out = s2_out;
    S.a_out = a_out;
    S.r_out = r_out;
    S.d_out = d_out;
    S.idx_out = idx_out;
    S.err = rb->err;
    DeviceGuard g(rb->device);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == G2048_F32)
        hipLaunchKernelGGL(k_sample<float>, dim3(grid_for(batch)), dim3(kBlock), 0, st, S);
    else
        hipLaunchKernelGGL(k_sample<double>, dim3(grid_for(batch)), dim3(kBlock), 0, st, S);
    G_HIP(hipGetLastError());
    return G2048_OK;
}

}  // extern "C"
