// g2048_qnet.hip -- fused forward of the reference conv Q-network on gfx950 f32 MFMA.
//
// Net (src/configs/double_dqn_conv.py:19-28): Conv2d(1,64,2) ReLU Conv2d(64,64,2) ReLU Flatten
// Linear(256,64) ReLU Linear(64,4).  Input = the board's 16 log2 exponents (log_scale(),
// src/board.py:224-231) read straight from u8 rows -- optionally gathered through replay
// indices, so sample_experiences + extract_samples_conv + forward are one launch.
//
// Every launch is persistent: a workgroup (256 threads, 4 waves, one per CU) stages the net
// once and loops over 16-board tiles; conv2 runs as nine Winograd-domain GEMMs on
// v_mfma_f32_16x16x4_f32 (layout and numerics: see the persist namespace below).
// Numerics: f32 in / f32 accumulate; results differ from torch's fp32 GEMMs by summation order
// and the Winograd transforms' adds (tests: rtol 2e-5 vs torch fp32 and fp64).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"
#include "g2048_convnet.hpp"

namespace {

using g2048::cnet::NetW;
using g2048::cnet::NT;

struct ConvNetArgs {
    const float* w1;   // [64][1][2][2]
    const float* b1;   // [64]
    const float* w2;   // [64][64][2][2]
    const float* b2;   // [64]
    const float* wf1;  // [64][256]
    const float* bf1;  // [64]
    const float* wf2;  // [4][64]
    const float* bf2;  // [4]
    const uint8_t* rows;   // [*][16] u8 boards
    const int64_t* idx;    // row of board b (nullptr: b)
    int64_t n;
    float* q;              // [n][4]
};

// Phase profiler (tools/prof_forward.hip builds with G2048_PHASE_PROF): thread 0 of workgroup 0
// accumulates s_memtime deltas between the tile's barriers.
#ifdef G2048_PHASE_PROF
__device__ unsigned long long g2048_phase_ticks[8];
#define PHASE_BEGIN() unsigned long long phase_t0_ = __builtin_amdgcn_s_memtime()
#define PHASE(k)                                                          \
    do {                                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                        \
            const unsigned long long n_ = __builtin_amdgcn_s_memtime();   \
            g2048_phase_ticks[k] += n_ - phase_t0_;                       \
            phase_t0_ = n_;                                               \
        }                                                                 \
    } while (0)
#else
#define PHASE_BEGIN()
#define PHASE(k)
#endif

// ---------------------------------------------------------------------------------------------
// Persistent kernels (every conv forward, Double-DQN targets): a workgroup stages a net once
// and then runs 16-board tiles through the blocks of g2048_convnet.hpp (conv1 + Winograd input
// transform, conv2 as nine Winograd-domain GEMMs with U in VGPRs, fc1 with fc1_w in LDS), then
// fc2 over all 256 threads.  On gfx950 a VALU op between f32 MFMAs is not hidden
// (tools/prof_forward.hip: +4 cycles per op, ~12 when the ops form dependent chains), so the
// MFMA loops carry no VALU at all.
namespace persist {
using namespace g2048::cnet;
constexpr int TMAX = 8;    // tiles per workgroup in the targets kernel
constexpr int OFF_X = 0;                          // [TMAX][S][16] boards (exponents as floats)
constexpr int OFF_B2 = OFF_X + TMAX * S * 16;     // 64
constexpr int OFF_BF1 = OFF_B2 + 64;              // 64
constexpr int OFF_WF2 = OFF_BF1 + 64;             // [4][WF2S]
constexpr int OFF_BF2 = OFF_WF2 + 4 * WF2S;       // 4
constexpr int OFF_WF1 = OFF_BF2 + 4;              // [64][WF1S]
constexpr int OFF_V = OFF_WF1 + 64 * WF1S;        // [9][S][VS]
constexpr int OFF_H2 = OFF_V + 9 * VXI;
constexpr int OFF_F = OFF_H2 + S * H2S;
constexpr int OFF_Q = OFF_F + S * FS;             // [2 TMAX][S][4] Q of the tiles (two nets)
constexpr int FLOATS = OFF_Q + 2 * TMAX * S * 4;
static_assert(OFF_WF1 % 4 == 0 && OFF_V % 4 == 0 && OFF_H2 % 4 == 0 && OFF_F % 4 == 0 &&
                  OFF_WF2 % 4 == 0 && OFF_Q % 4 == 0,
              "b128 alignment");
static_assert(FLOATS * 4 <= 156 * 1024, "LDS budget (persistent kernels, + the sample index)");

// Stage net W: U (forward layout) + conv1 into registers, fc1_w + small tensors into LDS.  All
// global loads are issued before the first LDS store (one memory round trip).  Starts and ends
// with __syncthreads().
__device__ __forceinline__ void stage(const NetW& W, float* lds, Regs& R) {
    const int t = threadIdx.x;
    PHASE_BEGIN();
    load_u_fwd(W.w2, R);
    load_conv1(W, R);
    const float b2 = t < 64 ? W.b2[t] : 0.f, bf1 = t < 64 ? W.bf1[t] : 0.f;
    const float wf2 = W.wf2[t], bf2 = t < 4 ? W.bf2[t] : 0.f;
    float f[64];  // fc1_w[i][t], i = 0..63
#pragma unroll
    for (int i = 0; i < 64; ++i) f[i] = W.wf1[i * NT + t];
    __syncthreads();  // previous users of the LDS weight areas are done
    PHASE(4);
    if (t < 64) {
        lds[OFF_B2 + t] = b2;
        lds[OFF_BF1 + t] = bf1;
    }
    lds[OFF_WF2 + (t >> 6) * WF2S + (t & 63)] = wf2;
    if (t < 4) lds[OFF_BF2 + t] = bf2;
    store_fc1(f, lds + OFF_WF1);
    __syncthreads();
    PHASE(5);
}

// fc2 of the tile whose f is in LDS -> qs[16][4] (LDS): output o = t >> 2 (board o >> 2, action
// o & 3), part p = t & 3 sums 16 units, then a 4-lane shuffle sum.
__device__ __forceinline__ void fc2_lds(const float* lds, float* qs) {
    const int t = threadIdx.x;
    const int o = t >> 2, p = t & 3, s = o >> 2, a = o & 3;
    const f32x4* fr = reinterpret_cast<const f32x4*>(lds + OFF_F + s * FS + 16 * p);
    const f32x4* wr = reinterpret_cast<const f32x4*>(lds + OFF_WF2 + a * WF2S + 16 * p);
    f32x4 pv = f32x4{0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const f32x4 f = fr[j], w = wr[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) pv[e] = fmaf(w[e], f[e], pv[e]);
    }
    float v = (pv[0] + pv[1]) + (pv[2] + pv[3]);
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    if (p == 0) qs[o] = v + lds[OFF_BF2 + a];
}

// Q of T >= 1 tiles whose boards sit in xs (tile k at k*S*16; visible, net staged) -> qdst + k*S*4,
// pipelined as k_conv_forward_pipe (two barriers per tile).  Ends with __syncthreads().
__device__ __forceinline__ void tiles_pipe(float* lds, const Regs& R, int T, float* qdst) {
    const float* xs = lds + OFF_X;
    conv1_v(xs, lds + OFF_V, R);
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        conv2_h2(lds + OFF_V, lds + OFF_H2, lds + OFF_B2, R);
        if (k > 0) fc2_lds(lds, qdst + (k - 1) * S * 4);
        __syncthreads();
        fc1_f(lds + OFF_H2, lds + OFF_WF1, lds + OFF_BF1, lds + OFF_F);
        if (k + 1 < T) conv1_v(xs + (k + 1) * S * 16, lds + OFF_V, R);
        __syncthreads();
    }
    fc2_lds(lds, qdst + (T - 1) * S * 4);
    __syncthreads();
}
}  // namespace persist

// fc2 of a tile straight to global Q: thread (o = t >> 2, part p = t & 3) sums 16 units; the
// float sequence of fc2_lds.
__device__ __forceinline__ void persist_fc2_store(const float* lds, float* q, int64_t b0,
                                                  int64_t n) {
    namespace P = persist;
    const int t = threadIdx.x;
    const int o = t >> 2, p = t & 3, s = o >> 2, a = o & 3;
    const P::f32x4* fr = reinterpret_cast<const P::f32x4*>(lds + P::OFF_F + s * P::FS + 16 * p);
    const P::f32x4* wr = reinterpret_cast<const P::f32x4*>(lds + P::OFF_WF2 + a * P::WF2S + 16 * p);
    P::f32x4 pv = P::f32x4{0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const P::f32x4 f = fr[j], w = wr[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) pv[e] = fmaf(w[e], f[e], pv[e]);
    }
    float v = (pv[0] + pv[1]) + (pv[2] + pv[3]);
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    if (p == 0 && b0 + s < n) q[b0 * 4 + o] = v + lds[P::OFF_BF2 + a];
}

// The same fc2 with board s of the tile at global row c0 + rows[s] (s < nb).
__device__ __forceinline__ void persist_fc2_scatter(const float* lds, float* q, int64_t c0,
                                                    const int32_t* rows, int nb) {
    namespace P = persist;
    const int t = threadIdx.x;
    const int o = t >> 2, p = t & 3, s = o >> 2, a = o & 3;
    const P::f32x4* fr = reinterpret_cast<const P::f32x4*>(lds + P::OFF_F + s * P::FS + 16 * p);
    const P::f32x4* wr = reinterpret_cast<const P::f32x4*>(lds + P::OFF_WF2 + a * P::WF2S + 16 * p);
    P::f32x4 pv = P::f32x4{0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const P::f32x4 f = fr[j], w = wr[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) pv[e] = fmaf(w[e], f[e], pv[e]);
    }
    float v = (pv[0] + pv[1]) + (pv[2] + pv[3]);
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    if (p == 0 && s < nb) q[(c0 + rows[s]) * 4 + a] = v + lds[P::OFF_BF2 + a];
}

// The rollout's Q over all n boards (g2048_convnet_forward): 256 workgroups stage the net once
// and loop over 16-board tiles, software-pipelined over two barriers per tile instead of four:
//   [conv2(k) ; fc2(k-1) -> Q]  sync  [fc1(k) ; conv1 + V(k+1)]  sync
// (V is free once conv2(k) has read it, h2 once fc1(k) has; fc2 reads f, which the next fc1
// rewrites only after the next sync).  Boards are double-buffered in xs and loaded two tiles
// ahead.  Same float sequence per board as conv1_v, conv2_h2, fc1_f and fc2_lds in sequence.
__global__ __launch_bounds__(NT) void k_conv_forward_pipe(ConvNetArgs A) {
    namespace P = persist;
    __shared__ __attribute__((aligned(16))) float lds[P::FLOATS];
    const int t = threadIdx.x;
    const NetW W{A.w1, A.b1, A.w2, A.b2, A.wf1, A.bf1, A.wf2, A.bf2};
    P::Regs R;
    const int64_t ntiles = (A.n + P::S - 1) / P::S;
    const int64_t G = gridDim.x;
    auto load_word = [&](int64_t tile) -> uint32_t {
        const int64_t b = tile * P::S + (t >> 2);
        if (t >= P::S * 4 || tile >= ntiles || b >= A.n) return 0u;
        return reinterpret_cast<const uint32_t*>(A.rows)[(A.idx ? A.idx[b] : b) * 4 + (t & 3)];
    };
    float* xs0 = lds + P::OFF_X;
    float* xs1 = lds + P::OFF_X + P::S * 16;
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    uint32_t w0 = load_word(tile), w1 = load_word(tile + G);
    P::stage(W, lds, R);
    if (t < P::S * 4) {
        P::put_word(xs0, t, w0);
        P::put_word(xs1, t, w1);
    }
    uint32_t wn = load_word(tile + 2 * G);  // boards of the tile after next
    __syncthreads();
    P::conv1_v(xs0, lds + P::OFF_V, R);
    __syncthreads();
    int64_t prev = -1;  // tile whose fc2 is pending
    for (int k = 0; tile < ntiles; ++k, tile += G) {
        P::conv2_h2(lds + P::OFF_V, lds + P::OFF_H2, lds + P::OFF_B2, R);
        if (prev >= 0) persist_fc2_store(lds, A.q, prev * P::S, A.n);
        __syncthreads();
        P::fc1_f(lds + P::OFF_H2, lds + P::OFF_WF1, lds + P::OFF_BF1, lds + P::OFF_F);
        if (tile + G < ntiles) P::conv1_v((k & 1) ? xs0 : xs1, lds + P::OFF_V, R);
        // xs of tile k is free: it takes the tile after next
        if (t < P::S * 4) P::put_word((k & 1) ? xs1 : xs0, t, wn);
        wn = load_word(tile + 3 * G);
        __syncthreads();
        prev = tile;
    }
    persist_fc2_store(lds, A.q, prev * P::S, A.n);
}

// The rollout's Q restricted to the boards whose next eps-greedy step is greedy
// (g2048_convnet_forward_greedy).  epsilon_greedy_policy evaluates the model only on that branch
// (src/dqn_lib.py:20-24), so early in the eps schedule most of the forward is skipped.
// Workgroup w owns the contiguous boards [w*chunk, (w+1)*chunk).  Per window of GW boards it
// repeats the step kernel's explore draw for each (same Philox block, same eps), appends the
// greedy ones to an LDS queue (ballot + popcount), then runs full 16-board tiles of the queue
// (the next tile's boards loaded during the current one) and scatters Q to the boards' own rows;
// fewer than 16 left over carry into the next window, and the last window runs a partial tile.
// The net is staged on the first tile only: a workgroup whose boards all explore never loads
// it.  Rows of explorers are not written.  Q of a board does not depend on its tile mates, so
// the rows written are bitwise those of g2048_convnet_forward.
struct GreedyArgs {
    ConvNetArgs net;        // rows = the env's boards, n = its size, q = [n][4]
    const uint64_t* clock;  // [ceil(n/64)] step clocks: the draw's counter (board i: clock[i/64])
    const uint32_t* ep;     // [n][4]: ep[4i] = episodes (the schedule's e)
    uint64_t board_offset;  // global id of board 0
    uint32_t seed_lo, seed_hi;
    const double* eps_dev;
    double eps, eps_decay, eps_min;
    int64_t chunk;
};

constexpr int GW = 4 * NT;       // boards selected per window (4 per thread)
constexpr int GQ = GW + 16;      // queue: a window + the carried remainder

__global__ __launch_bounds__(NT) void k_conv_forward_greedy(GreedyArgs G) {
    namespace P = persist;
    __shared__ __attribute__((aligned(16))) float lds[P::FLOATS];
    __shared__ int32_t queue[GQ];  // board - c0 of each selected board, in board order
    __shared__ int32_t wcnt[4][4];  // [k][wave] greedy count
    const ConvNetArgs& A = G.net;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const NetW W{A.w1, A.b1, A.w2, A.b2, A.wf1, A.bf1, A.wf2, A.bf2};
    P::Regs R;
    bool staged = false;
    const int64_t c0 = (int64_t)blockIdx.x * G.chunk;
    const int64_t c1 = c0 + G.chunk < A.n ? c0 + G.chunk : A.n;
    const uint32_t* rows32 = reinterpret_cast<const uint32_t*>(A.rows);
    float* xs0 = lds + P::OFF_X;
    float* xs1 = lds + P::OFF_X + P::S * 16;
    // word t & 3 of board t >> 2 of the tile at queue[h], nb boards (thread t < 64)
    auto load_word = [&](int h, int nb) -> uint32_t {
        if (t >= P::S * 4 || (t >> 2) >= nb) return 0u;
        return rows32[(c0 + queue[h + (t >> 2)]) * 4 + (t & 3)];
    };
    int qn = 0;  // queue length (uniform)
    for (int64_t w0 = c0; w0 < c1; w0 += GW) {
        const bool last = w0 + GW >= c1;
        uint64_t tt[4];
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = w0 + k * NT + t;
            tt[k] = 0u;
            e[k] = 0u;
            if (i < c1) {
                tt[k] = G.clock[i >> 6];
                if (G.eps_decay > 0.0) e[k] = G.ep[4 * i];
            }
        }
        uint64_t bal[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = w0 + k * NT + t;
            bool g = false;
            if (i < c1) {
                const uint4 u = g2048::draw(G.seed_lo, G.seed_hi, G.board_offset + (uint64_t)i,
                                            g2048::DOMAIN_STEP, tt[k]);
                g = !g2048::explores(u.y, g2048::step_eps(G.eps_decay, G.eps_min, G.eps_dev,
                                                          G.eps, e[k]));
            }
            bal[k] = __ballot(g);
            if (lane == 0) wcnt[k][wv] = __popcll(bal[k]);
        }
        __syncthreads();
        const uint64_t below = (1ull << lane) - 1ull;
        int base = qn;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) {
                const int c = wcnt[k][ww];
                if (ww == wv && ((bal[k] >> lane) & 1ull))
                    queue[base + __popcll(bal[k] & below)] = (int32_t)(w0 + k * NT + t - c0);
                base += c;
            }
        }
        qn = base;
        __syncthreads();
        // the window's tiles: full ones, plus the partial rest in the last window
        const int nt = last ? (qn + P::S - 1) / P::S : qn / P::S;
        if (nt == 0) continue;  // < 16 selected so far: carried as they are
        auto nb_of = [&](int j) { return qn - j * P::S < P::S ? qn - j * P::S : P::S; };
        auto word_of = [&](int j) -> uint32_t { return j < nt ? load_word(j * P::S, nb_of(j)) : 0u; };
        // pipelined as k_conv_forward_pipe: [conv2(j) ; fc2(j-1) -> Q] sync [fc1(j) ; conv1(j+1)]
        const uint32_t wa = word_of(0), wb = word_of(1);
        if (!staged) {
            P::stage(W, lds, R);
            staged = true;
        }
        if (t < P::S * 4) {
            P::put_word(xs0, t, wa);
            P::put_word(xs1, t, wb);
        }
        uint32_t wn = word_of(2);
        __syncthreads();
        P::conv1_v(xs0, lds + P::OFF_V, R);
        __syncthreads();
        for (int j = 0; j < nt; ++j) {
            P::conv2_h2(lds + P::OFF_V, lds + P::OFF_H2, lds + P::OFF_B2, R);
            if (j > 0) persist_fc2_scatter(lds, A.q, c0, queue + (j - 1) * P::S, nb_of(j - 1));
            __syncthreads();
            P::fc1_f(lds + P::OFF_H2, lds + P::OFF_WF1, lds + P::OFF_BF1, lds + P::OFF_F);
            if (j + 1 < nt) P::conv1_v((j & 1) ? xs0 : xs1, lds + P::OFF_V, R);
            if (t < P::S * 4) P::put_word((j & 1) ? xs1 : xs0, t, wn);
            wn = word_of(j + 3);
            __syncthreads();
        }
        persist_fc2_scatter(lds, A.q, c0, queue + (nt - 1) * P::S, nb_of(nt - 1));
        const int h = qn < nt * P::S ? qn : nt * P::S;
        const int rem = qn - h;  // < 16 (0 after the last window)
        const int v = t < rem ? queue[h + t] : 0;
        __syncthreads();
        if (t < rem) queue[t] = v;
        qn = rem;
        __syncthreads();
    }
}

// Double-DQN targets for a minibatch (src/dqn_lib.py:67-68,125-132), one launch:
//   idx_b = uniform row of the ring (Philox, epoch = the learner's update counter) or idx_in,
//   a*_b  = argmax_a Q_online(s'_b)  (first index on ties, torch.argmax),
//   y_b   = r_b + ((1 - d_b) * float32(gamma)) * Q_target(s'_b, a*_b)   (vanilla: max_a Q_target)
struct TargetArgs {
    NetW on, tg;
    const uint8_t* s2;
    const int32_t* r;
    const uint8_t* d;
    const unsigned long long* count;
    const unsigned long long* epoch;
    const int64_t* idx_in;
    int64_t batch;
    uint32_t seed_lo, seed_hi;
    float gamma;
    int double_dqn;
    int64_t* idx_out;
    float* y;
    // split roles (g2048_convnet_update, Double DQN): workgroups [0, G) run the online net and
    // write a*, workgroups [G, 2G) the target net and write Q_target(s') with (float)r and the
    // discount; the train launch forms y from them.  nullptr: each workgroup runs both nets.
    int32_t* astar;   // [B]
    float4* qtg;      // [B] Q_target(s'_b, .)
    float2* rdisc;    // [B] ((float)r_b, (1 - d_b) * gamma)
};

// torch.argmax over 4 Q-values: the first index wins ties, the first NaN wins over numbers.
__device__ __forceinline__ int argmax4_first(const float* q) {
    return (int)g2048::argmax4_torch(q[0], q[1], q[2], q[3]);
}

// Each workgroup owns up to TMAX 16-sample tiles (tile = blockIdx.x + k*gridDim.x): it draws
// their indices and loads their s' rows once, runs them through the online net (Q kept in
// LDS), stages the target net and runs them again, then writes y.  With split roles (A.qtg)
// the grid is two halves over the same tiles, each staging ONE net for twice the tiles: one
// staging per workgroup instead of two.
__global__ __launch_bounds__(NT) void k_conv_targets_persist(TargetArgs A) {
    namespace P = persist;
    __shared__ __attribute__((aligned(16))) float lds[P::FLOATS];
    __shared__ int64_t sidx[P::TMAX * P::S];
    const int t = threadIdx.x;
    // roles: 0 = online net only, 1 = target net only, 2 = both (no split)
    const bool split = A.qtg != nullptr;
    const int G = split ? (int)gridDim.x / 2 : (int)gridDim.x;
    const int role = split ? (int)blockIdx.x / G : 2;
    const int grp = split ? (int)blockIdx.x % G : (int)blockIdx.x;
    const int64_t ntiles = (A.batch + P::S - 1) / P::S;
    int T = 0;
    for (int64_t tl = grp; tl < ntiles && T < P::TMAX; tl += G) ++T;
    if (T == 0) return;  // (uniform; the host sizes the grid so that it does not happen)
    // sampler: thread t < 64 owns word t&3 of sample t>>2 of every tile; it draws the sample's
    // ring row itself (same draw as k_sample / o2048_replay_sample_f64, domain 3; the four
    // threads of a sample agree) and loads that word of s' at once
    int32_t rv[P::TMAX];  // r and d of sample t>>2 of every tile (threads t < 64, t&3 == 0)
    uint32_t dv[P::TMAX];
#pragma unroll
    for (int k = 0; k < P::TMAX; ++k) {
        rv[k] = 0;
        dv[k] = 0u;
    }
    if (t < P::S * 4) {
        const int s = t >> 2;
        const unsigned long long ep = A.idx_in ? 0ull : *A.epoch;
        const unsigned long long cnt = A.idx_in ? 0ull : *A.count;
        uint32_t w[P::TMAX];
#pragma unroll
        for (int k = 0; k < P::TMAX; ++k) {
            w[k] = 0u;
            if (k >= T) continue;
            const int64_t b = (grp + (int64_t)k * G) * P::S + s;
            int64_t j = 0;
            if (b < A.batch) {
                if (A.idx_in) {
                    j = A.idx_in[b];
                } else {
                    const uint4 u = g2048::philox10(
                        make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32), (uint32_t)ep,
                                   (uint32_t)(ep >> 32) | (g2048::DOMAIN_SAMPLE << 30)),
                        A.seed_lo, A.seed_hi);
                    const unsigned long long x = ((unsigned long long)u.y << 32) | u.x;
                    j = (int64_t)__umul64hi(x, cnt);
                }
                if ((t & 3) == 0 && role != 1) A.idx_out[b] = j;
            }
            if ((t & 3) == 0) {
                sidx[k * P::S + s] = j;
                if (role != 0) {
                    rv[k] = A.r[j];
                    dv[k] = A.d[j];
                }
            }
            w[k] = reinterpret_cast<const uint32_t*>(A.s2)[j * 4 + (t & 3)];
        }
#pragma unroll
        for (int k = 0; k < P::TMAX; ++k)
            if (k < T) P::put_word(lds + P::OFF_X + k * P::S * 16, t, w[k]);
    }
    P::Regs R;
    float* qon = lds + P::OFF_Q;               // [TMAX][16][4]
    float* qtg = qon + P::TMAX * P::S * 4;     // [TMAX][16][4]
    if (A.double_dqn && role != 1) {  // (vanilla DQN needs no online Q of s')
        P::stage(A.on, lds, R);  // (starts with __syncthreads: the s' boards are visible)
        P::tiles_pipe(lds, R, T, qon);
    }
    if (role == 0) {  // a* of every sample for the train launch
        for (int k = 0; k < T; ++k) {
            const int64_t b = (grp + (int64_t)k * G) * P::S + t;
            if (t < P::S && b < A.batch) A.astar[b] = argmax4_first(qon + (k * P::S + t) * 4);
        }
        return;
    }
    P::stage(A.tg, lds, R);
    P::tiles_pipe(lds, R, T, qtg);
    for (int k = 0; k < T; ++k) {
        const int sm = t >> 2;  // sample of this thread (t < 64, t & 3 == 0)
        const int64_t b = (grp + (int64_t)k * G) * P::S + sm;
        if (t < P::S * 4 && (t & 3) == 0 && b < A.batch) {
            const float* qt = qtg + (k * P::S + sm) * 4;
            const float disc = (float)(1 - (int)dv[k]) * A.gamma;
            if (role == 1) {
                A.qtg[b] = make_float4(qt[0], qt[1], qt[2], qt[3]);
                A.rdisc[b] = make_float2((float)rv[k], disc);
            } else {
                const float next = A.double_dqn ? qt[argmax4_first(qon + (k * P::S + sm) * 4)]
                                                : g2048::qmax4_torch(qt[0], qt[1], qt[2], qt[3]);
                A.y[b] = g2048::cnet::bellman_y((float)rv[k], disc, next);
            }
        }
    }
}

}  // namespace

extern "C" G2048_API int g2048_convnet_forward(const g2048_convnet_params* p, const uint8_t* rows,
                                               const int64_t* idx, int64_t n, float* q_out,
                                               void* stream) {
    if (!p || !rows || !q_out || n <= 0)
        return g2048_fail(G2048_EINVAL, "convnet_forward: NULL argument or n <= 0");
    if (!p->w1 || !p->b1 || !p->w2 || !p->b2 || !p->fc1_w || !p->fc1_b || !p->fc2_w || !p->fc2_b)
        return g2048_fail(G2048_EINVAL, "convnet_forward: NULL parameter pointer");
    ConvNetArgs A;
    A.w1 = p->w1;
    A.b1 = p->b1;
    A.w2 = p->w2;
    A.b2 = p->b2;
    A.wf1 = p->fc1_w;
    A.bf1 = p->fc1_b;
    A.wf2 = p->fc2_w;
    A.bf2 = p->fc2_b;
    A.rows = rows;
    A.idx = idx;
    A.n = n;
    A.q = q_out;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t tiles16 = (n + persist::S - 1) / persist::S;
    const unsigned grid = (unsigned)(tiles16 < 256 ? tiles16 : 256);  // one workgroup per CU
    hipLaunchKernelGGL(k_conv_forward_pipe, dim3(grid), dim3(NT), 0, st, A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_forward: %s", hipGetErrorString(e));
}

extern "C" G2048_API int g2048_convnet_forward_greedy(const g2048_convnet_params* p,
                                                      g2048_env* env, const double* eps_dev,
                                                      double eps, double eps_decay_episodes,
                                                      double eps_min, float* q_out, void* stream) {
    if (!p || !env || !q_out)
        return g2048_fail(G2048_EINVAL, "convnet_forward_greedy: NULL argument");
    if (!p->w1 || !p->b1 || !p->w2 || !p->b2 || !p->fc1_w || !p->fc1_b || !p->fc2_w || !p->fc2_b)
        return g2048_fail(G2048_EINVAL, "convnet_forward_greedy: NULL parameter pointer");
    uint8_t* board = nullptr;
    uint32_t* ep = nullptr;
    uint64_t* clock = nullptr;
    uint64_t seed = 0, offset = 0;
    if (g2048_env_views(env, &board, nullptr, &ep, &clock) != G2048_OK ||
        g2048_env_rng(env, &seed, &offset) != G2048_OK)
        return G2048_EINVAL;
    const int64_t n = g2048_env_size(env);
    if (n <= 0) return g2048_fail(G2048_EINVAL, "convnet_forward_greedy: empty env");
    GreedyArgs G;
    G.net = ConvNetArgs{p->w1, p->b1, p->w2, p->b2, p->fc1_w, p->fc1_b, p->fc2_w, p->fc2_b,
                        board, nullptr, n, q_out};
    G.clock = clock;
    G.ep = ep;
    G.board_offset = offset;
    G.seed_lo = (uint32_t)seed;
    G.seed_hi = (uint32_t)(seed >> 32);
    G.eps_dev = eps_dev;
    G.eps = eps;
    G.eps_decay = eps_decay_episodes > 0.0 ? eps_decay_episodes : 0.0;
    G.eps_min = eps_min;
    const int64_t tiles16 = (n + persist::S - 1) / persist::S;
    const int64_t grid = tiles16 < 256 ? tiles16 : 256;  // one workgroup per CU
    G.chunk = (n + grid - 1) / grid;
    hipLaunchKernelGGL(k_conv_forward_greedy, dim3((unsigned)grid), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), G);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_forward_greedy: %s",
                                        hipGetErrorString(e));
}

// Shared by g2048_convnet_targets (y_out) and g2048_convnet_update (g2048_qtrain.hip: split
// roles when split_ws is given -- a* i32[B] | Q_target f32[B][4] | (r, disc) f32[B][2]).
extern "C" int g2048_conv_targets_launch(const g2048_convnet_params* online,
                                         const g2048_convnet_params* target, g2048_replay* rb,
                                         const int64_t* idx_in, int64_t batch, uint64_t seed,
                                         const uint64_t* epoch_dev, float gamma, int double_dqn,
                                         int64_t* idx_out, float* y_out, float* split_ws,
                                         void* stream) {
    uint8_t *s2 = nullptr, *d = nullptr;
    int32_t* r = nullptr;
    uint64_t* count = nullptr;
    if (g2048_replay_views(rb, nullptr, &s2, nullptr, &r, &d, &count) != G2048_OK)
        return G2048_EINVAL;
    TargetArgs A;
    A.on = NetW{online->w1, online->b1, online->w2, online->b2, online->fc1_w, online->fc1_b,
                online->fc2_w, online->fc2_b};
    A.tg = NetW{target->w1, target->b1, target->w2, target->b2, target->fc1_w, target->fc1_b,
                target->fc2_w, target->fc2_b};
    A.s2 = s2;
    A.r = r;
    A.d = d;
    A.count = reinterpret_cast<const unsigned long long*>(count);
    A.epoch = reinterpret_cast<const unsigned long long*>(epoch_dev);
    A.idx_in = idx_in;
    A.batch = batch;
    A.seed_lo = (uint32_t)seed;
    A.seed_hi = (uint32_t)(seed >> 32);
    A.gamma = gamma;
    A.double_dqn = double_dqn;
    A.idx_out = idx_out;
    A.y = y_out;
    A.astar = nullptr;
    A.qtg = nullptr;
    A.rdisc = nullptr;
    const int64_t ntiles = (batch + persist::S - 1) / persist::S;
    int64_t grid;
    if (split_ws && double_dqn) {  // 2 x G workgroups, G <= 128 so both halves fit the 256 CUs
        int64_t G = ntiles < 128 ? ntiles : 128;
        if (G * persist::TMAX < ntiles) G = (ntiles + persist::TMAX - 1) / persist::TMAX;
        A.astar = reinterpret_cast<int32_t*>(split_ws);
        A.qtg = reinterpret_cast<float4*>(split_ws + g2048::cnet::conv_split_qtg_offset(batch));
        A.rdisc = reinterpret_cast<float2*>(split_ws + g2048::cnet::conv_split_rd_offset(batch));
        grid = 2 * G;
    } else {
        grid = ntiles < 256 ? ntiles : 256;
        if (grid * persist::TMAX < ntiles) grid = (ntiles + persist::TMAX - 1) / persist::TMAX;
    }
    hipLaunchKernelGGL(k_conv_targets_persist, dim3((unsigned)grid), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_targets: %s", hipGetErrorString(e));
}

extern "C" G2048_API int g2048_convnet_targets(const g2048_convnet_params* online,
                                               const g2048_convnet_params* target,
                                               g2048_replay* rb, const int64_t* idx_in,
                                               int64_t batch, uint64_t seed,
                                               const uint64_t* epoch_dev, float gamma,
                                               int double_dqn, int64_t* idx_out, float* y_out,
                                               void* stream) {
    if (!online || !target || !rb || batch <= 0 || !idx_out || !y_out || (!idx_in && !epoch_dev))
        return g2048_fail(G2048_EINVAL, "convnet_targets: NULL argument or batch <= 0");
    return g2048_conv_targets_launch(online, target, rb, idx_in, batch, seed, epoch_dev, gamma,
                                     double_dqn, idx_out, y_out, nullptr, stream);
}
