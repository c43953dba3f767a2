// g2048_qtrain.hip -- fused Double-DQN gradient of the reference conv Q-net on gfx950 f32 MFMA,
// with conv2 in the Winograd domain (g2048_convnet.hpp).
//
// For a minibatch of B replay rows (indices idx, Bellman targets y) the launches compute
//   q_b = Q(s_b)[a_b],  loss = sum_b (q_b - y_b)^2,  and d loss / d theta for all 33 476 params
// = the graded half of the reference train_step (src/dqn_lib.py:146-161: model(states), the
// one-hot gather, MSELoss(reduction='sum'), loss.backward()):
//
//   k_conv_train_fwd  per 16-board tile: conv1 + V, conv2 (9 Winograd GEMMs, U in VGPRs), fc1,
//                     fc2 at the taken action, loss, dq; dWf2 / dbf2, df, dbf1;
//                     dWf1 += df^T h2 (MFMA, AGPR accumulators across tiles);
//                     dY = (df Wf1) * relu'(h2) (MFMA), db2, dM = A dY A^T (lane-local);
//                     dU_xi += V_xi^T dM_xi (9 x 16 MFMAs, AGPR accumulators across tiles);
//                     dM -> workspace.  At the end dW2 = G^T dU G (lane-local) and the other
//                     partial gradients go to this workgroup's slab in torch order.
//   k_conv_train_bwd  per tile: dV_xi = dM_xi U_xi^T (U in the transposed register layout),
//                     dh1 = B dV B^T, relu'(h1) from conv1 recomputed in the forward's float
//                     order, dW1 / db1 -> the same slab.
//   k_reduce_pre      fixed-order sums (deterministic) -> the flat gradient bucket, optionally
//                     with Adam folded in: train fwd's slab terms arrive summed (train bwd adds
//                     them in the shadow of its MFMAs), conv1's are summed here over the slabs.
//                     (k_reduce_slabs: every term over the slabs, for grids too small to shadow.)
//
// g2048_convnet_update puts the targets launch (g2048_qnet.hip) in front: one whole train_step
// per call; with Double DQN, k_conv_train_fwd forms y from the targets' online / target halves.
//
// dM has to change register layout between the two data-gradient GEMMs (dU contracts over
// boards, dV over output channels), and U is needed in both orientations; one workgroup cannot
// hold both (144 VGPRs each), hence the two launches and the 36 KB-per-tile dM round trip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/g2048.h"
#include "g2048_common.hpp"
#include "g2048_convnet.hpp"

namespace {

using namespace g2048::cnet;

// parameter offsets in torch order (Conv2048.parameters())
constexpr int P_W1 = 0, P_B1 = 256, P_W2 = 320, P_B2 = 16704, P_WF1 = 16768, P_BF1 = 33152,
              P_WF2 = 33216, P_BF2 = 33472, P_TOTAL = 33476;
// slab = one workgroup's partial gradient, written coalesced in kernel order (k_reduce_slabs maps
// positions back to torch order): [dW2 16384 | dWf1 16384 | w1 256 | b1 64 | b2 64 | bf1 64 |
// wf2 256 | bf2 4 | loss 1], padded
constexpr int SL_W2 = 0, SL_WF1 = 16384, SL_SMALL = 32768, SL_LOSS = SL_SMALL + 708;
constexpr int SLAB = 33480;
static_assert(SL_LOSS == P_TOTAL && SLAB % 4 == 0, "slab layout");
constexpr int TMAXT = 4;               // tiles per workgroup (B <= 16384 on 256 workgroups)
// k_conv_train_bwd sums k_conv_train_fwd's slab terms in the shadow of its phases (SlabShadow):
// block g owns the float4s [g * chunk, (g + 1) * chunk) of the slab, one per lane, chunk <= 64, so
// the grid needs >= SHADOW_MIN_GRID blocks.  conv1's weight and bias (float4s [C1_F4_LO,
// C1_F4_HI)) are train bwd's own terms and stay with k_reduce_slabs, spread over C1_BLOCKS blocks
// of C1_PER_BLOCK float4s each.
constexpr int SLAB_F4 = SLAB / 4;
constexpr int SHADOW_MIN_GRID = (SLAB_F4 + 63) / 64;
constexpr int C1_F4_LO = SL_SMALL / 4, C1_F4_HI = (SL_SMALL + 320) / 4;
constexpr int C1_PER_BLOCK = 16, C1_BLOCKS = (C1_F4_HI - C1_F4_LO) / C1_PER_BLOCK;
static_assert(SL_SMALL % 4 == 0 && (C1_F4_HI - C1_F4_LO) % C1_PER_BLOCK == 0, "conv1 float4 ranges");
constexpr int DM_TILE = 9 * S * 64;    // dM floats per tile in the workspace: [xi][b][o]

// k_conv_train_fwd LDS carve (floats)
constexpr int K1_X = 0;                        // [TMAXT][S][16] boards
constexpr int K1_B2 = K1_X + TMAXT * S * 16;   // 64
constexpr int K1_BF1 = K1_B2 + 64;             // 64
constexpr int K1_WF2 = K1_BF1 + 64;            // [4][WF2S]
constexpr int K1_BF2 = K1_WF2 + 4 * WF2S;      // 4
constexpr int K1_SA = K1_BF2 + 4;              // [TMAXT][S] actions (int; -1 = padding row)
constexpr int K1_SY = K1_SA + TMAXT * S;       // [TMAXT][S] targets
constexpr int K1_SQ = K1_SY + TMAXT * S;       // [S] dq
constexpr int K1_WF1 = (K1_SQ + S + 3) & ~3;   // [64][WF1S]
constexpr int K1_V = K1_WF1 + 64 * WF1S;       // [9][S][VS]  (end: reduction scratch)
constexpr int K1_H2 = K1_V + 9 * VXI;          // [S][H2S]
constexpr int K1_F = K1_H2 + S * H2S;          // f [S][FS]
constexpr int K1_DF = K1_F + S * FS;           // df [S][FS]
constexpr int K1_FLOATS = K1_DF + S * FS;
static_assert(K1_WF1 % 4 == 0 && K1_V % 4 == 0 && K1_H2 % 4 == 0 && K1_F % 4 == 0 &&
                  K1_DF % 4 == 0 && K1_WF2 % 4 == 0,
              "b128 alignment");
static_assert(K1_FLOATS * 4 <= 160 * 1024, "LDS budget (train fwd)");
// k_conv_train_bwd LDS carve (floats)
constexpr int K2_X = 0;                        // [TMAXT][S][16]
constexpr int K2_DM = K2_X + TMAXT * S * 16;   // 2 x [9][S][VS]  (end: reduction scratch)
constexpr int K2_FLOATS = K2_DM + 2 * 9 * VXI;
static_assert(9 * VXI >= NT * 5 && 9 * VXI >= 2 * NT, "reduction scratch");

struct TrainArgs {
    NetW W;
    const uint8_t* rows;     // replay s rows [*][16]
    const uint8_t* actions;  // replay a [*]
    const int64_t* idx;      // [B]
    const float* y;          // [B] Bellman targets (unless the split inputs below are given)
    // split targets (g2048_convnet_update): y_b = r_b + disc_b * Q_target(s'_b)[a*_b], formed
    // here from the two halves of the targets launch and written to y_out
    const int32_t* astar;    // [B] (nullptr: read y)
    const float4* qtg;       // [B]
    const float2* rdisc;     // [B]
    float* y_out;            // [B]
    int64_t batch;
    float* slab;             // [gridDim.x][SLAB]
    float* dm;               // [ntiles][DM_TILE]
    float* pre;              // [SLAB] train fwd's slab terms summed by train bwd (null: the reduce)
    unsigned long long* step;  // optional update counter, += 1 by one thread (nullable)
};

#ifdef G2048_PHASE_PROF
__device__ unsigned long long g_tphase[16];
#define TPHASE_BEGIN() unsigned long long tph_ = __builtin_amdgcn_s_memtime()
#define TPHASE(k)                                                         \
    do {                                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                        \
            const unsigned long long n_ = __builtin_amdgcn_s_memtime();   \
            g_tphase[k] += n_ - tph_;                                     \
            tph_ = n_;                                                    \
        }                                                                 \
    } while (0)
#else
#define TPHASE_BEGIN()
#define TPHASE(k)
#endif

// Barrier for LDS hazards only: waits for this wave's LDS ops, not for its global stores (the
// dM / slab stores are read by later launches only), then s_barrier.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // -> s_waitcnt lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int tiles_here(int64_t ntiles) {
    int T = 0;
    for (int64_t tl = blockIdx.x; tl < ntiles && T < TMAXT; tl += gridDim.x) ++T;
    return T;
}

// The tile's boards (t < 64: word t & 3 of sample t >> 2) into xs as floats.
__device__ __forceinline__ uint32_t board_word(const TrainArgs& A, int64_t b0, int t) {
    const int64_t b = b0 + (t >> 2);
    if (t >= S * 4 || b >= A.batch) return 0u;
    return reinterpret_cast<const uint32_t*>(A.rows)[A.idx[b] * 4 + (t & 3)];
}

__global__ __launch_bounds__(NT) void k_conv_train_fwd(TrainArgs A) {
    __shared__ __attribute__((aligned(16))) float lds[K1_FLOATS];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g = lane >> 4, l16 = lane & 15;
    // nothing else in this launch reads the counter; stream order makes the bump visible to the
    // following launches and to the next update's sampler
    if (A.step && blockIdx.x == 0 && t == 0) *A.step += 1ull;
    const int64_t ntiles = (A.batch + S - 1) / S;
    const int T = tiles_here(ntiles);
    TPHASE_BEGIN();

    // ---- inputs of all tiles + the net, in one memory round trip
    uint32_t bw[TMAXT];
    int av[TMAXT];
    float yv[TMAXT];
#pragma unroll
    for (int k = 0; k < TMAXT; ++k) {
        bw[k] = 0u;
        av[k] = -1;
        yv[k] = 0.f;
        if (k < T) {
            const int64_t b0 = (blockIdx.x + (int64_t)k * gridDim.x) * S;
            bw[k] = board_word(A, b0, t);
            if (t < S && b0 + t < A.batch) {
                av[k] = A.actions[A.idx[b0 + t]];
                if (A.astar) {
                    const int a = A.astar[b0 + t];
                    const float4 q = A.qtg[b0 + t];
                    const float2 rd = A.rdisc[b0 + t];
                    const float next = a == 0 ? q.x : a == 1 ? q.y : a == 2 ? q.z : q.w;
                    yv[k] = bellman_y(rd.x, rd.y, next);
                    A.y_out[b0 + t] = yv[k];
                } else {
                    yv[k] = A.y[b0 + t];
                }
            }
        }
    }
    Regs R;
    load_u_fwd(A.W.w2, R);
    load_conv1(A.W, R);
    const float b2 = t < 64 ? A.W.b2[t] : 0.f, bf1 = t < 64 ? A.W.bf1[t] : 0.f;
    const float wf2 = A.W.wf2[t], bf2 = t < 4 ? A.W.bf2[t] : 0.f;
    float fcol[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) fcol[i] = A.W.wf1[i * NT + t];
    if (t < 64) {
        lds[K1_B2 + t] = b2;
        lds[K1_BF1 + t] = bf1;
    }
    lds[K1_WF2 + (t >> 6) * WF2S + (t & 63)] = wf2;
    if (t < 4) lds[K1_BF2 + t] = bf2;
    store_fc1(fcol, lds + K1_WF1);
    int* sa = reinterpret_cast<int*>(lds + K1_SA);
#pragma unroll
    for (int k = 0; k < TMAXT; ++k) {
        if (k < T) {
            if (t < S * 4) put_word(lds + K1_X + k * S * 16, t, bw[k]);
            if (t < S) {
                sa[k * S + t] = av[k];
                lds[K1_SY + k * S + t] = yv[k];
            }
        }
    }
    __syncthreads();
    TPHASE(0);

    f32x4 aU[9][4];   // dU_xi[c = 16mt + 4g + i][o = 16*wave + l16]
    f32x4 aF1[4][4];  // dWf1[j = 16jt + 4g + i][k' = 16(4*wave + e) + l16]
#pragma unroll
    for (int xi = 0; xi < 9; ++xi)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) aU[xi][mt] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e) aF1[jt][e] = f32x4{0, 0, 0, 0};
    float accWf2 = 0.f, accBf2 = 0.f, accBf1 = 0.f, accB2 = 0.f, accLoss = 0.f;
    float* V = lds + K1_V;
    float* h2 = lds + K1_H2;
    float* fa = lds + K1_F;
    float* df = lds + K1_DF;
    float* sq = lds + K1_SQ;
    const float* wf1s = lds + K1_WF1;
    const int o = 16 * wave + l16;

    for (int k = 0; k < T; ++k) {
        const int64_t tile = blockIdx.x + (int64_t)k * gridDim.x;
        const int* sak = sa + k * S;
        if (k > 0) lds_barrier();  // the previous tile's reads of V / h2 / f / df are done
        // ---- forward
        conv1_v(lds + K1_X + k * S * 16, V, R);
        lds_barrier();
        TPHASE(1);
        conv2_h2(V, h2, lds + K1_B2, R);
        lds_barrier();
        TPHASE(2);
        fc1_f(h2, wf1s, lds + K1_BF1, fa);
        lds_barrier();
        TPHASE(3);
        // ---- fc2 at the taken action (the one-hot gather), loss, dq = 2 (q - y):
        //      thread = (sample t >> 4, 4 units 4(t & 15)..), 16-lane shuffle sum
        {
            const int s2 = t >> 4, p4 = (t & 15) * 4, a = sak[s2];
            const f32x4 fv = *reinterpret_cast<const f32x4*>(fa + s2 * FS + p4);
            const f32x4 wv = *reinterpret_cast<const f32x4*>(lds + K1_WF2 + (a < 0 ? 0 : a) * WF2S + p4);
            float v = fmaf(wv[3], fv[3], fmaf(wv[2], fv[2], fmaf(wv[1], fv[1], wv[0] * fv[0])));
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if ((t & 15) == 0) {
                const float d = a >= 0 ? (v + lds[K1_BF2 + a]) - lds[K1_SY + k * S + s2] : 0.f;
                accLoss = fmaf(d, d, accLoss);
                sq[s2] = 2.f * d;
            }
        }
        lds_barrier();
        // ---- dWf2 / dbf2 (thread = (a, j)); df = dq * wf2[a_s] * relu'(f) (thread = (s, 4 j))
        {
            const int a = t >> 6, j = t & 63;
            float gw = 0.f, gb = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < S; ++s2) {
                const float gq = sak[s2] == a ? sq[s2] : 0.f;
                gw = fmaf(gq, fa[s2 * FS + j], gw);
                gb += gq;
            }
            accWf2 += gw;
            if (j == 0) accBf2 += gb;
            const int s2 = t >> 4, j0 = (t & 15) * 4;
            const int as = sak[s2];
            const float gq = sq[s2];
            const f32x4 fv = *reinterpret_cast<const f32x4*>(fa + s2 * FS + j0);
            f32x4 dv = f32x4{0, 0, 0, 0};
            if (as >= 0) {
                const f32x4 wv = *reinterpret_cast<const f32x4*>(lds + K1_WF2 + as * WF2S + j0);
#pragma unroll
                for (int e = 0; e < 4; ++e) dv[e] = fv[e] > 0.f ? gq * wv[e] : 0.f;
            }
            *reinterpret_cast<f32x4*>(df + s2 * FS + j0) = dv;
        }
        lds_barrier();
        TPHASE(4);
        // ---- dbf1; dWf1 += df^T h2  (m = j, k = board 4g + kk, n = k')
        if (t < 64) {
            float v = 0.f;
#pragma unroll 4
            for (int s2 = 0; s2 < S; ++s2) v += df[s2 * FS + t];
            accBf1 += v;
        }
        // operands of step n + 1 are read while step n's MFMAs run (sched_barrier pins the
        // order: at one wave per SIMD an exposed LDS latency per MFMA group is not hidden)
        {
            float a4[2][4], b4[2][4];
            auto ld = [&](int kk, int buf) {
                const int b = 4 * g + kk;
#pragma unroll
                for (int jt = 0; jt < 4; ++jt) a4[buf][jt] = df[b * FS + 16 * jt + l16];
#pragma unroll
                for (int e = 0; e < 4; ++e) b4[buf][e] = h2[b * H2S + 16 * (4 * wave + e) + l16];
            };
            ld(0, 0);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                if (kk < 3) ld(kk + 1, (kk + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int jt = 0; jt < 4; ++jt)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        aF1[jt][e] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            a4[kk & 1][jt], b4[kk & 1][e], aF1[jt][e], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- dY = df @ Wf1  (m = board, k = j(kk, g) = 16m4 + 4g + e4, n = k' = q*64 + o)
        f32x4 dY[4] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
        {
            f32x4 a4[2];
            float bq[2][4][4];
            auto ld = [&](int m4, int buf) {
                a4[buf] = *reinterpret_cast<const f32x4*>(df + l16 * FS + 16 * m4 + 4 * g);
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const float* brow = wf1s + (16 * m4 + 4 * g + e4) * WF1S;
#pragma unroll
                    for (int q = 0; q < 4; ++q) bq[buf][e4][q] = brow[wf1_col(64 * q + o)];
                }
            };
            ld(0, 0);
#pragma unroll
            for (int m4 = 0; m4 < 4; ++m4) {
                if (m4 < 3) ld(m4 + 1, (m4 + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        dY[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[m4 & 1][e4], bq[m4 & 1][e4][q],
                                                                     dY[q], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        TPHASE(5);
        // ---- relu'(h2), db2, dM = A dY A^T (lane-local: all four positions of (board, o))
        float dm[9][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float* hr = h2 + (4 * g + i) * H2S + o;
            float d[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = hr[64 * q] > 0.f ? dY[q][i] : 0.f;
            accB2 += (d[0] + d[1]) + (d[2] + d[3]);
            const float s01 = d[0] + d[1], s23 = d[2] + d[3], s02 = d[0] + d[2], s13 = d[1] + d[3];
            dm[0][i] = d[0];
            dm[1][i] = s01;
            dm[2][i] = d[1];
            dm[3][i] = s02;
            dm[4][i] = s02 + s13;
            dm[5][i] = s13;
            dm[6][i] = d[2];
            dm[7][i] = s23;
            dm[8][i] = d[3];
        }
        // ---- dU_xi += V_xi^T dM_xi  (m = c, k = board 4g + kk: the lane's own dM registers);
        //      point xi + 1's V operands are read during point xi's 16 MFMAs
        {
            float av[2][4][4];
            auto ld = [&](int xi, int buf) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const float* vrow = V + xi * VXI + (4 * g + kk) * VS + l16;
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt) av[buf][kk][mt] = vrow[16 * mt];
                }
            };
            ld(0, 0);
#pragma unroll
            for (int xi = 0; xi < 9; ++xi) {
                if (xi < 8) ld(xi + 1, (xi + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int mt = 0; mt < 4; ++mt)
                        aU[xi][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            av[xi & 1][kk][mt], dm[xi][kk], aU[xi][mt], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // ---- dM -> workspace [xi][board][o] for k_conv_train_bwd
        float* dst = A.dm + tile * DM_TILE + (4 * g) * 64 + o;
#pragma unroll
        for (int xi = 0; xi < 9; ++xi)
#pragma unroll
            for (int i = 0; i < 4; ++i) dst[(xi * S + i) * 64] = dm[xi][i];
        TPHASE(6);
    }
    __syncthreads();  // every tile is done: the V area becomes the reduction scratch

    // ---- this workgroup's partial gradient (coalesced, kernel order; see slab_to_param)
    float* slab = A.slab + (int64_t)blockIdx.x * SLAB;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // dW2[o][c = 16mt + 4g + i][kh][kw] = G^T dU G
            float u[9];
#pragma unroll
            for (int xi = 0; xi < 9; ++xi) u[xi] = aU[xi][mt][i];
            g2048::slab_store16(
                reinterpret_cast<float4*>(slab), SL_W2 / 4 + (mt * 4 + i) * NT + t,
                make_float4((u[0] + u[1]) + (u[3] + u[4]), (u[1] + u[2]) + (u[4] + u[5]),
                            (u[3] + u[4]) + (u[6] + u[7]), (u[4] + u[5]) + (u[7] + u[8])));
        }
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e)  // the accumulator's four rows i as one 16-byte store
            *reinterpret_cast<f32x4*>(slab + SL_WF1 + ((jt * 4 + e) * NT + t) * 4) = aF1[jt][e];
    float* red = lds + K1_V;
    red[t] = accB2;
    red[NT + t] = accLoss;
    __syncthreads();
    if (t < 64) {  // o = t: lanes (l16 = t & 15, g = 0..3) of wave t >> 4
        const float* rw = red + (t >> 4) * 64 + (t & 15);
        slab[SL_SMALL + 320 + t] = ((rw[0] + rw[16]) + rw[32]) + rw[48];  // b2
        slab[SL_SMALL + 384 + t] = accBf1;
    }
    slab[SL_SMALL + 448 + t] = accWf2;  // wf2[a][j], t = a*64 + j
    if ((t & 63) == 0) slab[SL_SMALL + 704 + (t >> 6)] = accBf2;
    if (t == 0) {  // per-sample partials live in the lanes t = 16 s
        float v = 0.f;
        for (int i = 0; i < S; ++i) v += red[NT + 16 * i];
        slab[SL_LOSS] = v;
    }
    TPHASE(7);
}

// slab position -> torch flat parameter index
__device__ __forceinline__ int slab_to_param(int pos) {
    if (pos < SL_WF1) {  // ((mt*4 + i)*NT + t)*4 + tap: o = 16*wave + l16, c = 16mt + 4g + i
        const int tap = pos & 3, t = (pos >> 2) & (NT - 1), r = pos >> 10;
        const int lane = t & 63, o = 16 * (t >> 6) + (lane & 15);
        const int c = 16 * (r >> 2) + 4 * (lane >> 4) + (r & 3);
        return P_W2 + o * 256 + c * 4 + tap;
    }
    if (pos < SL_SMALL) {  // ((jt*4 + e)*NT + t)*4 + i: j = 16jt + 4g + i, flat m = 4c' + q
                           // with c' = 16e + l16, q = wave
        const int p2 = pos - SL_WF1, i = p2 & 3, t = (p2 >> 2) & (NT - 1), je = p2 >> 10;
        const int lane = t & 63;
        const int j = 16 * (je >> 2) + 4 * (lane >> 4) + i;
        const int m = 4 * (16 * (je & 3) + (lane & 15)) + (t >> 6);
        return P_WF1 + j * 256 + m;
    }
    const int p3 = pos - SL_SMALL;  // w1 | b1 | b2 | bf1 | wf2 | bf2 in torch order
    if (p3 < 256) return P_W1 + p3;
    if (p3 < 320) return P_B1 + p3 - 256;
    if (p3 < 384) return P_B2 + p3 - 320;
    if (p3 < 448) return P_BF1 + p3 - 384;
    if (p3 < 704) return P_WF2 + p3 - 448;
    return P_BF2 + p3 - 704;
}

// train bwd's sums of train fwd's slab terms go to `pre` in torch parameter order, so that
// k_reduce_pre's Adam operands (m, v, the parameters) and its gradient stores are coalesced
// float4s.  A slab float4 is four contiguous, 16-byte aligned torch positions everywhere except in
// fc1.weight's block, whose four positions scatter (stride 4); the loss stays at P_TOTAL.
__device__ __forceinline__ void store_pre_torch(float* pre, int f4, float4 s) {
    const int pos = f4 * 4;
    if (pos >= SL_WF1 && pos < SL_SMALL) {
        pre[slab_to_param(pos)] = s.x;
        pre[slab_to_param(pos + 1)] = s.y;
        pre[slab_to_param(pos + 2)] = s.z;
        pre[slab_to_param(pos + 3)] = s.w;
    } else {
        *reinterpret_cast<float4*>(pre + slab_to_param(pos)) = s;
    }
}

__global__ __launch_bounds__(NT) void k_conv_train_bwd(TrainArgs A) {
    __shared__ __attribute__((aligned(16))) float lds[K2_FLOATS];
    const int t = threadIdx.x, lane = t & 63, g = lane >> 4, l16 = lane & 15, wave = t >> 6;
    const int64_t ntiles = (A.batch + S - 1) / S;
    const int T = tiles_here(ntiles);
    // train fwd's slab terms, summed between this launch's phases (A.pre: the grid is
    // >= SHADOW_MIN_GRID, so a block's chunk fits one float4 per lane)
    g2048::SlabShadow<float4, 8> sh;
    const int chunk = (SLAB_F4 + (int)gridDim.x - 1) / (int)gridDim.x;
    const int f4 = (int)blockIdx.x * chunk + lane;
    const bool sh_on =
        A.pre != nullptr && lane < chunk && f4 < SLAB_F4 && (f4 < C1_F4_LO || f4 >= C1_F4_HI);
    if (A.pre)
        sh.init(sh_on ? reinterpret_cast<const float4*>(A.slab) + f4 : nullptr, SLAB_F4,
                (int)gridDim.x, wave);
    // dM of tiles k and k + 1 -> the two LDS buffers [xi][b][VS] in one memory round trip
    // (coalesced float4: 9 per thread per tile)
    auto copy_pair = [&](int k) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (k + h >= T) break;
            const float4* src = reinterpret_cast<const float4*>(
                A.dm + (blockIdx.x + (int64_t)(k + h) * gridDim.x) * DM_TILE);
            float* dst = lds + K2_DM + h * 9 * VXI;
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                const int f4 = r * NT + t;
                *reinterpret_cast<float4*>(dst + (f4 >> 4) * VS + (f4 & 15) * 4) = src[f4];
            }
        }
    };
    // the first pair, the boards and the weights share one memory round trip
    copy_pair(0);
    uint32_t bw[TMAXT];
#pragma unroll
    for (int k = 0; k < TMAXT; ++k)
        bw[k] = k < T ? board_word(A, (blockIdx.x + (int64_t)k * gridDim.x) * S, t) : 0u;
    Regs R;
    load_u_bwd(A.W.w2, R);  // u[xi][kk] = U_xi[c = 16*wave + l16][o = 16g + kk]
    load_conv1(A.W, R);  // channel c = 16*wave + l16: the lane's dV column
#pragma unroll
    for (int k = 0; k < TMAXT; ++k)
        if (k < T && t < S * 4) put_word(lds + K2_X + k * S * 16, t, bw[k]);
    float gw[4] = {0.f, 0.f, 0.f, 0.f}, gb = 0.f;
    lds_barrier();
    TPHASE_BEGIN();
    TPHASE(8);
    // slab batches: phase p of a tile (three dV groups, then dh1) issues batch (p + 1) & 1 and
    // adds batch p & 1 (this kernel loads no other global data after its first pair of tiles, so
    // no wait below is held up by them)
    if (A.pre) sh.issue<0>();
    for (int k = 0; k < T; ++k) {
        float* dms = lds + K2_DM + (k & 1) * 9 * VXI;
        if ((k & 1) == 0 && k > 0) {
            lds_barrier();  // the previous pair's reads are done
            copy_pair(k);
            lds_barrier();
        }
        TPHASE(9);
        // ---- dV_xi = dM_xi U_xi^T  (m = board l16, k = o = 16g + kk, n = c): groups of three
        //      points, their accumulation chains interleaved (a chain of dependent MFMAs on one
        //      accumulator stalls on every step)
        f32x4 acc[9];
#pragma unroll
        for (int xi = 0; xi < 9; ++xi) acc[xi] = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int grp = 0; grp < 3; ++grp) {
            if (A.pre) {
                if (grp & 1) sh.issue<0>();
                else sh.issue<1>();
            }
            f32x4 a4[3][4];
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                const float* ar = dms + ((3 * grp + e) * S + l16) * VS + 16 * g;
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) a4[e][q4] = *reinterpret_cast<const f32x4*>(ar + 4 * q4);
            }
#pragma unroll
            for (int kk = 0; kk < 16; ++kk)
#pragma unroll
                for (int e = 0; e < 3; ++e)
                    acc[3 * grp + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        a4[e][kk >> 2][kk & 3], R.u[3 * grp + e][kk], acc[3 * grp + e], 0, 0, 0);
            if (A.pre) {
                if (grp & 1) sh.consume<1>();
                else sh.consume<0>();
            }
        }
        TPHASE(10);
        if (A.pre) sh.issue<0>();
        // ---- dh1 = B dV B^T, relu'(h1), dW1 / db1 for (board 4g + i, channel c)
        const float* xs = lds + K2_X + k * S * 16;
        f32x4 pre[9];
        conv1_pre_mfma(xs, R.w1t, pre);  // the forward's pre-activations, bitwise
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float x[16];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 xv = *reinterpret_cast<const float4*>(xs + (4 * g + i) * 16 + 4 * r);
                x[4 * r] = xv.x;
                x[4 * r + 1] = xv.y;
                x[4 * r + 2] = xv.z;
                x[4 * r + 3] = xv.w;
            }
            float rr[3][3];  // B dV: rows (dV0, dV1 - dV0 - dV2, dV2)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                rr[0][j] = acc[j][i];
                rr[1][j] = (acc[3 + j][i] - acc[j][i]) - acc[6 + j][i];
                rr[2][j] = acc[6 + j][i];
            }
#pragma unroll
            for (int ph = 0; ph < 3; ++ph) {
                const float dd[3] = {rr[ph][0], (rr[ph][1] - rr[ph][0]) - rr[ph][2], rr[ph][2]};
#pragma unroll
                for (int pw = 0; pw < 3; ++pw) {
                    const float gh = pre[3 * ph + pw][i] + R.b1o > 0.f ? dd[pw] : 0.f;
                    gb += gh;
                    gw[0] = fmaf(gh, x[ph * 4 + pw], gw[0]);
                    gw[1] = fmaf(gh, x[ph * 4 + pw + 1], gw[1]);
                    gw[2] = fmaf(gh, x[(ph + 1) * 4 + pw], gw[2]);
                    gw[3] = fmaf(gh, x[(ph + 1) * 4 + pw + 1], gw[3]);
                }
            }
        }
        if (A.pre) sh.consume<1>();
    }
    if (A.pre) {  // the batch still in flight, then whatever the tiles did not cover
        sh.consume<0>();
        while (sh.pending()) {
            sh.issue<0>();
            sh.consume<0>();
        }
    }
    TPHASE(11);
    // ---- fixed-order sum over the 4 lane groups that share channel c -> the slab
    __syncthreads();  // every tile's reads of both dM buffers are done
    float* red = lds + K2_DM;
#pragma unroll
    for (int e = 0; e < 4; ++e) red[t * 5 + e] = gw[e];
    red[t * 5 + 4] = gb;
    __syncthreads();
    if (t < 64) {  // channel t: lanes (l16 = t & 15, g = 0..3) of wave t >> 4
        const float* rw = red + ((t >> 4) * 64 + (t & 15)) * 5;
        float* slab = A.slab + (int64_t)blockIdx.x * SLAB;
#pragma unroll
        for (int e = 0; e < 5; ++e) {
            const float v = ((rw[e] + rw[80 + e]) + rw[160 + e]) + rw[240 + e];
            if (e < 4) slab[SL_SMALL + t * 4 + e] = v;  // w1[c][0][kh][kw]
            else slab[SL_SMALL + 256 + t] = v;          // b1
        }
    }
    if (A.pre) {  // the four waves' slab sums, added in wave order
        __shared__ float4 part[3][64];
        if (wave > 0) part[wave - 1][lane] = sh.acc;
        __syncthreads();
        if (wave == 0 && sh_on) {
            const float4 a = sh.acc, b = part[0][lane], c = part[1][lane], d = part[2][lane];
            store_pre_torch(A.pre, f4,
                            make_float4(((a.x + b.x) + c.x) + d.x, ((a.y + b.y) + c.y) + d.y,
                                        ((a.z + b.z) + c.z) + d.z, ((a.w + b.w) + c.w) + d.w));
        }
    }
}

// Optional Adam folded into the reduction (single process): each final gradient element is
// applied by its own thread with the shared adam_apply (bitwise k_adam on the same sums), and
// the target net is synced on the device counter like g2048_adam_step_sync.
struct ReduceAdam {
    float* p[8];   // parameters in torch order (w1, b1, w2, b2, fc1_w, fc1_b, fc2_w, fc2_b)
    float* tp[8];  // target-net parameters (nullable unless sync_every)
    float* m;
    float* v;
    const unsigned long long* step;  // t (already bumped by k_conv_train)
    double lr, b1, b2, eps;
    unsigned long long sync_every;
    int on;
    int vec;  // m, v, every parameter (both nets) and grad_out 16-byte aligned: float4 accesses
};

// The Adam operands of the four positions of slab float4 p4 (loaded with the slabs: they do not
// depend on the sums, so the update costs no memory round trip of its own).
struct AdamLane {
    int kt[4], ei[4];
    float am[4], av[4], ap[4];
};

// conv2.weight's slab float4s (positions < SL_WF1) hold the four taps of one (o, c): contiguous and
// 16-byte aligned in torch order too, so their Adam operands move as float4s (a quarter of the
// scattered lines per wave).  The test is wave-uniform: a wave's 256 positions never straddle
// SL_WF1.
__device__ __forceinline__ bool w2_vec(const ReduceAdam& R, int p4) {
    return R.vec && p4 * 4 < SL_WF1;
}

__device__ __forceinline__ void adam_load(const ReduceAdam& R, int p4, AdamLane& L) {
    constexpr int off[9] = {P_W1, P_B1, P_W2, P_B2, P_WF1, P_BF1, P_WF2, P_BF2, P_TOTAL};
    if (w2_vec(R, p4)) {
        const int pi = slab_to_param(p4 * 4);
        const float4 m4 = *reinterpret_cast<const float4*>(R.m + pi);
        const float4 v4 = *reinterpret_cast<const float4*>(R.v + pi);
        const float4 p4v = *reinterpret_cast<const float4*>(R.p[2] + (pi - P_W2));
        const float am[4] = {m4.x, m4.y, m4.z, m4.w}, av[4] = {v4.x, v4.y, v4.z, v4.w};
        const float ap[4] = {p4v.x, p4v.y, p4v.z, p4v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            L.kt[e] = 2;
            L.ei[e] = pi - P_W2 + e;
            L.am[e] = am[e];
            L.av[e] = av[e];
            L.ap[e] = ap[e];
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int pos = p4 * 4 + e;
        L.kt[e] = -1;
        if (pos >= SL_LOSS) continue;
        const int pi = slab_to_param(pos);
        int k = 0;
#pragma unroll
        for (int j = 1; j < 8; ++j) k += pi >= off[j] ? 1 : 0;
        L.kt[e] = k;
        L.ei[e] = pi - off[k];
        L.am[e] = R.m[pi];
        L.av[e] = R.v[pi];
        L.ap[e] = R.p[k][L.ei[e]];
    }
}

// The summed float4 p4: the loss, the gradient (torch order) and, with Adam, the update.
__device__ __forceinline__ void finish4(const ReduceAdam& R, bool adam, const g2048::AdamCoef& c,
                                        unsigned long long t, int p4, float4 sv, AdamLane& L,
                                        float* grad, float* loss) {
    const float se[4] = {sv.x, sv.y, sv.z, sv.w};
    if (w2_vec(R, p4)) {  // the same per-element update, float4 loads and stores (see adam_load)
        const int pi = slab_to_param(p4 * 4);
        if (grad) *reinterpret_cast<float4*>(grad + pi) = sv;
        if (adam) {
            float np[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) np[e] = g2048::adam_update(c, se[e], L.am[e], L.av[e], L.ap[e]);
            *reinterpret_cast<float4*>(R.m + pi) = make_float4(L.am[0], L.am[1], L.am[2], L.am[3]);
            *reinterpret_cast<float4*>(R.v + pi) = make_float4(L.av[0], L.av[1], L.av[2], L.av[3]);
            const float4 n4 = make_float4(np[0], np[1], np[2], np[3]);
            *reinterpret_cast<float4*>(R.p[2] + (pi - P_W2)) = n4;
            if (R.sync_every && t % R.sync_every == 0ull)
                *reinterpret_cast<float4*>(R.tp[2] + (pi - P_W2)) = n4;
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int pos = p4 * 4 + e;
        const float sm = se[e];
        if (pos > SL_LOSS) break;
        if (pos == SL_LOSS) {
            if (loss) *loss = sm;
        } else {
            const int pi = slab_to_param(pos);
            if (grad) grad[pi] = sm;
            if (adam) {
                const float np = g2048::adam_update(c, sm, L.am[e], L.av[e], L.ap[e]);
                R.m[pi] = L.am[e];
                R.v[pi] = L.av[e];
                R.p[L.kt[e]][L.ei[e]] = np;
                if (R.sync_every && t % R.sync_every == 0ull) R.tp[L.kt[e]][L.ei[e]] = np;
            }
        }
    }
}

// With `pre` (train bwd summed train fwd's slab terms into it, in torch order): blocks
// [0, NB_PRE4) take one torch float4 per thread of their first wave (the other three waves exit
// at once) -- coalesced loads of `pre`, m, v and the parameter, coalesced stores, spread one wave
// per CU.  conv1's weight and bias (torch float4s [0, C1_Q4)) are train bwd's own terms: blocks
// NB_PRE4 + c sum its float4s [16 c, + 16) over the slabs (slab float4 C1_F4_LO + q) -- thread
// (q = t % 16, j = t / 16) the slabs j, j + 16, ... (16 loads in flight), then 16 threads add the
// 16 partials in j order.
constexpr int PRE_F4_PER_BLOCK = 64;
constexpr int TQ4 = P_TOTAL / 4 + 1;  // torch float4s, the loss's last
constexpr int C1_Q4 = P_W2 / 4;
constexpr int NB_PRE4 = (TQ4 + PRE_F4_PER_BLOCK - 1) / PRE_F4_PER_BLOCK;
static_assert(C1_F4_HI - C1_F4_LO == C1_Q4 && SL_SMALL + P_W2 == C1_F4_HI * 4 &&
                  P_TOTAL % 4 == 0 && P_B1 % 4 == 0 && P_B2 % 4 == 0 && P_WF1 % 4 == 0 &&
                  P_BF1 % 4 == 0 && P_WF2 % 4 == 0 && P_BF2 % 4 == 0,
              "conv1 = torch [0, P_W2) = slab [SL_SMALL, + P_W2); no float4 straddles two tensors");

// four consecutive floats: one float4 access when the operands are 16-byte aligned (R.vec)
__device__ __forceinline__ float4 ld4(const float* p, bool vec) {
    if (vec) return *reinterpret_cast<const float4*>(p);
    return make_float4(p[0], p[1], p[2], p[3]);
}
__device__ __forceinline__ void st4(float* p, float4 v, bool vec) {
    if (vec) {
        *reinterpret_cast<float4*>(p) = v;
    } else {
        p[0] = v.x;
        p[1] = v.y;
        p[2] = v.z;
        p[3] = v.w;
    }
}

__global__ __launch_bounds__(256) void k_reduce_pre(const float* slab, int nslab, const float* pre,
                                                    float* grad, float* loss, ReduceAdam R) {
    __shared__ float4 part[16][16];
    const int t = threadIdx.x;
    const bool c1 = (int)blockIdx.x >= NB_PRE4;
    if (!c1 && t >= PRE_F4_PER_BLOCK) return;  // (no barrier in these blocks)
    const int q = c1 ? ((int)blockIdx.x - NB_PRE4) * C1_PER_BLOCK + (t & 15)
                     : (int)blockIdx.x * PRE_F4_PER_BLOCK + t;
    const bool fin = c1 ? t < C1_PER_BLOCK : q >= C1_Q4 && q < TQ4;
    const bool is_loss = q == TQ4 - 1;
    const bool adam = R.on && fin && !is_loss;
    const bool vec = R.vec != 0;
    // the Adam operands, loaded with the sums (independent of them)
    constexpr int off[8] = {P_W1, P_B1, P_W2, P_B2, P_WF1, P_BF1, P_WF2, P_BF2};
    int k = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j) k += q * 4 >= off[j] ? 1 : 0;
    const int ei = q * 4 - off[k];
    unsigned long long st = 0;
    float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f), v4 = m4, p4v = m4;
    if (adam) {
        st = *R.step;
        m4 = ld4(R.m + q * 4, vec);
        v4 = ld4(R.v + q * 4, vec);
        p4v = ld4(R.p[k] + ei, vec);
    }
    float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!c1) {
        if (fin) sv = reinterpret_cast<const float4*>(pre)[q];
    } else {
        const int j = t >> 4;
        const int s4 = C1_F4_LO + q;
        for (int g0 = 0; g0 < nslab; g0 += 256) {
            float4 r[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int g = g0 + j + 16 * u;
                r[u] = g < nslab ? reinterpret_cast<const float4*>(slab + (int64_t)g * SLAB)[s4]
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                sv.x += r[u].x;
                sv.y += r[u].y;
                sv.z += r[u].z;
                sv.w += r[u].w;
            }
        }
        part[j][t & 15] = sv;
    }
    g2048::AdamCoef c{};
    if (adam) c = g2048::adam_coef((double)st, R.lr, R.b1, R.b2, R.eps);
    if (c1) {
        __syncthreads();
        if (!fin) return;
        sv = part[0][t];
#pragma unroll
        for (int j = 1; j < 16; ++j) {
            const float4 pj = part[j][t];
            sv.x += pj.x;
            sv.y += pj.y;
            sv.z += pj.z;
            sv.w += pj.w;
        }
    }
    if (!fin) return;
    if (is_loss) {
        if (loss) *loss = sv.x;
        return;
    }
    if (grad) st4(grad + q * 4, sv, vec);
    if (!adam) return;
    const float4 n4 = make_float4(g2048::adam_update(c, sv.x, m4.x, v4.x, p4v.x),
                                  g2048::adam_update(c, sv.y, m4.y, v4.y, p4v.y),
                                  g2048::adam_update(c, sv.z, m4.z, v4.z, p4v.z),
                                  g2048::adam_update(c, sv.w, m4.w, v4.w, p4v.w));
    st4(R.m + q * 4, m4, vec);
    st4(R.v + q * 4, v4, vec);
    st4(R.p[k] + ei, n4, vec);
    if (R.sync_every && st % R.sync_every == 0ull) st4(R.tp[k] + ei, n4, vec);
}

// Deterministic slab reduction (without `pre`: small batches, grid < SHADOW_MIN_GRID): a block
// owns 256 slab positions (a float4 per lane); its 16 waves sum the slabs g = wave, wave + 16, ...
// (16 independent float4 loads per lane in flight: one memory round trip per 256 slabs), then the
// 16 partials are added in a fixed order.
constexpr int RW = 16;  // waves per reduction block

__global__ __launch_bounds__(64 * RW) void k_reduce_slabs(const float* slab, int nslab,
                                                          float* grad, float* loss, ReduceAdam R) {
    __shared__ float4 part[RW][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p4 = (int)blockIdx.x * 64 + lane;  // float4 index within a slab
    const bool in = p4 * 4 <= SL_LOSS;
    const bool fin = wave == 0 && in;
    const bool adam = R.on && fin;
    AdamLane L;
    unsigned long long t = 0;
    if (adam) {
        t = *R.step;
        adam_load(R, p4, L);
    }
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int g0 = 0; g0 < nslab; g0 += RW * 16) {
        float4 r[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int g = g0 + wave + RW * u;
            r[u] = (in && g < nslab) ? reinterpret_cast<const float4*>(slab + (int64_t)g * SLAB)[p4]
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            v.x += r[u].x;
            v.y += r[u].y;
            v.z += r[u].z;
            v.w += r[u].w;
        }
    }
    // Adam's step scalars (two f64 pow) formed while the loads are in flight, not after the
    // barrier on the update's critical path
    g2048::AdamCoef c{};
    if (adam) c = g2048::adam_coef((double)t, R.lr, R.b1, R.b2, R.eps);
    part[wave][lane] = v;
    __syncthreads();
    if (!fin) return;
    float4 sv = part[0][lane];
#pragma unroll
    for (int k = 1; k < RW; ++k) {
        sv.x += part[k][lane].x;
        sv.y += part[k][lane].y;
        sv.z += part[k][lane].z;
        sv.w += part[k][lane].w;
    }
    finish4(R, adam, c, t, p4, sv, L, grad, loss);
}

}  // namespace

static int64_t train_grid(int64_t batch) {
    const int64_t ntiles = (batch + S - 1) / S;
    int64_t g = ntiles < 256 ? ntiles : 256;
    if (g * TMAXT < ntiles) g = (ntiles + TMAXT - 1) / TMAXT;
    return g;
}

// float offset of train bwd's slab sums (16-byte aligned)
static int64_t pre_offset(int64_t batch) {
    const int64_t ntiles = (batch + S - 1) / S;
    return (train_grid(batch) * SLAB + ntiles * DM_TILE + conv_split_floats(batch) + 3) & ~3ll;
}

extern "C" G2048_API int64_t g2048_convnet_train_workspace(int64_t batch) {
    if (batch <= 0) return 0;
    // slabs | dM of every tile | split-target scratch of g2048_convnet_update | train bwd's sums
    return pre_offset(batch) + SLAB;
}

static float* split_scratch(float* workspace, int64_t batch) {
    const int64_t ntiles = (batch + S - 1) / S;
    return workspace + train_grid(batch) * SLAB + ntiles * DM_TILE;
}

static int train_launch(const g2048_convnet_params* p, const uint8_t* rows,
                        const uint8_t* actions, const int64_t* idx, const float* y, int64_t batch,
                        float* workspace, float* grad_out, float* loss_out, uint64_t* step_dev,
                        const ReduceAdam& R, void* stream, const float* split = nullptr,
                        float* y_out = nullptr) {
    ReduceAdam Rv = R;
    {
        auto a16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0u; };
        bool ok = a16(grad_out);
        if (R.on) {
            ok = ok && a16(R.m) && a16(R.v);
            for (int k = 0; k < 8; ++k) ok = ok && a16(R.p[k]) && (!R.sync_every || a16(R.tp[k]));
        }
        Rv.vec = ok;
    }
    TrainArgs A{};
    A.W = NetW{p->w1, p->b1, p->w2, p->b2, p->fc1_w, p->fc1_b, p->fc2_w, p->fc2_b};
    A.rows = rows;
    A.actions = actions;
    A.idx = idx;
    A.y = y;
    A.astar = split ? reinterpret_cast<const int32_t*>(split) : nullptr;
    A.qtg = split ? reinterpret_cast<const float4*>(split + conv_split_qtg_offset(batch)) : nullptr;
    A.rdisc = split ? reinterpret_cast<const float2*>(split + conv_split_rd_offset(batch)) : nullptr;
    A.y_out = y_out;
    A.batch = batch;
    A.slab = workspace;
    const int grid = (int)train_grid(batch);
    A.dm = workspace + (int64_t)grid * SLAB;
    A.pre = grid >= SHADOW_MIN_GRID ? workspace + pre_offset(batch) : nullptr;
    A.step = reinterpret_cast<unsigned long long*>(step_dev);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_conv_train_fwd, dim3(grid), dim3(NT), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_conv_train_fwd: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(k_conv_train_bwd, dim3(grid), dim3(NT), 0, st, A);
    e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_conv_train_bwd: %s", hipGetErrorString(e));
    if (A.pre)
        hipLaunchKernelGGL(k_reduce_pre, dim3(NB_PRE4 + C1_BLOCKS), dim3(256), 0, st, workspace,
                           grid, A.pre, grad_out, loss_out, Rv);
    else
        hipLaunchKernelGGL(k_reduce_slabs, dim3((SL_LOSS / 4 + 64) / 64), dim3(64 * RW), 0, st,
                           workspace, grid, grad_out, loss_out, Rv);
    e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "k_reduce_slabs: %s", hipGetErrorString(e));
}

static bool ok_params(const g2048_convnet_params* p) {
    return p && p->w1 && p->b1 && p->w2 && p->b2 && p->fc1_w && p->fc1_b && p->fc2_w && p->fc2_b;
}

extern "C" G2048_API int g2048_convnet_train_grad(const g2048_convnet_params* p,
                                                  const uint8_t* rows, const uint8_t* actions,
                                                  const int64_t* idx, const float* y, int64_t batch,
                                                  float* workspace, float* grad_out,
                                                  float* loss_out, uint64_t* step_dev,
                                                  void* stream) {
    if (!ok_params(p) || !rows || !actions || !idx || !y || !workspace || !grad_out || batch <= 0)
        return g2048_fail(G2048_EINVAL, "convnet_train_grad: NULL argument or batch <= 0");
    ReduceAdam R;
    memset(&R, 0, sizeof(R));
    return train_launch(p, rows, actions, idx, y, batch, workspace, grad_out, loss_out, step_dev,
                        R, stream);
}

static void fill_adam(ReduceAdam& R, const g2048_convnet_params* p,
                      const g2048_convnet_params* target, uint64_t sync_every, float* m, float* v,
                      const uint64_t* step_dev, double lr, double beta1, double beta2,
                      double eps) {
    memset(&R, 0, sizeof(R));
    const g2048_convnet_params* nets[2] = {p, sync_every ? target : nullptr};
    for (int h = 0; h < 2; ++h) {
        if (!nets[h]) continue;
        const float* ps[8] = {nets[h]->w1, nets[h]->b1, nets[h]->w2, nets[h]->b2,
                              nets[h]->fc1_w, nets[h]->fc1_b, nets[h]->fc2_w, nets[h]->fc2_b};
        for (int k = 0; k < 8; ++k) (h ? R.tp : R.p)[k] = const_cast<float*>(ps[k]);
    }
    R.m = m;
    R.v = v;
    R.step = reinterpret_cast<const unsigned long long*>(step_dev);
    R.lr = lr;
    R.b1 = beta1;
    R.b2 = beta2;
    R.eps = eps;
    R.sync_every = sync_every;
    R.on = 1;
}

extern "C" int g2048_conv_targets_launch(const g2048_convnet_params* online,
                                         const g2048_convnet_params* target, g2048_replay* rb,
                                         const int64_t* idx_in, int64_t batch, uint64_t seed,
                                         const uint64_t* epoch_dev, float gamma, int double_dqn,
                                         int64_t* idx_out, float* y_out, float* split_ws,
                                         void* stream);

extern "C" G2048_API int g2048_convnet_update(
    const g2048_convnet_params* online, const g2048_convnet_params* target, g2048_replay* rb,
    const int64_t* idx_in, int64_t batch, uint64_t seed, uint64_t* step_dev, float gamma,
    int double_dqn, int64_t* idx_out, float* y_out, float* workspace, float* grad_out,
    float* loss_out, float* exp_avg, float* exp_avg_sq, double lr, double beta1, double beta2,
    double eps, uint64_t sync_every, void* stream) {
    if (!ok_params(online) || !ok_params(target) || !rb || batch <= 0 || !step_dev ||
        !idx_out || !y_out || !workspace)
        return g2048_fail(G2048_EINVAL, "convnet_update: NULL argument or batch <= 0");
    const bool adam = exp_avg && exp_avg_sq;
    if (!adam && !grad_out)
        return g2048_fail(G2048_EINVAL, "convnet_update: no Adam state and no grad_out");
    uint8_t* s = nullptr;
    uint8_t* a = nullptr;
    if (g2048_replay_views(rb, &s, nullptr, &a, nullptr, nullptr, nullptr) != G2048_OK)
        return G2048_EINVAL;
    float* split = double_dqn ? split_scratch(workspace, batch) : nullptr;
    int rc = g2048_conv_targets_launch(online, target, rb, idx_in, batch, seed, step_dev, gamma,
                                       double_dqn, idx_out, y_out, split, stream);
    if (rc != G2048_OK) return rc;
    ReduceAdam R;
    if (adam)
        fill_adam(R, online, target, sync_every, exp_avg, exp_avg_sq, step_dev, lr, beta1, beta2,
                  eps);
    else
        memset(&R, 0, sizeof(R));
    return train_launch(online, s, a, idx_out, y_out, batch, workspace, grad_out, loss_out,
                        step_dev, R, stream, split, split ? y_out : nullptr);
}

extern "C" G2048_API int g2048_convnet_train_adam(
    const g2048_convnet_params* p, const uint8_t* rows, const uint8_t* actions,
    const int64_t* idx, const float* y, int64_t batch, float* workspace, float* grad_out,
    float* loss_out, uint64_t* step_dev, float* exp_avg, float* exp_avg_sq, double lr,
    double beta1, double beta2, double eps, const g2048_convnet_params* target,
    uint64_t sync_every, void* stream) {
    if (!ok_params(p) || !rows || !actions || !idx || !y || !workspace || !step_dev || !exp_avg ||
        !exp_avg_sq || batch <= 0)
        return g2048_fail(G2048_EINVAL, "convnet_train_adam: NULL argument or batch <= 0");
    if (sync_every && !ok_params(target))
        return g2048_fail(G2048_EINVAL, "convnet_train_adam: sync_every > 0 needs the target net");
    ReduceAdam R;
    fill_adam(R, p, target, sync_every, exp_avg, exp_avg_sq, step_dev, lr, beta1, beta2, eps);
    return train_launch(p, rows, actions, idx, y, batch, workspace, grad_out, loss_out, step_dev,
                        R, stream);
}
