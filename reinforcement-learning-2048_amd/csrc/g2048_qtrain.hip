// g2048_qtrain.hip -- fused Double-DQN gradient of the reference conv Q-net on gfx950 f32 MFMA.
//
// One launch computes, for a minibatch of B replay rows (indices idx, Bellman targets y):
//   q_b = Q(s_b)[a_b],  loss = sum_b (q_b - y_b)^2,  and d loss / d theta for all 33 476 params
// = the graded half of the reference train_step (src/dqn_lib.py:146-161: model(states), the
// one-hot gather, MSELoss(reduction='sum'), loss.backward()).  A second launch reduces the
// per-workgroup partial gradients (fixed order -> deterministic) straight into the learner's
// flat gradient bucket in torch's parameter layout, so Adam / the RCCL all-reduce follow as usual.
//
// Per tile of S = 32 boards (256 threads = 4 waves, everything in LDS / registers):
//   fwd   conv2 [128 x 256] @ W2t [256 x 64]    MFMA 32x32x2, A = conv1 output recomputed from
//                                               the board in registers (h1 is never stored)
//         fc1   [32 x 256] @ Wf1t [256 x 64]    MFMA 16x16x4
//         fc2 + loss + dq                       VALU
//   bwd   dWf2, dbf2, df, dbf1                   VALU
//         dWf1 += df^T [64 x 32] @ h2 [32 x 256]       MFMA (accumulators persist across tiles)
//         dh2   = df [32 x 64] @ Wf1 [64 x 256] * relu' MFMA
//         dW2^T += P^T [256 x 128] @ dh2 [128 x 64]     MFMA (A = recomputed conv1 patches)
//         dP    = dh2 [128 x 64] @ W2 [64 x 256]        MFMA; its epilogue folds the col2im +
//               relu' of conv1 straight into per-lane dW1 / db1 sums (dh1 is never stored)
// The weight matrix needed by each phase is staged into one 65 KB LDS region (padded strides).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/g2048.h"
#include "g2048_common.hpp"

namespace {

constexpr int S = 32;
constexpr int NT = 256;
constexpr int WT_STRIDE = 65;   // transposed weights [k][n]
constexpr int WR_STRIDE = 257;  // row-major weights [row][256]
constexpr int H2_STRIDE = 257;  // h2 / dh2 [s][q*64 + c']
constexpr int F_STRIDE = 65;    // f / df [s][j]

// parameter offsets in torch order (Conv2048.parameters())
constexpr int P_W1 = 0, P_B1 = 256, P_W2 = 320, P_B2 = 16704, P_WF1 = 16768, P_BF1 = 33152,
              P_WF2 = 33216, P_BF2 = 33472, P_TOTAL = 33476;
// slab layout (kernel order): [W2 tiles 16384 | Wf1 tiles 16384 | w1 256 | b1 64 | b2 64 |
//                              bf1 64 | wf2 256 | bf2 4 | loss 1], padded
constexpr int SL_W2 = 0, SL_WF1 = 16384, SL_SMALL = 32768, SL_LOSS = SL_SMALL + 708;
constexpr int SLAB = 33480;
static_assert(SL_LOSS + 1 <= SLAB && SL_SMALL + 708 == P_TOTAL - 16384 * 2 + SL_SMALL, "slab layout");

// LDS carve (floats)
constexpr int OFF_X = 0;                          // [S][16]
constexpr int OFF_W1 = OFF_X + S * 16;            // [64][4]
constexpr int OFF_B1 = OFF_W1 + 256;
constexpr int OFF_B2 = OFF_B1 + 64;
constexpr int OFF_BF1 = OFF_B2 + 64;
constexpr int OFF_WF2 = OFF_BF1 + 64;             // [4][65]
constexpr int OFF_BF2 = OFF_WF2 + 4 * 65;         // 4
constexpr int OFF_A = OFF_BF2 + 4;                // actions [S] (as float)
constexpr int OFF_Y = OFF_A + S;                  // targets [S]
constexpr int OFF_G = OFF_Y + S;                  // dq [S]
constexpr int OFF_H2 = (OFF_G + S + 3) & ~3;      // [S][257]
constexpr int OFF_F = OFF_H2 + ((S * H2_STRIDE + 3) & ~3);  // [S][65]
constexpr int OFF_W = OFF_F + ((S * F_STRIDE + 3) & ~3);    // max(256*65, 64*257)
constexpr int W_FLOATS = 64 * WR_STRIDE > 256 * WT_STRIDE ? 64 * WR_STRIDE : 256 * WT_STRIDE;
constexpr int OFF_RED = OFF_W;                    // reused at the end for the dW1/db1 reduction
constexpr int LDS_FLOATS = OFF_W + W_FLOATS;
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
static_assert(NT * 10 <= W_FLOATS, "reduction scratch");

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct TrainArgs {
    const float *w1, *b1, *w2, *b2, *wf1, *bf1, *wf2, *bf2;
    const uint8_t* rows;     // replay s rows [*][16]
    const uint8_t* actions;  // replay a [*]
    const int64_t* idx;      // [B]
    const float* y;          // [B] Bellman targets
    int64_t batch;
    float* slab;             // [gridDim.x][SLAB]
    unsigned long long* step;  // optional update counter, += 1 by one thread (nullable)
};

// conv1 pre-activation of board s (x in LDS) at output position (ph, pw), channel weights w/b
[[maybe_unused]] __device__ __forceinline__ float conv1_pre(const float* x, int ph, int pw, float4 w, float b) {
    float v = b;
    v = fmaf(w.x, x[ph * 4 + pw], v);
    v = fmaf(w.y, x[ph * 4 + pw + 1], v);
    v = fmaf(w.z, x[(ph + 1) * 4 + pw], v);
    v = fmaf(w.w, x[(ph + 1) * 4 + pw + 1], v);
    return v;
}

__device__ __forceinline__ int acc_row32(int i, int lane) {  // 32x32 C/D row of register i
    return (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
}

#ifdef G2048_PHASE_PROF
__device__ unsigned long long g_tphase[4][16];
#define TPHASE(k)                                                         \
    do {                                                                  \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
        ph[k] += now_ - ph_last;                                          \
        ph_last = now_;                                                   \
    } while (0)
#else
#define TPHASE(k) do {} while (0)
#endif

__global__ __launch_bounds__(NT) void k_conv_train(TrainArgs A) {
#ifdef G2048_PHASE_PROF
    unsigned long long ph[16] = {0}, ph_last = __builtin_amdgcn_s_memtime();
#endif
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
    float* xs = lds + OFF_X;
    float* sw1 = lds + OFF_W1;
    float* sb1 = lds + OFF_B1;
    float* sb2 = lds + OFF_B2;
    float* sbf1 = lds + OFF_BF1;
    float* swf2 = lds + OFF_WF2;
    float* sbf2 = lds + OFF_BF2;
    float* sa = lds + OFF_A;
    float* sy = lds + OFF_Y;
    float* sg = lds + OFF_G;
    float* h2 = lds + OFF_H2;
    float* fa = lds + OFF_F;
    float* w = lds + OFF_W;

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int half = lane >> 5, l32 = lane & 31;
    // nothing else in this launch reads the counter; stream order makes the bump visible to the
    // following optimizer launch and to the next update's sampler
    if (A.step && blockIdx.x == 0 && t == 0) *A.step += 1ull;

    // small weights, once per workgroup
    sw1[t] = A.w1[t];
    if (t < 64) {
        sb1[t] = A.b1[t];
        sb2[t] = A.b2[t];
        sbf1[t] = A.bf1[t];
    }
    swf2[(t >> 6) * 65 + (t & 63)] = A.wf2[t];
    if (t < 4) sbf2[t] = A.bf2[t];

    // persistent accumulators
    f32x16 accWf1[4], accW2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        accWf1[i] = f32x16{0};
        accW2[i] = f32x16{0};
    }
    float accw1[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, accb1[2] = {0, 0};
    float accWf2 = 0.f, accBf2 = 0.f, accBf1 = 0.f, accB2 = 0.f, accLoss = 0.f;

    // W2 and fc1_w columns of this thread (w2[i][t], wf1[i][t], i < 64), loaded once in one
    // batch; the four per-tile LDS layouts below are stored from these registers
    float vW2[64], vF[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        vW2[i] = A.w2[i * NT + t];
        vF[i] = A.wf1[i * NT + t];
    }

    const int64_t ntiles = (A.batch + S - 1) / S;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b0 = tile * S;
        __syncthreads();  // previous tile fully consumed
        TPHASE(0);
        // ---- A: boards, actions, targets; W2 transposed into w[k][n]
        if (t < S * 4) {
            const int s = t >> 2, wd = t & 3;
            const int64_t b = b0 + s;
            uint32_t v = 0;
            if (b < A.batch) v = reinterpret_cast<const uint32_t*>(A.rows)[A.idx[b] * 4 + wd];
            float* dst = xs + s * 16 + wd * 4;
            dst[0] = (float)(v & 0xFFu);
            dst[1] = (float)((v >> 8) & 0xFFu);
            dst[2] = (float)((v >> 16) & 0xFFu);
            dst[3] = (float)(v >> 24);
        }
        if (t < S) {
            const int64_t b = b0 + t;
            const bool ok = b < A.batch;
            sa[t] = ok ? (float)A.actions[A.idx[b]] : 0.f;
            sy[t] = ok ? A.y[b] : 0.f;
            sg[t] = ok ? 1.f : 0.f;  // validity, replaced by dq in phase E
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) w[t * WT_STRIDE + i] = vW2[i];
        __syncthreads();

        TPHASE(1);
        // ---- B: conv2 forward.  rows r = 32*wave + l32 (board s = r>>2, position q = r&3)
        {
            f32x16 c0 = f32x16{0}, c1 = f32x16{0};
            const int r = wave * 32 + l32, s = r >> 2, q = r & 3, qh = q >> 1, qw = q & 1;
            const float* x = xs + s * 16;
            // k = 2kk + half: kw = half is fixed per lane and kh = kk & 1, so the lane only ever
            // reads the 3x2 window xv[rr][cc] = x[qh + rr][qw + half + cc] -- in registers, the
            // same products in the same order as conv1_pre
            float xv[3][2];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                for (int cc = 0; cc < 2; ++cc) xv[rr][cc] = x[(qh + rr) * 4 + qw + half + cc];
            // chunks of 16 k-steps: the 16 conv1 operands as independent VALU chains first
            // (full issue rate), then their 32 MFMAs with no VALU in between (a dependent conv1
            // chain feeding every MFMA is not hidden at one wave per SIMD)
#pragma unroll 1
            for (int ch = 0; ch < 8; ++ch) {
                float av[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int c = (ch * 32 + 2 * j) >> 2, kh = j & 1;
                    const float4 wc = *reinterpret_cast<const float4*>(sw1 + c * 4);
                    float pre = sb1[c];
                    pre = fmaf(wc.x, xv[kh][0], pre);
                    pre = fmaf(wc.y, xv[kh][1], pre);
                    pre = fmaf(wc.z, xv[kh + 1][0], pre);
                    pre = fmaf(wc.w, xv[kh + 1][1], pre);
                    av[j] = fmaxf(pre, 0.f);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int k = 2 * (ch * 16 + j) + half;
                    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], w[k * WT_STRIDE + l32], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], w[k * WT_STRIDE + 32 + l32], c1, 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int rr = wave * 32 + acc_row32(i, lane), ss = rr >> 2, qq = rr & 3;
                h2[ss * H2_STRIDE + qq * 64 + l32] = fmaxf(c0[i] + sb2[l32], 0.f);
                h2[ss * H2_STRIDE + qq * 64 + 32 + l32] = fmaxf(c1[i] + sb2[32 + l32], 0.f);
            }
        }
        __syncthreads();
        TPHASE(2);
        // ---- C: Wf1 transposed into w[k'][j], k' = q*64 + c' (h2's order), m = c'*4 + q
#pragma unroll
        for (int i = 0; i < 64; ++i) w[((t & 3) * 64 + (t >> 2)) * WT_STRIDE + i] = vF[i];
        __syncthreads();
        TPHASE(3);
        // ---- D: fc1 forward (16x16x4) -> f
        {
            const int mt = wave & 1, nt0 = (wave >> 1) * 2, arow = mt * 16 + (lane & 15);
            const int kq = lane >> 4, ncol = lane & 15;
            f32x4 c0 = f32x4{0}, c1 = f32x4{0};
#pragma unroll 8
            for (int kk = 0; kk < 64; ++kk) {
                const int k = 4 * kk + kq;
                const float a = h2[arow * H2_STRIDE + k];
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[k * WT_STRIDE + nt0 * 16 + ncol], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[k * WT_STRIDE + (nt0 + 1) * 16 + ncol], c1, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = mt * 16 + (lane >> 4) * 4 + i;
                const int ja = nt0 * 16 + ncol, jb = (nt0 + 1) * 16 + ncol;
                fa[row * F_STRIDE + ja] = fmaxf(c0[i] + sbf1[ja], 0.f);
                fa[row * F_STRIDE + jb] = fmaxf(c1[i] + sbf1[jb], 0.f);
            }
        }
        __syncthreads();
        TPHASE(4);
        // ---- E: fc2 at the taken action, loss, dq = 2 (q - y)
        if (t < S) {
            const int a = (int)sa[t];
            float q = sbf2[a];
#pragma unroll 16
            for (int j = 0; j < 64; ++j) q = fmaf(swf2[a * 65 + j], fa[t * F_STRIDE + j], q);
            const float d = (q - sy[t]) * sg[t];
            accLoss = fmaf(d, d, accLoss);
            sg[t] = 2.f * d;
        }
        __syncthreads();
        TPHASE(5);
        // ---- F: dWf2 / dbf2 (thread = (action a, unit j)); stage Wf1 row-major, permuted columns
        {
            const int a = t >> 6, j = t & 63;
            float gw = 0.f, gb = 0.f;
#pragma unroll 8
            for (int s = 0; s < S; ++s) {
                const float g = (int)sa[s] == a ? sg[s] : 0.f;
                gw = fmaf(g, fa[s * F_STRIDE + j], gw);
                gb += g;
            }
            accWf2 += gw;
            if (j == 0) accBf2 += gb;
        }
        // w[j][k'] (stride 257) = wf1[j][m], k' = q*64 + c', m = c'*4 + q
#pragma unroll
        for (int i = 0; i < 64; ++i) w[i * WR_STRIDE + (t & 3) * 64 + (t >> 2)] = vF[i];
        __syncthreads();
        TPHASE(6);
        // ---- G: df = dq * Wf2[a] * relu'(f), in place over f
        {
            const int s = t >> 3, j0 = (t & 7) * 8;
            const int a = (int)sa[s];
            const float g = sg[s];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const int j = j0 + jj;
                const float f = fa[s * F_STRIDE + j];
                fa[s * F_STRIDE + j] = f > 0.f ? g * swf2[a * 65 + j] : 0.f;
            }
        }
        __syncthreads();
        TPHASE(7);
        // ---- H: dbf1; dWf1 += df^T @ h2 (persistent); dh2_pre = df @ Wf1p
        if (t < 64) {
            float v = 0.f;
#pragma unroll 8
            for (int s = 0; s < S; ++s) v += fa[s * F_STRIDE + t];
            accBf1 += v;
        }
        {
            const int jt = wave & 1, mt0 = (wave >> 1) * 4;
#pragma unroll 4
            for (int kk = 0; kk < S / 2; ++kk) {
                const int s = 2 * kk + half;
                const float a = fa[s * F_STRIDE + jt * 32 + l32];
#pragma unroll
                for (int tt = 0; tt < 4; ++tt)
                    accWf1[tt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                        a, h2[s * H2_STRIDE + (mt0 + tt) * 32 + l32], accWf1[tt], 0, 0, 0);
            }
        }
        f32x16 dh0 = f32x16{0}, dh1 = f32x16{0};
        {
            const int nt0 = wave * 2;
#pragma unroll 4
            for (int kk = 0; kk < 32; ++kk) {
                const int j = 2 * kk + half;
                const float a = fa[l32 * F_STRIDE + j];
                dh0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w[j * WR_STRIDE + nt0 * 32 + l32], dh0, 0, 0, 0);
                dh1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w[j * WR_STRIDE + (nt0 + 1) * 32 + l32], dh1, 0, 0, 0);
            }
        }
        __syncthreads();  // every read of h2 (dWf1) and of Wf1p is done
        TPHASE(8);
        // ---- I: dh2 = dh2_pre * relu'(h2), in place over h2
        {
            const int nt0 = wave * 2;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int s = acc_row32(i, lane);
                float* p0 = h2 + s * H2_STRIDE + nt0 * 32 + l32;
                float* p1 = p0 + 32;
                *p0 = *p0 > 0.f ? dh0[i] : 0.f;
                *p1 = *p1 > 0.f ? dh1[i] : 0.f;
            }
        }
        // stage W2 row-major w[c'][k] (stride 257) for dP
#pragma unroll
        for (int i = 0; i < 64; ++i) w[i * WR_STRIDE + t] = vW2[i];
        __syncthreads();
        TPHASE(9);
        // ---- J: db2; dW2^T += P^T @ dh2 (persistent; A = recomputed conv1 patches)
        if (t < 64) {
            float v = 0.f;
#pragma unroll 8
            for (int s = 0; s < S; ++s)
                v += h2[s * H2_STRIDE + t] + h2[s * H2_STRIDE + 64 + t] + h2[s * H2_STRIDE + 128 + t] +
                     h2[s * H2_STRIDE + 192 + t];
            accB2 += v;
        }
        {
            // lane row k = kt*32 + l32 for kt in {2*wave, 2*wave+1}: c, kh, kw fixed per lane
            // (kh, kw the same for both kt).  Row m = 2kk + half: board kk >> 1, position
            // (qh, qw) = (kk & 1, half).  Chunks of 8 k-steps: the 16 conv1 operands from a 3x2
            // register window of each of the chunk's 4 boards (independent VALU chains, the
            // products of conv1_pre in its order), then their 32 MFMAs.
            const int kdh = (l32 >> 1) & 1, kdw = l32 & 1;
            float4 wc[2];
            float bc[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int c = ((2 * wave + u) * 32 + l32) >> 2;
                wc[u] = *reinterpret_cast<const float4*>(sw1 + c * 4);
                bc[u] = sb1[c];
            }
#pragma unroll 1
            for (int ch = 0; ch < 8; ++ch) {
                float av[2][8];
#pragma unroll
                for (int jb = 0; jb < 4; ++jb) {
                    const float* x = xs + (4 * ch + jb) * 16;
                    float xv[3][2];
#pragma unroll
                    for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                        for (int cc = 0; cc < 2; ++cc) xv[rr][cc] = x[(kdh + rr) * 4 + half + kdw + cc];
#pragma unroll
                    for (int e = 0; e < 2; ++e)
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            float pre = bc[u];
                            pre = fmaf(wc[u].x, xv[e][0], pre);
                            pre = fmaf(wc[u].y, xv[e][1], pre);
                            pre = fmaf(wc[u].z, xv[e + 1][0], pre);
                            pre = fmaf(wc[u].w, xv[e + 1][1], pre);
                            av[u][2 * jb + e] = fmaxf(pre, 0.f);
                        }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int m = 2 * (8 * ch + j) + half, s = m >> 2, q = m & 3;
                    const float g0 = h2[s * H2_STRIDE + q * 64 + l32];
                    const float g1 = h2[s * H2_STRIDE + q * 64 + 32 + l32];
                    accW2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][j], g0, accW2[0], 0, 0, 0);
                    accW2[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][j], g1, accW2[1], 0, 0, 0);
                    accW2[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][j], g0, accW2[2], 0, 0, 0);
                    accW2[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][j], g1, accW2[3], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        TPHASE(10);
        // ---- K: dP = dh2 @ W2 per (m-tile, k-tile); epilogue folds col2im + relu'(h1) into
        //         per-lane dW1 / db1 sums.  Lane col k_u = (2*wave + u)*32 + l32: kh, kw are
        //         the same for both u (k & 3 = l32 & 3), so per m-tile one MFMA loop makes both
        //         k-tiles (shared A operand), and the lane's 3x3 input window of each of its 4
        //         boards is read once into registers for both epilogues.
        {
            const int kh = (l32 >> 1) & 1, kw = l32 & 1;
            float4 wc[2];
            float bc[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int c = ((2 * wave + u) * 32 + l32) >> 2;
                wc[u] = *reinterpret_cast<const float4*>(sw1 + c * 4);
                bc[u] = sb1[c];
            }
#pragma unroll 1
            for (int mt = 0; mt < 4; ++mt) {
                f32x16 dp0 = f32x16{0}, dp1 = f32x16{0};
                const int m = mt * 32 + l32, s = m >> 2, q = m & 3;
#pragma unroll 8
                for (int kk = 0; kk < 32; ++kk) {
                    const int cp = 2 * kk + half;
                    const float av = h2[s * H2_STRIDE + q * 64 + cp];
                    dp0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, w[cp * WR_STRIDE + (2 * wave) * 32 + l32], dp0, 0, 0, 0);
                    dp1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, w[cp * WR_STRIDE + (2 * wave + 1) * 32 + l32], dp1, 0, 0, 0);
                }
                // rows of register i: board sr = mt*8 + 2*(i>>2) + half, position qr = i & 3
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float* x = xs + (mt * 8 + 2 * j + half) * 16;
                    float xw[3][3];
#pragma unroll
                    for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                        for (int cc = 0; cc < 3; ++cc) xw[rr][cc] = x[(kh + rr) * 4 + kw + cc];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
#pragma unroll
                        for (int qr = 0; qr < 4; ++qr) {
                            const int qh = qr >> 1, qw = qr & 1, i = 4 * j + qr;
                            const float x00 = xw[qh][qw], x01 = xw[qh][qw + 1];
                            const float x10 = xw[qh + 1][qw], x11 = xw[qh + 1][qw + 1];
                            float pre = bc[u];  // conv1_pre's products, in its order
                            pre = fmaf(wc[u].x, x00, pre);
                            pre = fmaf(wc[u].y, x01, pre);
                            pre = fmaf(wc[u].z, x10, pre);
                            pre = fmaf(wc[u].w, x11, pre);
                            const float v = pre > 0.f ? (u ? dp1[i] : dp0[i]) : 0.f;
                            accb1[u] += v;
                            accw1[u][0] = fmaf(v, x00, accw1[u][0]);
                            accw1[u][1] = fmaf(v, x01, accw1[u][1]);
                            accw1[u][2] = fmaf(v, x10, accw1[u][2]);
                            accw1[u][3] = fmaf(v, x11, accw1[u][3]);
                        }
                    }
                }
            }
        }
    }
    __syncthreads();

    TPHASE(11);
    // ---- write this workgroup's partial gradient slab (coalesced, kernel order)
    float* slab = A.slab + (int64_t)blockIdx.x * SLAB;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            slab[SL_W2 + ((wave * 4 + tt) * 16 + i) * 64 + lane] = accW2[tt][i];
            slab[SL_WF1 + ((wave * 4 + tt) * 16 + i) * 64 + lane] = accWf1[tt][i];
        }
    // conv1 grads: lanes (kh,kw) of one channel and both halves -> deterministic LDS reduction
    float* red = lds + OFF_RED;  // [t][u*5 + {w0..w3, b}]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) red[t * 10 + u * 5 + i] = accw1[u][i];
        red[t * 10 + u * 5 + 4] = accb1[u];
    }
    __syncthreads();
    if (t < 64) {  // channel c = t: k = 4c + kk4 -> kt = k >> 5, lane l32 = k & 31
        const int c = t;
        float gw[4] = {0, 0, 0, 0}, gb = 0.f;
#pragma unroll
        for (int kk4 = 0; kk4 < 4; ++kk4) {
            const int k = c * 4 + kk4, kt = k >> 5, l = k & 31;
            const int wv = kt >> 1, u = kt & 1;
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int tt = wv * 64 + hh * 32 + l;
#pragma unroll
                for (int i = 0; i < 4; ++i) gw[i] += red[tt * 10 + u * 5 + i];
                gb += red[tt * 10 + u * 5 + 4];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[SL_SMALL + c * 4 + i] = gw[i];
        slab[SL_SMALL + 256 + c] = gb;
        slab[SL_SMALL + 320 + c] = accB2;
        slab[SL_SMALL + 384 + c] = accBf1;
    }
    slab[SL_SMALL + 448 + t] = accWf2;  // wf2[a][j], t = a*64 + j
    if ((t & 63) == 0) slab[SL_SMALL + 704 + (t >> 6)] = accBf2;
    // loss: threads 0..31 hold per-sample partials
    __syncthreads();
    red[t] = accLoss;
    __syncthreads();
    if (t == 0) {
        float v = 0.f;
        for (int i = 0; i < S; ++i) v += red[i];
        slab[SL_LOSS] = v;
    }
    TPHASE(12);
#ifdef G2048_PHASE_PROF
    if (blockIdx.x == 0 && (t & 63) == 0)
        for (int k = 0; k < 16; ++k) g_tphase[t >> 6][k] = ph[k];
#endif
}
#undef TPHASE

// slab position -> torch flat parameter index
__device__ __forceinline__ int slab_to_param(int pos) {
    if (pos < SL_WF1) {  // dW2^T tiles: tile = wave*4 + tt (kt = 2*wave + (tt>>1), ct = tt&1)
        const int lane = pos & 63, i = (pos >> 6) & 15, tile = pos >> 10;
        const int wv = tile >> 2, tt = tile & 3;
        const int k = (2 * wv + (tt >> 1)) * 32 + acc_row32(i, lane);
        const int cp = (tt & 1) * 32 + (lane & 31);
        return P_W2 + cp * 256 + k;
    }
    if (pos < SL_SMALL) {  // dWf1 tiles: jt = wave&1, m'-tile = (wave>>1)*4 + tt
        const int p2 = pos - SL_WF1;
        const int lane = p2 & 63, i = (p2 >> 6) & 15, tile = p2 >> 10;
        const int wv = tile >> 2, tt = tile & 3;
        const int j = (wv & 1) * 32 + acc_row32(i, lane);
        const int mp = ((wv >> 1) * 4 + tt) * 32 + (lane & 31);  // k' = q*64 + c'
        const int m = (mp & 63) * 4 + (mp >> 6);
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
};

// Deterministic slab reduction: a block owns 64 slab positions; its 16 waves sum the slabs
// g = wave, wave + 16, ... (<= 16 independent loads per lane, all issued at once: one memory
// round trip for the ~34 MB instead of 8), then the 16 partials are added in a fixed order.
constexpr int RW = 16;  // waves per reduction block

__global__ __launch_bounds__(64 * RW) void k_reduce_slabs(const float* slab, int nslab,
                                                          float* grad, float* loss, ReduceAdam R) {
    __shared__ float part[RW][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pos = blockIdx.x * 64 + lane;
    float r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int g = wave + RW * u;
        r[u] = (pos <= SL_LOSS && g < nslab) ? slab[(int64_t)g * SLAB + pos] : 0.f;
    }
    float v = r[0];
#pragma unroll
    for (int u = 1; u < 16; ++u) v += r[u];
    part[wave][lane] = v;
    __syncthreads();
    if (wave == 0 && pos <= SL_LOSS) {
        float s = part[0][lane];
#pragma unroll
        for (int k = 1; k < RW; ++k) s += part[k][lane];
        if (pos == SL_LOSS) {
            if (loss) *loss = s;
        } else {
            const int pi = slab_to_param(pos);
            if (grad) grad[pi] = s;
            if (R.on) {
                constexpr int off[9] = {P_W1, P_B1, P_W2, P_B2, P_WF1, P_BF1, P_WF2, P_BF2, P_TOTAL};
                int k = 0;
#pragma unroll
                for (int j = 1; j < 8; ++j) k += pi >= off[j] ? 1 : 0;
                const int e = pi - off[k];
                const unsigned long long t = *R.step;
                const g2048::AdamCoef c = g2048::adam_coef((double)t, R.lr, R.b1, R.b2, R.eps);
                float* pp = R.p[k] + e;
                const float np = g2048::adam_apply(c, s, R.m + pi, R.v + pi, *pp);
                *pp = np;
                if (R.sync_every && t % R.sync_every == 0ull) R.tp[k][e] = np;
            }
        }
    }
}

}  // namespace

extern "C" G2048_API int64_t g2048_convnet_train_workspace(int64_t batch) {
    const int64_t ntiles = (batch + S - 1) / S;
    const int64_t g = ntiles < 256 ? ntiles : 256;
    return g * SLAB;
}

static int train_launch(const g2048_convnet_params* p, const uint8_t* rows,
                        const uint8_t* actions, const int64_t* idx, const float* y, int64_t batch,
                        float* workspace, float* grad_out, float* loss_out, uint64_t* step_dev,
                        const ReduceAdam& R, void* stream) {
    TrainArgs A;
    A.w1 = p->w1;
    A.b1 = p->b1;
    A.w2 = p->w2;
    A.b2 = p->b2;
    A.wf1 = p->fc1_w;
    A.bf1 = p->fc1_b;
    A.wf2 = p->fc2_w;
    A.bf2 = p->fc2_b;
    A.rows = rows;
    A.actions = actions;
    A.idx = idx;
    A.y = y;
    A.batch = batch;
    A.slab = workspace;
    A.step = reinterpret_cast<unsigned long long*>(step_dev);
    const int64_t ntiles = (batch + S - 1) / S;
    const int grid = (int)(ntiles < 256 ? ntiles : 256);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_conv_train, dim3(grid), dim3(NT), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_conv_train: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(k_reduce_slabs, dim3((SL_LOSS + 64) / 64), dim3(64 * RW), 0, st,
                       workspace, grid, grad_out, loss_out, R);
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
    memset(&R, 0, sizeof(R));
    const g2048_convnet_params* nets[2] = {p, sync_every ? target : nullptr};
    for (int h = 0; h < 2; ++h) {
        if (!nets[h]) continue;
        const float* ps[8] = {nets[h]->w1, nets[h]->b1, nets[h]->w2, nets[h]->b2,
                              nets[h]->fc1_w, nets[h]->fc1_b, nets[h]->fc2_w, nets[h]->fc2_b};
        for (int k = 0; k < 8; ++k) (h ? R.tp : R.p)[k] = const_cast<float*>(ps[k]);
    }
    R.m = exp_avg;
    R.v = exp_avg_sq;
    R.step = reinterpret_cast<const unsigned long long*>(step_dev);
    R.lr = lr;
    R.b1 = beta1;
    R.b2 = beta2;
    R.eps = eps;
    R.sync_every = sync_every;
    R.on = 1;
    return train_launch(p, rows, actions, idx, y, batch, workspace, grad_out, loss_out, step_dev,
                        R, stream);
}
