// g2048_qnet.hip -- fused forward of the reference conv Q-network on gfx950 f32 MFMA.
//
// Net (src/configs/double_dqn_conv.py:19-28): Conv2d(1,64,2) ReLU Conv2d(64,64,2) ReLU Flatten
// Linear(256,64) ReLU Linear(64,4).  Input = the board's 16 log2 exponents (log_scale(),
// src/board.py:224-231) read straight from u8 rows -- optionally gathered through replay
// indices, so sample_experiences + extract_samples_conv + forward are one launch.
//
// One workgroup (256 threads, 4 waves) = a tile of S = 32 boards; everything stays in LDS:
//   conv1  VALU: 32 x 9 positions x 64 channels, 4 MACs each               -> h1  (LDS)
//   conv2  MFMA v_mfma_f32_32x32x2_f32: [128 = 32 boards x 4 positions] x [256 = c,kh,kw]
//          @ [256 x 64]; wave w owns rows 32w..32w+31 and both 32-col tiles  -> h2  (LDS)
//   fc1    MFMA v_mfma_f32_16x16x4_f32: [32 x 256] @ [256 x 64], 2 tiles per wave -> f (LDS)
//   fc2    VALU: 32 x 4 dot products of length 64                          -> Q (HBM)
// Weight matrices are staged transposed ([k][n], row stride 65 floats: conflict-free both for
// the coalesced staging writes and the MFMA B-operand reads); fc1's weights are prefetched into
// VGPRs during the conv2 MFMA loop (one wave per SIMD leaves plenty of registers).
// Numerics: f32 in / f32 accumulate; each MFMA is an exact k-ordered fmaf chain, so results
// differ from torch's GEMMs only by summation order (tests: rtol 1e-5 vs torch fp32).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"

namespace {

constexpr int S = 32;            // boards per workgroup
constexpr int NT = 256;          // threads per workgroup
constexpr int H1_STRIDE = 65;    // floats per (board, position) row of h1
constexpr int WT_STRIDE = 65;    // floats per k row of a staged transposed weight
constexpr int H2_STRIDE = 257;   // floats per board row of h2, stored [q][c'] (k' = q*64 + c')
constexpr int F_STRIDE = 65;

// LDS carve (floats)
constexpr int OFF_X = 0;                                  // [S][16]
constexpr int OFF_SMALL = OFF_X + S * 16;                 // w1 256, b1 64, b2 64, bf1 64, wf2 4x65, bf2 4
constexpr int SMALL_FLOATS = 256 + 64 + 64 + 64 + 4 * 65 + 4;
constexpr int OFF_R1 = OFF_SMALL + ((SMALL_FLOATS + 3) & ~3);
constexpr int R1_FLOATS = S * 9 * H1_STRIDE;              // h1, later h2 + f
constexpr int OFF_R2 = OFF_R1 + ((R1_FLOATS + 3) & ~3);
constexpr int R2_FLOATS = 256 * WT_STRIDE;                // W2t, later Wf1t
constexpr int LDS_FLOATS = OFF_R2 + R2_FLOATS;
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
static_assert(S * H2_STRIDE + S * F_STRIDE <= R1_FLOATS, "h2 + f must fit in the h1 region");

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

struct NetW {
    const float *w1, *b1, *w2, *b2, *wf1, *bf1, *wf2, *bf2;
};

// Q-values of the S boards staged in lds[OFF_X] (exponents as floats) with net weights W;
// writes qs[s*4 + a] (LDS).  Caller: __syncthreads() before (xs staged) -- this function ends
// with one after qs is written.
__device__ __forceinline__ void conv_forward_tile(const NetW& W, float* lds, float* qs) {
    float* xs = lds + OFF_X;
    float* sw1 = lds + OFF_SMALL;       // [c][4]
    float* sb1 = sw1 + 256;
    float* sb2 = sb1 + 64;
    float* sbf1 = sb2 + 64;
    float* swf2 = sbf1 + 64;            // [a][j] stride 65
    float* sbf2 = swf2 + 4 * 65;
    float* h1 = lds + OFF_R1;           // [(s*9+p)][c] stride 65
    float* h2 = lds + OFF_R1;           // [s][q*64+c'] stride 257 (after conv2)
    float* fa = lds + OFF_R1 + S * H2_STRIDE;  // [s][j] stride 65
    float* wt = lds + OFF_R2;           // [k][n] stride 65

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;

    // ---- stage small weights and W2 transposed: wt[k][n] = w2[n][k], k = c*4 + kh*2 + kw
    sw1[t] = W.w1[t];
    if (t < 64) {
        sb1[t] = W.b1[t];
        sb2[t] = W.b2[t];
        sbf1[t] = W.bf1[t];
    }
    swf2[(t >> 6) * 65 + (t & 63)] = W.wf2[t];
    if (t < 4) sbf2[t] = W.bf2[t];
#pragma unroll 4
    for (int i = 0; i < 64; ++i) wt[t * WT_STRIDE + i] = W.w2[i * NT + t];
    __syncthreads();

    // ---- conv1 -> h1 (VALU).  thread: channel c = lane, boards s = wave*8 .. wave*8+7
    {
        const int c = lane;
        const float w00 = sw1[c * 4 + 0], w01 = sw1[c * 4 + 1], w10 = sw1[c * 4 + 2],
                    w11 = sw1[c * 4 + 3], bb = sb1[c];
#pragma unroll
        for (int si = 0; si < 8; ++si) {
            const int s = wave * 8 + si;
            const float* x = xs + s * 16;
#pragma unroll
            for (int p = 0; p < 9; ++p) {
                const int ph = p / 3, pw = p % 3;
                float v = bb;
                v = fmaf(w00, x[ph * 4 + pw], v);
                v = fmaf(w01, x[ph * 4 + pw + 1], v);
                v = fmaf(w10, x[(ph + 1) * 4 + pw], v);
                v = fmaf(w11, x[(ph + 1) * 4 + pw + 1], v);
                h1[(s * 9 + p) * H1_STRIDE + c] = fmaxf(v, 0.0f);
            }
        }
    }
    // prefetch fc1 weights into registers (consumed after conv2): 64 per thread
    float pf[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) pf[i] = W.wf1[i * NT + t];
    __syncthreads();

    // ---- conv2 (MFMA 32x32x2): rows r = 32*wave + (lane&31): board s = r>>2, position q = r&3
    f32x16 acc0 = {0}, acc1 = {0};
    {
        const int r = wave * 32 + (lane & 31);
        const int s = r >> 2, q = r & 3;
        const int qh = q >> 1, qw = q & 1;
        const float* h1s = h1 + s * 9 * H1_STRIDE;
        const int khalf = lane >> 5;
        const int ncol = lane & 31;
#pragma unroll 8
        for (int kk = 0; kk < 128; ++kk) {
            const int k = 2 * kk + khalf;
            const int c = k >> 2, kh = (k >> 1) & 1, kw = k & 1;
            const float a = h1s[((qh + kh) * 3 + (qw + kw)) * H1_STRIDE + c];
            const float bA = wt[k * WT_STRIDE + ncol];
            const float bB = wt[k * WT_STRIDE + 32 + ncol];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bA, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bB, acc1, 0, 0, 0);
        }
    }
    __syncthreads();  // h1 and W2t are dead from here

    // ---- conv2 epilogue: bias + ReLU -> h2[s][q*64 + c']; stage fc1 weights transposed
    {
        const int col = lane & 31;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
            const int r = wave * 32 + row;
            const int s = r >> 2, q = r & 3;
            h2[s * H2_STRIDE + q * 64 + col] = fmaxf(acc0[i] + sb2[col], 0.0f);
            h2[s * H2_STRIDE + q * 64 + col + 32] = fmaxf(acc1[i] + sb2[col + 32], 0.0f);
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            // wf1[j][m], j = i, m = t (flatten index c'*4 + q) -> row k' = q*64 + c'
            wt[((t & 3) * 64 + (t >> 2)) * WT_STRIDE + i] = pf[i];
        }
    }
    __syncthreads();

    // ---- fc1 (MFMA 16x16x4): [32 boards x 256] @ [256 x 64]; wave w: m-tile w&1, n-tiles (w>>1)*2 + {0,1}
    {
        const int mt = wave & 1;
        const int nt0 = (wave >> 1) * 2;
        f32x4 c0 = {0}, c1 = {0};
        const int arow = mt * 16 + (lane & 15);
        const int kq = lane >> 4;
        const int ncol = lane & 15;
#pragma unroll 8
        for (int kk = 0; kk < 64; ++kk) {
            const int k = 4 * kk + kq;
            const float a = h2[arow * H2_STRIDE + k];
            const float bA = wt[k * WT_STRIDE + nt0 * 16 + ncol];
            const float bB = wt[k * WT_STRIDE + (nt0 + 1) * 16 + ncol];
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bA, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bB, c1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = mt * 16 + (lane >> 4) * 4 + i;
            const int ja = nt0 * 16 + ncol, jb = (nt0 + 1) * 16 + ncol;
            fa[row * F_STRIDE + ja] = fmaxf(c0[i] + sbf1[ja], 0.0f);
            fa[row * F_STRIDE + jb] = fmaxf(c1[i] + sbf1[jb], 0.0f);
        }
    }
    __syncthreads();

    // ---- fc2 (VALU): thread t < 128 -> board s = t>>2, action a = t&3
    if (t < S * 4) {
        const int s = t >> 2, a = t & 3;
        float v = sbf2[a];
#pragma unroll 16
        for (int j = 0; j < 64; ++j) v = fmaf(swf2[a * 65 + j], fa[s * F_STRIDE + j], v);
        qs[t] = v;
    }
    __syncthreads();
}

// stage 32 boards (rows[idx[b]] or rows[b]) as float exponents into xs
__device__ __forceinline__ void stage_boards(float* xs, const uint8_t* rows, const int64_t* idx,
                                             int64_t b0, int64_t n) {
    const int t = threadIdx.x;
    if (t < S * 4) {
        const int s = t >> 2, w = t & 3;
        const int64_t b = b0 + s;
        uint32_t v = 0;
        if (b < n) {
            const int64_t row = idx ? idx[b] : b;
            v = reinterpret_cast<const uint32_t*>(rows)[row * 4 + w];
        }
        float* dst = xs + s * 16 + w * 4;
        dst[0] = (float)(v & 0xFFu);
        dst[1] = (float)((v >> 8) & 0xFFu);
        dst[2] = (float)((v >> 16) & 0xFFu);
        dst[3] = (float)(v >> 24);
    }
}

__global__ __launch_bounds__(NT) void k_conv_forward(ConvNetArgs A) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
    __shared__ float qs[S * 4];
    const int64_t b0 = (int64_t)blockIdx.x * S;
    stage_boards(lds + OFF_X, A.rows, A.idx, b0, A.n);
    __syncthreads();
    conv_forward_tile(NetW{A.w1, A.b1, A.w2, A.b2, A.wf1, A.bf1, A.wf2, A.bf2}, lds, qs);
    const int t = threadIdx.x;
    if (t < S * 4 && b0 + (t >> 2) < A.n) A.q[b0 * 4 + t] = qs[t];
}

// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
// Persistent kernels (rollout forward for large n, Double-DQN targets): a workgroup stages a
// net's W2 once (LDS) and its fc1_w once (registers: each wave keeps its 16-unit slice in 64
// VGPRs, fc1's B operand), then runs 16-board tiles.
//
// On gfx950 a VALU op between f32 MFMAs is not hidden (tools/prof_forward.hip: +4 cycles per op,
// ~12 when the ops form dependent chains), so the MFMA loops carry no VALU at all:
//  * conv1 runs as its own phase: thread (channel c = t&63, board group t>>6) reads its 4
//    boards' 64 cells at once and runs 36 independent fma chains into h1[c][board*9 + pos]
//    (channel stride 145 = 17 mod 64: conflict-free writes and reads);
//  * conv2 is split by ROWS: wave w owns boards 4w..4w+3 (16 rows (s, q)) x all 64 channels as
//    four 16x16x4 tiles.  Lane group g = lane>>4 is the tap (kh, kw) = (g>>1, g&1) and step c is
//    the input channel, so k = 4c + g is conv2's flat weight index.  Per step: one ds_read_b32
//    of h1 (A, shared by the four tiles) + one ds_read_b128 of W2 (B) -> 4 MFMAs;
//  * fc1: A = h2 read along k as ds_read_b128, B = the wave's fc1_w slice in registers;
//  * fc2 uses all 256 threads and leaves Q[16][4] in LDS.
namespace persist {
constexpr int S = 16;
constexpr int TMAX = 8;   // tiles per workgroup in the targets kernel
constexpr int H1S = 145;  // floats per channel of h1: [c][board*9 + pos], 16*9 = 144 used
constexpr int H2S = 260;  // h2[s][k'], k' = q*64 + n (fc1's input index permuted)
constexpr int FS = 68;    // fa[s][j] (16-byte aligned rows for fc2's b128 reads)
constexpr int WF2S = 68;  // swf2[a][j]
constexpr int OFF_X = 0;                          // [TMAX][S][16] boards (exponents as floats)
constexpr int OFF_B2 = OFF_X + TMAX * S * 16;     // 64
constexpr int OFF_BF1 = OFF_B2 + 64;              // 64
constexpr int OFF_WF2 = OFF_BF1 + 64;             // [4][WF2S]
constexpr int OFF_BF2 = OFF_WF2 + 4 * WF2S;       // 4
constexpr int OFF_W2 = OFF_BF2 + 4;               // W2s[k][16 x 4] swizzled, see w2s_index
constexpr int OFF_H1 = OFF_W2 + 256 * 64;         // also the fc1_w staging area (32 x 260)
constexpr int OFF_H2 = (OFF_H1 + 64 * H1S + 3) & ~3;
constexpr int OFF_F = OFF_H2 + S * H2S;
constexpr int OFF_Q = OFF_F + S * FS;             // [TMAX + 1][S][4] Q of a tile
constexpr int FLOATS = OFF_Q + (TMAX + 1) * S * 4;
static_assert(OFF_W2 % 4 == 0 && OFF_H2 % 4 == 0 && OFF_F % 4 == 0 && OFF_WF2 % 4 == 0 &&
                  OFF_Q % 4 == 0,
              "b128 alignment");
static_assert(64 * H1S >= 32 * 260, "fc1_w staging must fit in the h1 area");
static_assert(FLOATS * 4 <= 160 * 1024, "LDS budget (persistent kernels)");
// W2s row k holds w2[16nt + j][k] at 4*(j ^ (k & 15)) + nt: a lane group reads 16 distinct
// 16-byte slots of one row (conflict-free b128) and the staging writes spread over 16 banks.
__device__ __forceinline__ int w2s_index(int k, int j, int nt) {
    return k * 64 + 4 * (j ^ (k & 15)) + nt;
}

struct Regs {  // per-thread weights held in registers
    float4 w1c;    // conv1 weights of channel t & 63
    float b1c;
    float wf[64];  // fc1_w[16*wave + l16][kk*4 + g]  (k' = 64g + kk <-> orig kk*4 + g)
};

// Stage net W: W2 + small tensors into LDS, conv1 channel + fc1_w slice into registers.  All
// global loads (W2 and both fc1_w halves) are issued before the first LDS store: one memory
// round trip.  Starts and ends with __syncthreads().
__device__ __forceinline__ void stage(const NetW& W, float* lds, Regs& R) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g = lane >> 4, l16 = lane & 15;
    float v2[64], f[2][32];
#pragma unroll
    for (int i = 0; i < 64; ++i) v2[i] = W.w2[i * NT + t];  // w2[n = i][k = t]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 32; ++i) f[h][i] = W.wf1[(32 * h + i) * NT + t];
    const int cc = t & 63;
    R.w1c = make_float4(W.w1[4 * cc], W.w1[4 * cc + 1], W.w1[4 * cc + 2], W.w1[4 * cc + 3]);
    R.b1c = W.b1[cc];
    const float b2 = t < 64 ? W.b2[t] : 0.f, bf1 = t < 64 ? W.bf1[t] : 0.f;
    const float wf2 = W.wf2[t], bf2 = t < 4 ? W.bf2[t] : 0.f;
    __syncthreads();  // previous users of W2s / the h1 area are done
    float* w2s = lds + OFF_W2;
#pragma unroll
    for (int i = 0; i < 64; ++i) w2s[w2s_index(t, i & 15, i >> 4)] = v2[i];
    if (t < 64) {
        lds[OFF_B2 + t] = b2;
        lds[OFF_BF1 + t] = bf1;
    }
    lds[OFF_WF2 + (t >> 6) * WF2S + (t & 63)] = wf2;
    if (t < 4) lds[OFF_BF2 + t] = bf2;
    // fc1_w through the h1 area in two halves of 32 rows (row stride 260 = 4 mod 64, so the
    // stride-4 register gather is conflict-free)
    float* st = lds + OFF_H1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 32; ++i) st[i * 260 + t] = f[h][i];
        __syncthreads();
        if ((wave >> 1) == h) {
            const float* src = st + (16 * (wave & 1) + l16) * 260 + g;
#pragma unroll
            for (int kk = 0; kk < 64; ++kk) R.wf[kk] = src[4 * kk];
        }
        __syncthreads();
    }
}

// Q[16][4] of the 16 boards in xs (exponents as floats, visible to all threads) -> qs (LDS).
// Ends with __syncthreads() (qs visible; h1 / h2 / fa free for the next tile).
__device__ __forceinline__ void tile(const float* xs, float* lds, const Regs& R, float* qs) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g = lane >> 4, l16 = lane & 15;
    const float* w2s = lds + OFF_W2;
    float* h1 = lds + OFF_H1;
    float* h2 = lds + OFF_H2;
    float* fa = lds + OFF_F;
    // ---- conv1 -> h1: channel cc at the 9 positions of boards 4*wave .. 4*wave+3: the 64
    //      input cells are read at once (one LDS round trip), then 36 independent fma chains
    {
        const int cc = t & 63;
        float x[4][16];
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 v = *reinterpret_cast<const float4*>(xs + (4 * wave + bb) * 16 + 4 * r);
                x[bb][4 * r] = v.x;
                x[bb][4 * r + 1] = v.y;
                x[bb][4 * r + 2] = v.z;
                x[bb][4 * r + 3] = v.w;
            }
        const float wt[4] = {R.w1c.x, R.w1c.y, R.w1c.z, R.w1c.w};
        float v[4][9];
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int p = 0; p < 9; ++p) v[bb][p] = R.b1c;
#pragma unroll
        for (int tap = 0; tap < 4; ++tap)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                for (int p = 0; p < 9; ++p) {
                    const int pr = p / 3 + (tap >> 1), pc = p % 3 + (tap & 1);
                    v[bb][p] = fmaf(wt[tap], x[bb][pr * 4 + pc], v[bb][p]);
                }
        float* dst = h1 + cc * H1S + 4 * wave * 9;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int p = 0; p < 9; ++p) dst[bb * 9 + p] = fmaxf(v[bb][p], 0.f);
    }
    __syncthreads();
    // ---- conv2: 64 steps x (A from h1, B from W2s) -> 4 MFMAs, chunks of 8 steps with the next
    //      chunk's LDS reads in flight
    {
        const int s_r = 4 * wave + (l16 >> 2), q_r = l16 & 3;
        const int pos_r = ((q_r >> 1) + (g >> 1)) * 3 + (q_r & 1) + (g & 1);
        const float* abase = h1 + s_r * 9 + pos_r;
        f32x4 acc[4] = {f32x4{0}, f32x4{0}, f32x4{0}, f32x4{0}};
        float av[2][8];
        f32x4 bv[2][8];
        auto load = [&](int chunk, int buf) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = chunk * 8 + j;
                av[buf][j] = abase[c * H1S];
                bv[buf][j] = *reinterpret_cast<const f32x4*>(w2s + w2s_index(4 * c + g, l16, 0));
            }
        };
        load(0, 0);
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
            const int cur = ch & 1;
            if (ch < 7) load(ch + 1, cur ^ 1);
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[cur][j], bv[cur][j][nt],
                                                                   acc[nt], 0, 0, 0);
        }
        // C: row 4g + i of the wave's 16 -> board 4*wave + g, q = i; col n = 16nt + l16
        const float* sb2 = lds + OFF_B2;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int n = 16 * nt + l16;
            const float bn = sb2[n];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                h2[(4 * wave + g) * H2S + i * 64 + n] = fmaxf(acc[nt][i] + bn, 0.f);
        }
    }
    __syncthreads();
    // ---- fc1 (16x16x4): [16 boards x 256] @ [256 x 64]; wave w: units 16w .. 16w+15.
    //      Lane group g covers k' in [64g, 64g+64): A read 4 steps at a time, B in registers.
    {
        f32x4 c0 = f32x4{0}, c1 = f32x4{0};
        const int jc = wave * 16 + l16;
        const float* ap = h2 + l16 * H2S + 64 * g;
#pragma unroll
        for (int kk = 0; kk < 64; kk += 8) {
            const f32x4 av0 = *reinterpret_cast<const f32x4*>(ap + kk);
            const f32x4 av1 = *reinterpret_cast<const f32x4*>(ap + kk + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0[e], R.wf[kk + e], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1[e], R.wf[kk + 4 + e], c1, 0, 0, 0);
            }
        }
        const float* sbf1 = lds + OFF_BF1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            fa[(4 * g + i) * FS + jc] = fmaxf((c0[i] + c1[i]) + sbf1[jc], 0.f);
    }
    __syncthreads();
    // ---- fc2: output o = t >> 2 (board o >> 2, action o & 3), part p = t & 3 sums 16 units
    {
        const int o = t >> 2, p = t & 3, s = o >> 2, a = o & 3;
        const f32x4* fr = reinterpret_cast<const f32x4*>(fa + s * FS + 16 * p);
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
    __syncthreads();
}

// One board word (t < 64: word t&3 of board t>>2) -> 4 exponent floats in xs.
__device__ __forceinline__ void put_word(float* xs, int t, uint32_t v) {
    float* dst = xs + (t >> 2) * 16 + (t & 3) * 4;
    dst[0] = (float)(v & 0xFFu);
    dst[1] = (float)((v >> 8) & 0xFFu);
    dst[2] = (float)((v >> 16) & 0xFFu);
    dst[3] = (float)(v >> 24);
}
}  // namespace persist

// The rollout's Q over all n boards (g2048_convnet_forward for n >= 16k): 256 workgroups stage
// the net once and loop over 16-board tiles; the next tile's boards are loaded during the
// current one.
__global__ __launch_bounds__(NT) void k_conv_forward_persist(ConvNetArgs A) {
    namespace P = persist;
    __shared__ __attribute__((aligned(16))) float lds[P::FLOATS];
    const int t = threadIdx.x;
    const NetW W{A.w1, A.b1, A.w2, A.b2, A.wf1, A.bf1, A.wf2, A.bf2};
    P::Regs R;
    const int64_t ntiles = (A.n + P::S - 1) / P::S;
    auto load_word = [&](int64_t tile) -> uint32_t {
        const int64_t b = tile * P::S + (t >> 2);
        if (t >= P::S * 4 || tile >= ntiles || b >= A.n) return 0u;
        return reinterpret_cast<const uint32_t*>(A.rows)[(A.idx ? A.idx[b] : b) * 4 + (t & 3)];
    };
    uint32_t next_word = load_word(blockIdx.x);
    P::stage(W, lds, R);
    float* xs = lds + P::OFF_X;
    float* qs = lds + P::OFF_Q;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b0 = tile * P::S;
        if (t < P::S * 4) P::put_word(xs, t, next_word);
        __syncthreads();
        next_word = load_word(tile + gridDim.x);  // in flight during this tile
        P::tile(xs, lds, R, qs);
        if (t < P::S * 4 && b0 + (t >> 2) < A.n) A.q[b0 * 4 + t] = qs[t];
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
};

// Each workgroup owns up to TMAX 16-sample tiles (tile = blockIdx.x + k*gridDim.x): it draws
// their indices and loads their s' rows once, runs them through the online net (Q kept in
// LDS), stages the target net and runs them again, then writes y.
__global__ __launch_bounds__(NT) void k_conv_targets_persist(TargetArgs A) {
    namespace P = persist;
    __shared__ __attribute__((aligned(16))) float lds[P::FLOATS];
    __shared__ int64_t sidx[P::TMAX * P::S];
    const int t = threadIdx.x;
    const int64_t ntiles = (A.batch + P::S - 1) / P::S;
    int T = 0;
    for (int64_t tl = blockIdx.x; tl < ntiles && T < P::TMAX; tl += gridDim.x) ++T;
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
            const int64_t b = (blockIdx.x + (int64_t)k * gridDim.x) * P::S + s;
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
                if ((t & 3) == 0) A.idx_out[b] = j;
            }
            if ((t & 3) == 0) {
                sidx[k * P::S + s] = j;
                rv[k] = A.r[j];
                dv[k] = A.d[j];
            }
            w[k] = reinterpret_cast<const uint32_t*>(A.s2)[j * 4 + (t & 3)];
        }
#pragma unroll
        for (int k = 0; k < P::TMAX; ++k)
            if (k < T) P::put_word(lds + P::OFF_X + k * P::S * 16, t, w[k]);
    }
    P::Regs R;
    float* qon = lds + P::OFF_Q;               // [TMAX][16][4]
    float* qtg = qon + P::TMAX * P::S * 4;     // [16][4]
    P::stage(A.on, lds, R);  // (starts with __syncthreads: the s' boards are visible)
    for (int k = 0; k < T; ++k)
        P::tile(lds + P::OFF_X + k * P::S * 16, lds, R, qon + k * P::S * 4);
    P::stage(A.tg, lds, R);
    for (int k = 0; k < T; ++k) {
        P::tile(lds + P::OFF_X + k * P::S * 16, lds, R, qtg);
        const int sm = t >> 2;  // sample of this thread (t < 64, t & 3 == 0)
        const int64_t b = (blockIdx.x + (int64_t)k * gridDim.x) * P::S + sm;
        if (t < P::S * 4 && (t & 3) == 0 && b < A.batch) {
#pragma clang fp contract(off)
            const float* qo = qon + (k * P::S + sm) * 4;
            const float* qt = qtg + sm * 4;
            float next;
            if (A.double_dqn) {
                int a = 0;
                float best = qo[0];
                for (int e = 1; e < 4; ++e)
                    if (qo[e] > best) { best = qo[e]; a = e; }
                next = qt[a];
            } else {
                next = fmaxf(fmaxf(qt[0], qt[1]), fmaxf(qt[2], qt[3]));
            }
            const float disc = (float)(1 - (int)dv[k]) * A.gamma;
            A.y[b] = (float)rv[k] + disc * next;
        }
        // qtg is rewritten by the next tile only after that tile's internal barriers
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
    if (tiles16 >= 4 * 256) {  // >= 4 tiles per CU: stage weights once per workgroup
        hipLaunchKernelGGL(k_conv_forward_persist, dim3(256), dim3(NT), 0, st, A);
    } else {
        const unsigned grid = (unsigned)((n + S - 1) / S);
        hipLaunchKernelGGL(k_conv_forward, dim3(grid), dim3(NT), 0, st, A);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_forward: %s", hipGetErrorString(e));
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
    const int64_t ntiles = (batch + persist::S - 1) / persist::S;
    int64_t grid = ntiles < 256 ? ntiles : 256;
    if (grid * persist::TMAX < ntiles) grid = (ntiles + persist::TMAX - 1) / persist::TMAX;
    hipLaunchKernelGGL(k_conv_targets_persist, dim3((unsigned)grid), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_targets: %s", hipGetErrorString(e));
}
