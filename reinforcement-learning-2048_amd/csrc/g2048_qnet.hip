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

__global__ __launch_bounds__(NT) void k_conv_forward(ConvNetArgs A) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
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
    const int64_t b0 = (int64_t)blockIdx.x * S;

    // ---- stage boards (one u32 word = 4 exponents per thread: 32 boards x 4 words = 128 threads)
    if (t < S * 4) {
        const int s = t >> 2, w = t & 3;
        const int64_t b = b0 + s;
        uint32_t v = 0;
        if (b < A.n) {
            const int64_t row = A.idx ? A.idx[b] : b;
            v = reinterpret_cast<const uint32_t*>(A.rows)[row * 4 + w];
        }
        float* dst = xs + s * 16 + w * 4;
        dst[0] = (float)(v & 0xFFu);
        dst[1] = (float)((v >> 8) & 0xFFu);
        dst[2] = (float)((v >> 16) & 0xFFu);
        dst[3] = (float)(v >> 24);
    }
    // ---- stage small weights
    sw1[t] = A.w1[t];
    if (t < 64) {
        sb1[t] = A.b1[t];
        sb2[t] = A.b2[t];
        sbf1[t] = A.bf1[t];
    }
    swf2[(t >> 6) * 65 + (t & 63)] = A.wf2[t];
    if (t < 4) sbf2[t] = A.bf2[t];
    // ---- stage W2 transposed: wt[k][n] = w2[n][k], k = c*4 + kh*2 + kw (coalesced global reads)
#pragma unroll 4
    for (int i = 0; i < 64; ++i) {
        const int e = i * NT + t;  // n = e >> 8, k = e & 255
        wt[(e & 255) * WT_STRIDE + (e >> 8)] = A.w2[e];
    }
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
    for (int i = 0; i < 64; ++i) pf[i] = A.wf1[i * NT + t];
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
        const int64_t b = b0 + s;
        float v = sbf2[a];
#pragma unroll 16
        for (int j = 0; j < 64; ++j) v = fmaf(swf2[a * 65 + j], fa[s * F_STRIDE + j], v);
        if (b < A.n) A.q[b * 4 + a] = v;
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
    const unsigned grid = (unsigned)((n + S - 1) / S);
    hipLaunchKernelGGL(k_conv_forward, dim3(grid), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "convnet_forward: %s", hipGetErrorString(e));
}
