// g2048_convnet.hpp -- device building blocks of the reference conv Q-net on gfx950 (shared by
// the forward / targets kernels in g2048_qnet.hip and the train kernels in g2048_qtrain.hip).
//
// Net (src/configs/double_dqn_conv.py:19-28): Conv2d(1,64,2) ReLU Conv2d(64,64,2) ReLU Flatten
// Linear(256,64) ReLU Linear(64,4) on the 4x4 board of log2 exponents.
//
// A tile is S = 16 boards; a workgroup is 256 threads (4 waves, one per SIMD).  conv2 runs in
// the Winograd domain F(2x2, 2x2):
//
//   Y = A^T [ sum_c (G g_oc G^T) .* (B^T d_c B) ] A,
//   B^T = [[1,-1,0],[0,1,0],[0,-1,1]]   G = [[1,0],[1,1],[0,1]]   A^T = [[1,1,0],[0,1,1]]
//
// with d_c the 3x3 relu(conv1) map of input channel c and g_oc the 2x2 kernel: nine
// [16 boards x 64 c] @ [64 c x 64 o] GEMMs per tile (36 864 MAC per board instead of 65 536).
// All transform coefficients are 0 / +-1 (measured fp32 error 1.4x that of the direct sum, both
// ~1e-7 relative).  The backward uses the transposed transforms: dM = A dY A^T (same shape as
// G g G^T), dU = sum_b V^T dM, dW2 = G^T dU G, dV = dM U^T, dh1 = B dV B^T.
//
// MFMA: v_mfma_f32_16x16x4_f32, lane (l16 = lane & 15, g = lane >> 4) supplies A[m = l16][k = g]
// and B[k = g][n = l16]; D lane holds D[m = 4g + i][n = l16], i = 0..3.  The k index of a step
// may be any permutation shared by A and B -- each GEMM below picks the one that makes its
// operands contiguous (ds_read_b128) or register-resident.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {
namespace cnet {

constexpr int NT = 256;     // threads per workgroup
constexpr int S = 16;       // boards per tile
constexpr int VS = 68;      // floats per board row of V[xi][board][c] / dM[xi][board][o]
constexpr int VXI = S * VS; // floats per Winograd point
constexpr int H2S = 260;    // h2[s][k'], k' = q*64 + o (Flatten's index c'*4 + q permuted)
constexpr int WF1S = 260;   // fc1_w[j][k']
constexpr int FS = 68;      // f[s][j] (16-byte aligned rows)
constexpr int WF2S = 68;    // wf2[a][j]

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct NetW {
    const float *w1, *b1, *w2, *b2, *wf1, *bf1, *wf2, *bf2;
};

struct Regs {       // per-thread weights held in registers
    float w1t;      // conv1 weight w1[c = 16*wave + l16][tap = g] (conv1's MFMA B operand)
    float b1o;      // conv1 bias b1[16*wave + l16]
    float u[9][16]; // Winograd-domain conv2 weights, layout chosen by the loader
};

// (G g G^T) with g = [[a, b], [c, d]] (rows kh, columns kw):
//   [[a, a+b, b], [a+c, (a+c)+(b+d), b+d], [c, c+d, d]]
__device__ __forceinline__ void winograd_u(const float4 w, float (&u)[9][16], int kk) {
    const float a = w.x, b = w.y, c = w.z, d = w.w;
    const float ac = a + c, bd = b + d;
    u[0][kk] = a;
    u[1][kk] = a + b;
    u[2][kk] = b;
    u[3][kk] = ac;
    u[4][kk] = ac + bd;
    u[5][kk] = bd;
    u[6][kk] = c;
    u[7][kk] = c + d;
    u[8][kk] = d;
}

// Forward layout: u[xi][kk] = U_xi[c = 16g + kk][o = 16*wave + l16] (conv2's B operand, k = c).
__device__ __forceinline__ void load_u_fwd(const float* w2, Regs& R) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    const float4* src = reinterpret_cast<const float4*>(w2 + (16 * wave + l16) * 256 + 64 * g);
    float4 wv[16];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) wv[kk] = src[kk];  // w2[o][c][kh][kw], 64 contiguous floats
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) winograd_u(wv[kk], R.u, kk);
}

// Transposed layout: u[xi][kk] = U_xi[c = 16*wave + l16][o = 16g + kk] (dV = dM U^T, k = o).
__device__ __forceinline__ void load_u_bwd(const float* w2, Regs& R) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    const int c = 16 * wave + l16;
    float4 wv[16];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
        wv[kk] = *reinterpret_cast<const float4*>(w2 + (16 * g + kk) * 256 + 4 * c);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) winograd_u(wv[kk], R.u, kk);
}

// conv1 operands of this lane: channel 16*wave + l16, tap g (w1[c][0][kh][kw], tap = 2kh + kw).
__device__ __forceinline__ void load_conv1(const NetW& W, Regs& R) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = 16 * wave + (lane & 15);
    R.w1t = W.w1[4 * c + (lane >> 4)];
    R.b1o = W.b1[c];
}

// fc1_w[j][k], k = c'*4 + q (torch Flatten order) -> wf1s[j][wf1_col(k' = q*64 + c')] (row
// stride WF1S).  The column swizzle (c' ^ 16q) puts the four q of one c' -- written by four
// adjacent lanes -- in different banks; it keeps every aligned group of 4 columns together, so
// the b128 reads along k' stay contiguous.
__device__ __forceinline__ int wf1_col(int kp) { return kp ^ (16 * (kp >> 6)); }

// f[64] = this thread's column t of fc1_w (loaded by the caller with the other staging loads).
__device__ __forceinline__ void store_fc1(const float (&f)[64], float* wf1s) {
    const int t = threadIdx.x;
    float* dst = wf1s + wf1_col((t & 3) * 64 + (t >> 2));
#pragma unroll
    for (int i = 0; i < 64; ++i) dst[i * WF1S] = f[i];
}

// ---- conv1 without bias as 9 MFMAs per wave (M = 16 boards, K = 4 taps, N = the wave's 16
//      channels): pre[p][i] = sum_tap x[b = 4g + i][cell(p, tap)] * w1[16*wave + l16][tap].
//      The forward (relu(pre + b1)) and the backward's relu' mask (pre + b1 > 0) both use this,
//      so they see the same float.  xs: the tile's boards as floats [S][16].
__device__ __forceinline__ void conv1_pre_mfma(const float* xs, float w1t, f32x4 (&pre)[9]) {
    const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
    const float* xr = xs + l16 * 16 + (g >> 1) * 4 + (g & 1);  // A: board l16, tap g
#pragma unroll
    for (int p = 0; p < 9; ++p)
        pre[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[(p / 3) * 4 + p % 3], w1t,
                                                      f32x4{0, 0, 0, 0}, 0, 0, 0);
}

// ---- conv1 + ReLU + input transform -> V[xi][b][c] (stride VS, point stride VXI): lane
//      (channel 16*wave + l16, boards 4g .. 4g+3) from conv1_pre_mfma's accumulators.
__device__ __forceinline__ void conv1_v(const float* xs, float* V, const Regs& R) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    f32x4 pre[9];
    conv1_pre_mfma(xs, R.w1t, pre);
    float* vdst = V + 4 * g * VS + 16 * wave + l16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float d[9];
#pragma unroll
        for (int p = 0; p < 9; ++p) d[p] = fmaxf(pre[p][i] + R.b1o, 0.f);
        float r[3][3];  // B^T d: rows (d0 - d1, d1, d2 - d1)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            r[0][j] = d[j] - d[3 + j];
            r[1][j] = d[3 + j];
            r[2][j] = d[6 + j] - d[3 + j];
        }
        float* vb = vdst + i * VS;
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // (B^T d) B: the same on columns
            vb[(3 * k + 0) * VXI] = r[k][0] - r[k][1];
            vb[(3 * k + 1) * VXI] = r[k][1];
            vb[(3 * k + 2) * VXI] = r[k][2] - r[k][1];
        }
    }
}

// ---- conv2 in the Winograd domain: M_xi[s][o] = sum_c V_xi[s][c] U_xi[c][o] (U in the forward
//      register layout; wave w = output channels 16w..16w+15; 9 x 16 MFMAs, three point chains
//      interleaved), then Y = A^T M A + b2, ReLU -> h2[s][q*64 + o].
__device__ __forceinline__ void conv2_h2(const float* V, float* h2, const float* sb2,
                                         const Regs& R) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    f32x4 acc[9];
#pragma unroll
    for (int xi = 0; xi < 9; ++xi) acc[xi] = f32x4{0, 0, 0, 0};
    const float* vsrc = V + l16 * VS + 16 * g;
#pragma unroll
    for (int grp = 0; grp < 3; ++grp) {
        f32x4 av[3][4];
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4)
                av[e][q4] = *reinterpret_cast<const f32x4*>(vsrc + (3 * grp + e) * VXI + 4 * q4);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
#pragma unroll
            for (int e = 0; e < 3; ++e)
                acc[3 * grp + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                    av[e][kk >> 2][kk & 3], R.u[3 * grp + e][kk], acc[3 * grp + e], 0, 0, 0);
    }
    // C: row 4g + i -> board 4g + i; col -> o = 16*wave + l16
    const int o = 16 * wave + l16;
    const float bo = sb2[o];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float m[9];
#pragma unroll
        for (int xi = 0; xi < 9; ++xi) m[xi] = acc[xi][i];
        const float r0a = m[0] + m[1], r0b = m[1] + m[2];
        const float r1a = m[3] + m[4], r1b = m[4] + m[5];
        const float r2a = m[6] + m[7], r2b = m[7] + m[8];
        float* hrow = h2 + (4 * g + i) * H2S + o;
        hrow[0] = fmaxf((r0a + r1a) + bo, 0.f);    // (qh, qw) = (0, 0)
        hrow[64] = fmaxf((r0b + r1b) + bo, 0.f);   // (0, 1)
        hrow[128] = fmaxf((r1a + r2a) + bo, 0.f);  // (1, 0)
        hrow[192] = fmaxf((r1b + r2b) + bo, 0.f);  // (1, 1)
    }
}

// ---- fc1 (16x16x4): [16 boards x 256] @ [256 x 64]; wave w: units 16w .. 16w+15.  Lane group
//      g covers k' in [64g, 64g+64): A (h2) and B (wf1s) read 4 steps at a time.
//      f[s][j] = relu(fc1(h2) + bf1).
__device__ __forceinline__ void fc1_f(const float* h2, const float* wf1s, const float* sbf1,
                                      float* fa) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    f32x4 c0 = f32x4{0}, c1 = f32x4{0};
    const int jc = wave * 16 + l16;
    const float* ap = h2 + l16 * H2S + 64 * g;
    const float* bp = wf1s + jc * WF1S;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 8) {
        const f32x4 av0 = *reinterpret_cast<const f32x4*>(ap + kk);
        const f32x4 av1 = *reinterpret_cast<const f32x4*>(ap + kk + 4);
        const f32x4 bv0 = *reinterpret_cast<const f32x4*>(bp + wf1_col(64 * g + kk));
        const f32x4 bv1 = *reinterpret_cast<const f32x4*>(bp + wf1_col(64 * g + kk + 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0[e], bv0[e], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1[e], bv1[e], c1, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        fa[(4 * g + i) * FS + jc] = fmaxf((c0[i] + c1[i]) + sbf1[jc], 0.f);
}

// Split-role target scratch (g2048_convnet_update), in floats from its base: a* i32[B], then
// Q_target f32[B][4] (16-byte aligned), then (r, disc) f32[B][2].
__host__ __device__ constexpr int64_t conv_split_qtg_offset(int64_t batch) {
    return (batch + 3) & ~int64_t(3);
}
__host__ __device__ constexpr int64_t conv_split_rd_offset(int64_t batch) {
    return conv_split_qtg_offset(batch) + 4 * batch;
}
__host__ __device__ constexpr int64_t conv_split_floats(int64_t batch) {
    return conv_split_rd_offset(batch) + 2 * batch;
}

// The Bellman target y = r + disc * next, disc = (1 - d) * float32(gamma), rounded after the
// product (no FMA contraction): the same float in the targets launch and the train launch.
__device__ __forceinline__ float bellman_y(float r, float disc, float next) {
#pragma clang fp contract(off)
    return r + disc * next;
}

// One board word (t < 64: word t&3 of board t>>2) -> 4 exponent floats in xs[S][16].
__device__ __forceinline__ void put_word(float* xs, int t, uint32_t v) {
    float* dst = xs + (t >> 2) * 16 + (t & 3) * 4;
    dst[0] = (float)(v & 0xFFu);
    dst[1] = (float)((v >> 8) & 0xFFu);
    dst[2] = (float)((v >> 16) & 0xFFu);
    dst[3] = (float)(v >> 24);
}

}  // namespace cnet
}  // namespace g2048
