// g2048_mlp.hip -- fused Double-DQN kernels for the dense 16 -> 64 -> 4 Q-network
// (BASELINE.json configs[2]; the reference's dense family, src/configs/double_dqn_dense.py:7-15,
// at width 64).  At 1 280 MACs per board this net is pure launch overhead in torch (~50 small
// kernels per update); here an update is targets + gradient + reduce + Adam = 4 launches.
//
// Tile = 64 boards per 256-thread workgroup, VALU (every output element owned by ONE thread, so
// all sums run in a fixed order -> bit-reproducible):
//   h[s][j] = relu(b1[j] + W1[j] . x[s])      thread (j = t&63, boards 16*(t>>6) ..)
//   Q[s][a] = b2[a] + W2[a] . h[s]            thread (s = t>>2, a = t&3)
//   backward: dW2 / db2 (thread (a, j)), dh in place over h, dW1 (thread (j, 4 inputs)), db1;
// gradient accumulators persist in registers across the tiles a workgroup owns and are written
// once per workgroup in torch's parameter order; a deterministic reduction sums the slabs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"

namespace {

constexpr int NT = 256, H = 64;
// rows of x / h / W2 are float4-aligned (b128 LDS reads); W1 rows odd-strided (b32, per-lane j)
constexpr int XS = 20, W1S = 17, HS = 68, W2S = 68;
constexpr int S_FWD = 64;  // boards per tile: forward / targets / train_grad launches
constexpr int S_UPD = 32;  // the fused update (batch 8192 -> 256 tiles = one per CU)
// torch order: 0.weight [64][16], 0.bias [64], 2.weight [4][64], 2.bias [4]
constexpr int P_W1 = 0, P_B1 = 1024, P_W2 = 1088, P_B2 = 1344, P_N = 1348;
constexpr int SLAB = 1352;  // params + loss, padded
constexpr int MAX_SLABS = 256;

struct MlpW {
    const float *w1, *b1, *w2, *b2;
};

struct alignas(16) LW {  // one net's weights in LDS
    float w1[H * W1S];
    float b1[H];
    float w2[4 * W2S];
    float b2[4];
};

template <int S>
struct alignas(16) Tile {  // one tile of S boards
    float x[S * XS];
    float h[S * HS];
    float q[S * 4];
    float a[S], y[S], g[S];
};

__device__ __forceinline__ void stage_weights(const MlpW& W, LW& L) {
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * NT + t;  // w1[j][i], j = e >> 4, i = e & 15
        L.w1[(e >> 4) * W1S + (e & 15)] = W.w1[e];
    }
    if (t < H) L.b1[t] = W.b1[t];
    L.w2[(t >> 6) * W2S + (t & 63)] = W.w2[t];
    if (t < 4) L.b2[t] = W.b2[t];
}

// one u32 board word (4 exponents) -> 4 floats of an x row
__device__ __forceinline__ void put_word(float* dst, uint32_t v) {
    *reinterpret_cast<float4*>(dst) = make_float4((float)(v & 0xFFu), (float)((v >> 8) & 0xFFu),
                                                  (float)((v >> 16) & 0xFFu), (float)(v >> 24));
}

template <int S>
__device__ __forceinline__ void stage_boards(Tile<S>& T, const uint8_t* rows, const int64_t* idx,
                                             int64_t b0, int64_t n) {
    const int t = threadIdx.x;  // S boards x 4 words
    if (t >= 4 * S) return;
    const int s = t >> 2, w = t & 3;
    const int64_t b = b0 + s;
    uint32_t v = 0;
    if (b < n) v = reinterpret_cast<const uint32_t*>(rows)[(idx ? idx[b] : b) * 4 + w];
    put_word(T.x + s * XS + w * 4, v);
}

// Q = h W2^T + b2 over the tile (h post-ReLU in LDS, visible); ends with a sync.
template <int S>
__device__ __forceinline__ void layer2_tile(Tile<S>& T, const LW& W) {
    const int t = threadIdx.x;
    if (t < 4 * S) {
        const int s = t >> 2, a = t & 3;
        const float4* hr = reinterpret_cast<const float4*>(T.h + s * HS);
        const float4* wr = reinterpret_cast<const float4*>(W.w2 + a * W2S);
        float e = W.b2[a], o = 0.f;  // even / odd j, same order as k_step_dense64
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float4 hv = hr[u], wv = wr[u];
            e = fmaf(wv.x, hv.x, e);
            o = fmaf(wv.y, hv.y, o);
            e = fmaf(wv.z, hv.z, e);
            o = fmaf(wv.w, hv.w, o);
        }
        T.q[t] = e + o;
    }
    __syncthreads();
}

// weights + boards staged (caller syncs); leaves h (post-ReLU) and q in LDS, ends with a sync.
// VALU, in the float order of the fused step kernel (the rollout forward).
template <int S>
__device__ __forceinline__ void forward_tile(Tile<S>& T, const LW& W) {
    const int t = threadIdx.x;
    {
        constexpr int SPT = S / 4;  // boards per thread
        const int j = t & 63, s0 = (t >> 6) * SPT;
        float w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = W.w1[j * W1S + i];
        const float bb = W.b1[j];
        // h = (p0 + p1) + (p2 + p3), p_r summing i = r (mod 4) with the bias in p0: the order
        // of the packed (v_pk_fma_f32) Q evaluation inside the fused step kernel (g2048.hip
        // k_step_dense64), so the two agree bit for bit
#pragma unroll 4
        for (int ss = 0; ss < SPT; ++ss) {
            const int s = s0 + ss;
            const float4* xr = reinterpret_cast<const float4*>(T.x + s * XS);  // broadcast
            float p[4] = {bb, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4 xv = xr[u];
                p[0] = fmaf(w[4 * u + 0], xv.x, p[0]);
                p[1] = fmaf(w[4 * u + 1], xv.y, p[1]);
                p[2] = fmaf(w[4 * u + 2], xv.z, p[2]);
                p[3] = fmaf(w[4 * u + 3], xv.w, p[3]);
            }
            T.h[s * HS + j] = fmaxf((p[0] + p[1]) + (p[2] + p[3]), 0.f);
        }
    }
    __syncthreads();
    layer2_tile<S>(T, W);
}

// ---- MFMA form of layer 1 for the learner kernels (targets, gradient).  v_mfma_f32_16x16x4_f32:
// lane (l16 = lane & 15, g = lane >> 4) supplies A[m = l16][k = g] and B[k = g][n = l16]; D lane
// holds D[m = 4g + i][n = l16].  Wave w owns hidden units 16w .. 16w+15; the K index of step u is
// input 4g + u, so a lane's A (its board's inputs) and B (its unit's weights) are float4s.
typedef float f32x4m __attribute__((ext_vector_type(4)));

// this lane's layer-1 weights W1[16w + l16][4g .. 4g+3] (registers, from global)
__device__ __forceinline__ float4 w1_lane(const MlpW& W) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    return reinterpret_cast<const float4*>(W.w1)[(16 * wave + (lane & 15)) * 4 + (lane >> 4)];
}

// h = relu(x W1^T + b1) on MFMA, then layer 2 as forward_tile.  Ends with a sync.
template <int S>
__device__ __forceinline__ void forward_tile_mfma(Tile<S>& T, const LW& W, float4 w1v) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    const int j = 16 * wave + l16;
    const float bj = W.b1[j];
#pragma unroll
    for (int mb = 0; mb < S / 16; ++mb) {
        const float4 xv = *reinterpret_cast<const float4*>(T.x + (16 * mb + l16) * XS + 4 * g);
        f32x4m acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, w1v.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, w1v.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.z, w1v.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.w, w1v.w, acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) T.h[(16 * mb + 4 * g + i) * HS + j] = fmaxf(acc[i] + bj, 0.f);
    }
    __syncthreads();
    layer2_tile<S>(T, W);
}

// Double-DQN target of board t of the tile (src/dqn_lib.py:125-132): qo = Q_online(s'),
// qt = Q_target(s') rows of this board
__device__ __forceinline__ float bellman(const float* qo, const float* qt, int32_t r, uint8_t d,
                                         float gamma, int double_dqn) {
#pragma clang fp contract(off)
    float next;
    if (double_dqn) {
        next = qt[g2048::argmax4_torch(qo[0], qo[1], qo[2], qo[3])];  // torch.argmax: NaN first
    } else {
        next = g2048::qmax4_torch(qt[0], qt[1], qt[2], qt[3]);          // torch.max: NaN wins
    }
    const float disc = (float)(1 - (int)d) * gamma;
    return (float)r + disc * next;
}

// uniform ring index of minibatch row b, the draw of k_sample (domain 3)
__device__ __forceinline__ int64_t sample_row(int64_t b, unsigned long long ep,
                                              unsigned long long count, uint32_t lo, uint32_t hi) {
    const uint4 u = g2048::philox10(
        make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32), (uint32_t)ep,
                   (uint32_t)(ep >> 32) | (g2048::DOMAIN_SAMPLE << 30)),
        lo, hi);
    return (int64_t)__umul64hi(((unsigned long long)u.y << 32) | u.x, count);
}

struct GradAcc {  // per-thread gradient accumulators, persistent across a workgroup's tiles
    f32x4m w1a = {0.f, 0.f, 0.f, 0.f};  // dW1[16w + 4g + i][l16], even / odd K-steps
    f32x4m w1b = {0.f, 0.f, 0.f, 0.f};
    float b1 = 0.f, w2 = 0.f, b2 = 0.f, loss = 0.f;
};

// forward + MSE + backward of one staged tile (x, a, y and the validity mask g in LDS, synced)
template <int S>
__device__ __forceinline__ void grad_tile(Tile<S>& T, const LW& W, float4 w1v, GradAcc& G) {
    const int t = threadIdx.x;
    forward_tile_mfma<S>(T, W, w1v);
    if (t < S) {  // loss and dq = 2 (q - y) at the taken action
        const float d = (T.q[t * 4 + (int)T.a[t]] - T.y[t]) * T.g[t];
        G.loss = fmaf(d, d, G.loss);
        T.g[t] = 2.f * d;
    }
    __syncthreads();
    {  // dW2[a][j] / db2[a]: thread (a = t>>6, j = t&63)
        const int a = t >> 6, j = t & 63;
        float gw = 0.f, gb = 0.f;
#pragma unroll 8
        for (int s = 0; s < S; ++s) {
            const float g = (int)T.a[s] == a ? T.g[s] : 0.f;
            gw = fmaf(g, T.h[s * HS + j], gw);
            gb += g;
        }
        G.w2 += gw;
        if (j == 0) G.b2 += gb;
    }
    __syncthreads();
    {  // dh = dq * W2[a] * relu'(h), in place
        constexpr int SPT = S / 4;
        const int j = t & 63, s0 = (t >> 6) * SPT;
#pragma unroll 4
        for (int ss = 0; ss < SPT; ++ss) {
            const int s = s0 + ss;
            const float hv = T.h[s * HS + j];
            T.h[s * HS + j] = hv > 0.f ? T.g[s] * W.w2[(int)T.a[s] * W2S + j] : 0.f;
        }
    }
    __syncthreads();
    {  // dW1 += dh^T x on MFMA (m = unit, n = input, k = board: 4 boards per step, two chains);
       // db1 by threads j < 64
        const int lane = t & 63, wave = t >> 6, g = lane >> 4, l16 = lane & 15;
        const float* hc = T.h + 16 * wave + l16;
        const float* xc = T.x + l16;
#pragma unroll
        for (int st = 0; st < S / 4; st += 2) {
            G.w1a = __builtin_amdgcn_mfma_f32_16x16x4f32(hc[(4 * st + g) * HS], xc[(4 * st + g) * XS],
                                                         G.w1a, 0, 0, 0);
            G.w1b = __builtin_amdgcn_mfma_f32_16x16x4f32(hc[(4 * st + 4 + g) * HS],
                                                         xc[(4 * st + 4 + g) * XS], G.w1b, 0, 0, 0);
        }
        if (t < H) {
            float v = 0.f;
#pragma unroll 8
            for (int s = 0; s < S; ++s) v += T.h[s * HS + t];
            G.b1 += v;
        }
    }
}

// A slab element: a plain store, or (COH) a device-scope store -- the sc1 cache policy (the bits
// the compiler gives an agent-scope atomic store on gfx950) writes it through the XCD's L2 to the
// coherent level, so a workgroup of the same launch on another XCD can read it (with sc1 loads)
// without an L2 write-back or invalidate (k_mlp_update1).  Buffer forms, not atomics: relaxed
// atomic loads are each followed by a vmcnt(0) wait, which would serialise the reduction's loads.
constexpr int AUX_SC1 = 16;  // gfx950 buffer cache-policy word: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const float* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
// slab: the workgroup's slab (wave-uniform, so the resource is built in SGPRs once; a per-lane
// base would need a waterfall loop over the lanes' resources); e: the element
template <bool COH>
__device__ __forceinline__ void slab_put(float* slab, int e, float v) {
    if constexpr (COH)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), slab_rsrc(slab),
                                              (uint32_t)e * 4u, 0u, AUX_SC1);
    else
        slab[e] = v;
}

// the workgroup's gradient slab in torch parameter order + its loss (scratch: S*4 >= 64 floats)
template <int S, bool COH = false>
__device__ __forceinline__ void write_slab(const GradAcc& G, Tile<S>& T, float* slab) {
    const int t = threadIdx.x;
    {  // dW1[16w + 4g + i][l16]
        const int lane = t & 63, wave = t >> 6, g = lane >> 4, l16 = lane & 15;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            slab_put<COH>(slab, P_W1 + (16 * wave + 4 * g + i) * 16 + l16, G.w1a[i] + G.w1b[i]);
    }
    if (t < H) slab_put<COH>(slab, P_B1 + t, G.b1);
    slab_put<COH>(slab, P_W2 + t, G.w2);  // t = a*64 + j
    if ((t & 63) == 0) slab_put<COH>(slab, P_B2 + (t >> 6), G.b2);
    __syncthreads();
    if (t < S) T.q[t] = G.loss;  // threads >= S hold 0
    __syncthreads();
    if (t == 0) {
        float v = 0.f;
        for (int i = 0; i < S; ++i) v += T.q[i];
        slab_put<COH>(slab, P_N, v);
    }
}

struct FwdArgs {
    MlpW W;
    const uint8_t* rows;
    const int64_t* idx;
    int64_t n;
    float* q;
};

__global__ __launch_bounds__(NT) void k_mlp_forward(FwdArgs A) {
    constexpr int S = S_FWD;
    __shared__ LW W;
    __shared__ Tile<S> T;
    const int64_t b0 = (int64_t)blockIdx.x * S;
    stage_weights(A.W, W);
    stage_boards<S>(T, A.rows, A.idx, b0, A.n);
    __syncthreads();
    forward_tile<S>(T, W);
    const int t = threadIdx.x;
    if (b0 + (t >> 2) < A.n) A.q[b0 * 4 + t] = T.q[t];
}

struct TargetArgs {
    MlpW on, tg;
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

__global__ __launch_bounds__(NT) void k_mlp_targets(TargetArgs A) {
    constexpr int S = S_FWD;
    __shared__ LW W;
    __shared__ Tile<S> T;
    __shared__ float qon[S * 4];
    __shared__ int64_t sidx[S];
    const int t = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * S;
    if (t < S) {
        const int64_t b = b0 + t;
        int64_t j = 0;
        if (b < A.batch) {
            j = A.idx_in ? A.idx_in[b] : sample_row(b, *A.epoch, *A.count, A.seed_lo, A.seed_hi);
            A.idx_out[b] = j;
        }
        sidx[t] = j;
    }
    const float4 w1on = w1_lane(A.on), w1tg = w1_lane(A.tg);
    stage_weights(A.on, W);
    __syncthreads();
    stage_boards<S>(T, A.s2, sidx, 0, S);
    __syncthreads();
    forward_tile_mfma<S>(T, W, w1on);
    qon[t] = T.q[t];
    stage_weights(A.tg, W);  // forward_tile ended with a sync: the online weights are dead
    __syncthreads();
    forward_tile_mfma<S>(T, W, w1tg);
    if (t < S && b0 + t < A.batch) {
        const int64_t j = sidx[t];
        A.y[b0 + t] = bellman(qon + t * 4, T.q + t * 4, A.r[j], A.d[j], A.gamma, A.double_dqn);
    }
}

struct TrainArgs {
    MlpW W;
    const uint8_t* rows;
    const uint8_t* actions;
    const int64_t* idx;
    const float* y;
    int64_t batch;
    float* slab;
    unsigned long long* step;
};

__global__ __launch_bounds__(NT) void k_mlp_train(TrainArgs A) {
    constexpr int S = S_FWD;
    __shared__ LW W;
    __shared__ Tile<S> T;
    const int t = threadIdx.x;
    if (A.step && blockIdx.x == 0 && t == 0) *A.step += 1ull;
    stage_weights(A.W, W);
    const float4 w1v = w1_lane(A.W);
    GradAcc G;
    const int64_t ntiles = (A.batch + S - 1) / S;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b0 = tile * S;
        __syncthreads();
        stage_boards<S>(T, A.rows, A.idx, b0, A.batch);
        if (t < S) {
            const int64_t b = b0 + t;
            const bool ok = b < A.batch;
            T.a[t] = ok ? (float)A.actions[A.idx[b]] : 0.f;
            T.y[t] = ok ? A.y[b] : 0.f;
            T.g[t] = ok ? 1.f : 0.f;
        }
        __syncthreads();
        grad_tile<S>(T, W, w1v, G);
    }
    write_slab<S>(G, T, A.slab + (int64_t)blockIdx.x * SLAB);
}

// The whole graded + target half of train_step in one launch (src/dqn_lib.py:116-161): per tile
// of S_UPD minibatch rows, draw the ring rows, Q_target(s') and Q_online(s') -> y, then
// Q_online(s) -> MSE -> gradient slab.  Both nets' weights are staged once per workgroup.
// *step is the sampler epoch (read only here); block 0 publishes *step + 1 in *step_next, which
// the reduction commits to *step (Adam's t) -- no block reads a value another block writes.
struct UpdateArgs {
    MlpW on, tg;
    const uint8_t *s, *a, *s2, *d;
    const int32_t* r;
    const unsigned long long* count;
    const unsigned long long* step;
    const int64_t* idx_in;
    int64_t batch;
    uint32_t seed_lo, seed_hi;
    float gamma;
    int double_dqn;
    int64_t* idx_out;
    float* y_out;
    float* slab;
    unsigned long long* step_next;
#ifdef G2048_MLP_PHASE
    long long* phase;
#endif
};

#ifdef G2048_MLP_PHASE
#define MPHASE(k) \
    if (threadIdx.x == 0) A.phase[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define MPHASE(k)
#endif

// the update's per-workgroup work (k_mlp_update, and the first half of k_mlp_update1): every
// tile of the workgroup, then its gradient slab (COH: written through to the coherent level)
template <bool COH>
__device__ __forceinline__ void update_tiles(const UpdateArgs& A) {
    constexpr int S = S_UPD;
    MPHASE(0);
    __shared__ LW Won, Wtg;
    __shared__ Tile<S> T;
    __shared__ float qtg[S * 4];
    const int t = threadIdx.x;
    const unsigned long long ep = A.idx_in ? 0ull : *A.step;
    const unsigned long long count = A.idx_in ? 0ull : *A.count;
    if (blockIdx.x == 0 && t == 0) *A.step_next = *A.step + 1ull;
    stage_weights(A.on, Won);
    stage_weights(A.tg, Wtg);
    const float4 w1on = w1_lane(A.on), w1tg = w1_lane(A.tg);
    GradAcc G;
    const int64_t ntiles = (A.batch + S - 1) / S;
    const int sl = t >> 2, w = t & 3;  // threads t < 4S: board sl of the tile, word w
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b0 = tile * S;
        // every thread of a board draws its row itself and fetches its s' and s words in the
        // same round trip as a / r / d (no LDS hand-off of the indices)
        const int64_t b = b0 + sl;
        const bool ok = t < 4 * S && b < A.batch;
        uint32_t s2w = 0, sw = 0;
        int32_t rj = 0;
        uint8_t dj = 0, aj = 0;
        if (ok) {
            const int64_t j =
                A.idx_in ? A.idx_in[b] : sample_row(b, ep, count, A.seed_lo, A.seed_hi);
            s2w = reinterpret_cast<const uint32_t*>(A.s2)[j * 4 + w];
            sw = reinterpret_cast<const uint32_t*>(A.s)[j * 4 + w];
            if (w == 0) {
                A.idx_out[b] = j;
                rj = A.r[j];
                dj = A.d[j];
                aj = A.a[j];
            }
        }
        __syncthreads();  // the previous tile's grad_tile is done with T
        MPHASE(1);
        if (t < 4 * S) {
            put_word(T.x + sl * XS + w * 4, s2w);
            if (w == 0) {
                T.a[sl] = (float)aj;
                T.g[sl] = ok ? 1.f : 0.f;
            }
        }
        __syncthreads();
        MPHASE(2);
        forward_tile_mfma<S>(T, Wtg, w1tg);
        if (t < 4 * S) qtg[t] = T.q[t];
        forward_tile_mfma<S>(T, Won, w1on);
        if (t < 4 * S && w == 0) {
            const float y = bellman(T.q + sl * 4, qtg + sl * 4, rj, dj, A.gamma, A.double_dqn);
            T.y[sl] = y;
            if (ok) A.y_out[b] = y;
        }
        __syncthreads();  // T.x is restaged below; T.y visible to grad_tile
        MPHASE(3);
        if (t < 4 * S) put_word(T.x + sl * XS + w * 4, sw);
        __syncthreads();
        MPHASE(4);
        grad_tile<S>(T, Won, w1on, G);
#ifdef G2048_MLP_PHASE
        __syncthreads();
#endif
        MPHASE(5);
    }
    write_slab<S, COH>(G, T, A.slab + (int64_t)blockIdx.x * SLAB);
    MPHASE(6);
}

__global__ __launch_bounds__(NT) void k_mlp_update(UpdateArgs A) { update_tiles<false>(A); }

// block = 64 slab positions x 16 waves: wave w sums slabs w, w+16, ... (<= 16 loads, all in
// flight at once), then a fixed-order combine of the 16 partials.  With `adam`, the summed
// gradient of each parameter is applied right here (torch Adam, t read from *step_next) and
// *step_next is committed to *step.
constexpr int RW = 16;  // waves per reduction block
static_assert(MAX_SLABS <= RW * 16, "reduction covers at most RW*16 slabs");

struct ReduceArgs {
    const float* slab;
    int nslab;
    float* grad;
    float* loss;
    const unsigned long long* step_next;
    unsigned long long* step;
    float* p[4];   // w1, b1, w2, b2 (updated in place when adam)
    float* tp[4];  // target net: receives the new params when t % sync_every == 0
    unsigned long long sync_every;
    float* m;
    float* v;
    double lr, b1, b2, eps;
    int adam;
};

// The fixed-order sum of slab position `pos` (partials p_w = slab[w] + slab[w + 16] + ... for
// w = 0 .. 15, then p_0 + ... + p_15) and what follows it: the gradient / loss written and, with
// `adam`, torch Adam applied (step t) + the target sync.  `part` is LDS [RW][64]; the calling
// block's NW waves compute the partials w = wave, wave + NW, ... (all of a wave's slab loads in
// flight at once); wave 0 finishes.  k_mlp_reduce (16 waves) and k_mlp_update1's reducers (4
// waves, COH: agent-scope loads of the slabs other XCDs wrote in the same launch) run it, so both
// sum in exactly this order (bitwise the same update).
template <int NW, bool COH>
__device__ __forceinline__ void reduce_positions(const ReduceArgs& A, int chunk,
                                                 unsigned long long t, float (*part)[64]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pos = chunk * 64 + lane;
    // Adam operands (wave 0) loaded with the slabs: independent of the sums
    const bool adam = A.adam && wave == 0 && pos < P_N;
    const int k = pos < P_B1 ? 0 : pos < P_W2 ? 1 : pos < P_B2 ? 2 : 3;
    const int base[4] = {P_W1, P_B1, P_W2, P_B2};
    float am = 0.f, av = 0.f, ap = 0.f;
    if (adam) {
        am = A.m[pos];
        av = A.v[pos];
        ap = A.p[k][pos - base[k]];
    }
    constexpr int PW = RW / NW;  // partials per wave
    // unconditional loads from clamped (valid) addresses, zeroed after: a load under a per-slab
    // branch is issued alone (the compiler cannot batch loads across the branches)
    const bool okp = pos <= P_N;
    const int pc = okp ? pos : P_N;
    float r[PW][16];
#pragma unroll
    for (int i = 0; i < PW; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int g = wave + NW * i + RW * u;
            const bool ok = okp && g < A.nslab;
            const int64_t e = (int64_t)(g < A.nslab ? g : 0) * SLAB + pc;
            float x;
            if constexpr (COH)
                x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  slab_rsrc(A.slab), (uint32_t)(e * 4), 0u, AUX_SC1));
            else
                x = A.slab[e];
            r[i][u] = ok ? x : 0.f;
        }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        float v = r[i][0];
#pragma unroll
        for (int u = 1; u < 16; ++u) v += r[i][u];
        part[wave + NW * i][lane] = v;
    }
    __syncthreads();
    if (wave == 0 && pos <= P_N) {
        float sum = part[0][lane];
#pragma unroll
        for (int k2 = 1; k2 < RW; ++k2) sum += part[k2][lane];
        if (pos == P_N) {
            if (A.loss) *A.loss = sum;
        } else {
            if (A.grad) A.grad[pos] = sum;
            if (adam) {
                const g2048::AdamCoef c = g2048::adam_coef((double)t, A.lr, A.b1, A.b2, A.eps);
                const float np = g2048::adam_update(c, sum, am, av, ap);
                A.m[pos] = am;
                A.v[pos] = av;
                A.p[k][pos - base[k]] = np;
                if (A.sync_every && t % A.sync_every == 0ull) A.tp[k][pos - base[k]] = np;
            }
        }
    }
}

constexpr int RCHUNKS = (P_N + 64) / 64;  // 64-position chunks of the slab (loss included)

__global__ __launch_bounds__(64 * RW) void k_mlp_reduce(ReduceArgs A) {
    __shared__ float part[RW][64];
    reduce_positions<RW, false>(A, blockIdx.x, A.adam ? *A.step_next : 0ull, part);
    if (A.step && blockIdx.x == 0 && threadIdx.x == 0) *A.step = *A.step_next;
}

// The whole dense-64 update in ONE launch: every workgroup runs its tiles and writes its slab
// (k_mlp_update's work) with agent-scope stores (through the XCD's L2 to the coherent level, no
// L2 write-back needed), waits for them and counts its arrival; the last min(RCHUNKS, grid)
// workgroups to arrive become the reducers -- each waits until every workgroup has arrived, then
// sums its 64-position chunks with agent-scope loads exactly as k_mlp_reduce does and applies
// Adam with t = *step + 1 (read by every workgroup before it counts itself; reducer 0 commits the
// counter last).  The workgroups a reducer waits for have all started or are next in line for the
// CUs the early finishers freed, so the wait always ends; it is capped anyway (an error count in
// the workspace; the tests check it stays 0).  The last reducer to finish returns both counters
// to 0 for the next launch (the workspace must be zeroed before its first use).  Replaces the
// k_mlp_update -> k_mlp_reduce kernel boundary.
struct Update1Args {
    UpdateArgs U;
    ReduceArgs R;
    unsigned int* arrive;  // [0] arrivals, [1] reducers done, [2] error count
};

__global__ __launch_bounds__(NT) void k_mlp_update1(Update1Args A) {
    const unsigned long long t_next = *A.U.step + 1ull;
    update_tiles<true>(A.U);
    __shared__ unsigned int s_arrival;
    __shared__ float part[RW][64];
    const unsigned grid = gridDim.x;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's slab stores are complete
    __syncthreads();
    if (threadIdx.x == 0)
        s_arrival = __hip_atomic_fetch_add(&A.arrive[0], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned a = s_arrival;
    const unsigned nred = grid < (unsigned)RCHUNKS ? grid : (unsigned)RCHUNKS;
    if (a >= grid) {  // a workspace that was not zeroed: nothing here can be trusted
        if (threadIdx.x == 0) atomicAdd(&A.arrive[2], 1u);
        return;
    }
    if (a < grid - nred) return;
    const unsigned me = a - (grid - nred);  // this reducer's index
    if (threadIdx.x == 0) {
        unsigned it = 0;
        while (__hip_atomic_load(&A.arrive[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < grid) {
            __builtin_amdgcn_s_sleep(1);
            if (++it == (1u << 24)) {
                atomicAdd(&A.arrive[2], 1u);
                break;
            }
        }
    }
    __syncthreads();
    for (unsigned c = me; c < (unsigned)RCHUNKS; c += nred) {
        reduce_positions<NT / 64, true>(A.R, (int)c, t_next, part);
        __syncthreads();  // part is reused by the next chunk
    }
    if (threadIdx.x == 0) {
        if (me == 0 && A.R.step) *A.R.step = t_next;
        if (__hip_atomic_fetch_add(&A.arrive[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            nred - 1) {
            __hip_atomic_store(&A.arrive[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&A.arrive[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

namespace {
inline MlpW mlp_w(const g2048_dense64_params* p) { return MlpW{p->w1, p->b1, p->w2, p->b2}; }
inline bool ok_params(const g2048_dense64_params* p) {
    return p && p->w1 && p->b1 && p->w2 && p->b2;
}

}  // namespace

extern "C" G2048_API int g2048_dense64_forward(const g2048_dense64_params* p, const uint8_t* rows,
                                               const int64_t* idx, int64_t n, float* q_out,
                                               void* stream) {
    if (!ok_params(p) || !rows || !q_out || n <= 0)
        return g2048_fail(G2048_EINVAL, "dense64_forward: NULL argument or n <= 0");
    FwdArgs A{mlp_w(p), rows, idx, n, q_out};
    hipLaunchKernelGGL(k_mlp_forward, dim3((unsigned)((n + S_FWD - 1) / S_FWD)), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "dense64_forward: %s", hipGetErrorString(e));
}

extern "C" G2048_API int g2048_dense64_targets(const g2048_dense64_params* online,
                                               const g2048_dense64_params* target,
                                               g2048_replay* rb, const int64_t* idx_in,
                                               int64_t batch, uint64_t seed,
                                               const uint64_t* epoch_dev, float gamma,
                                               int double_dqn, int64_t* idx_out, float* y_out,
                                               void* stream) {
    if (!ok_params(online) || !ok_params(target) || !rb || batch <= 0 || !idx_out || !y_out ||
        (!idx_in && !epoch_dev))
        return g2048_fail(G2048_EINVAL, "dense64_targets: NULL argument or batch <= 0");
    uint8_t *s2 = nullptr, *d = nullptr;
    int32_t* r = nullptr;
    uint64_t* count = nullptr;
    if (g2048_replay_views(rb, nullptr, &s2, nullptr, &r, &d, &count) != G2048_OK)
        return G2048_EINVAL;
    TargetArgs A;
    A.on = mlp_w(online);
    A.tg = mlp_w(target);
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
    hipLaunchKernelGGL(k_mlp_targets, dim3((unsigned)((batch + S_FWD - 1) / S_FWD)), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "dense64_targets: %s", hipGetErrorString(e));
}

extern "C" G2048_API int64_t g2048_dense64_train_workspace(int64_t batch) {
    const int64_t ntiles = (batch + S_FWD - 1) / S_FWD;
    return (ntiles < MAX_SLABS ? ntiles : MAX_SLABS) * SLAB;
}

extern "C" G2048_API int g2048_dense64_train_grad(const g2048_dense64_params* p,
                                                  const uint8_t* rows, const uint8_t* actions,
                                                  const int64_t* idx, const float* y, int64_t batch,
                                                  float* workspace, float* grad_out,
                                                  float* loss_out, uint64_t* step_dev,
                                                  void* stream) {
    if (!ok_params(p) || !rows || !actions || !idx || !y || !workspace || !grad_out || batch <= 0)
        return g2048_fail(G2048_EINVAL, "dense64_train_grad: NULL argument or batch <= 0");
    const int64_t ntiles = (batch + S_FWD - 1) / S_FWD;
    const int grid = (int)(ntiles < MAX_SLABS ? ntiles : MAX_SLABS);
    TrainArgs A{mlp_w(p), rows, actions, idx, y, batch, workspace,
                reinterpret_cast<unsigned long long*>(step_dev)};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_mlp_train, dim3(grid), dim3(NT), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_mlp_train: %s", hipGetErrorString(e));
    ReduceArgs R{};
    R.slab = workspace;
    R.nslab = grid;
    R.grad = grad_out;
    R.loss = loss_out;
    hipLaunchKernelGGL(k_mlp_reduce, dim3((P_N + 64) / 64), dim3(64 * RW), 0, st, R);
    e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "k_mlp_reduce: %s", hipGetErrorString(e));
}

// workspace: slabs | u64 step_next | u32 arrivals, reducers done, errors, pad (k_mlp_update1)
constexpr int WS_TAIL = 2 + 4;

extern "C" G2048_API int64_t g2048_dense64_update_workspace(int64_t batch) {
    const int64_t ntiles = (batch + S_UPD - 1) / S_UPD;
#ifdef G2048_MLP_PHASE
    return (ntiles < MAX_SLABS ? ntiles : MAX_SLABS) * SLAB + WS_TAIL + 2 * 8 * MAX_SLABS;
#endif
    return (ntiles < MAX_SLABS ? ntiles : MAX_SLABS) * SLAB + WS_TAIL;
}

// G2048_DENSE64_ONE_LAUNCH=1 selects the one-launch update (k_mlp_update1; read per call, so the
// tests compare the two forms bitwise in one process).  Measured and not the default
// (tools/dense64_onelaunch_ab.py, profiles/r06/dense64_onelaunch_ab.txt): 23.7 us per update against
// 19.4 us for the two launches -- a workgroup's wait for its slab stores to be acknowledged at
// the coherent level plus the arrival atomic cost ~5.8 us, more than the kernel boundary it
// replaces.
static bool dense64_one_launch() {
    const char* e = getenv("G2048_DENSE64_ONE_LAUNCH");
    return e && e[0] == '1';
}

extern "C" G2048_API int g2048_dense64_update(const g2048_dense64_params* online,
                                              const g2048_dense64_params* target,
                                              g2048_replay* rb, const int64_t* idx_in,
                                              int64_t batch, uint64_t seed, uint64_t* step_dev,
                                              float gamma, int double_dqn, int64_t* idx_out,
                                              float* y_out, float* workspace, float* grad_out,
                                              float* loss_out, float* exp_avg, float* exp_avg_sq,
                                              double lr, double beta1, double beta2, double eps,
                                              uint64_t sync_every, void* stream) {
    if (!ok_params(online) || !ok_params(target) || !rb || batch <= 0 || !step_dev || !idx_out ||
        !y_out || !workspace)
        return g2048_fail(G2048_EINVAL, "dense64_update: NULL argument or batch <= 0");
    if ((exp_avg == nullptr) != (exp_avg_sq == nullptr) || (!exp_avg && !grad_out))
        return g2048_fail(G2048_EINVAL,
                          "dense64_update: need exp_avg and exp_avg_sq (Adam) or grad_out");
    uint8_t *s = nullptr, *a = nullptr, *s2 = nullptr, *d = nullptr;
    int32_t* r = nullptr;
    uint64_t* count = nullptr;
    if (g2048_replay_views(rb, &s, &s2, &a, &r, &d, &count) != G2048_OK) return G2048_EINVAL;
    const int64_t ntiles = (batch + S_UPD - 1) / S_UPD;
    const int grid = (int)(ntiles < MAX_SLABS ? ntiles : MAX_SLABS);
    unsigned long long* step_next =
        reinterpret_cast<unsigned long long*>(workspace + (int64_t)grid * SLAB);
    UpdateArgs U;
    U.on = mlp_w(online);
    U.tg = mlp_w(target);
    U.s = s;
    U.a = a;
    U.s2 = s2;
    U.d = d;
    U.r = r;
    U.count = reinterpret_cast<const unsigned long long*>(count);
    U.step = reinterpret_cast<const unsigned long long*>(step_dev);
    U.idx_in = idx_in;
    U.batch = batch;
    U.seed_lo = (uint32_t)seed;
    U.seed_hi = (uint32_t)(seed >> 32);
    U.gamma = gamma;
    U.double_dqn = double_dqn;
    U.idx_out = idx_out;
    U.y_out = y_out;
    U.slab = workspace;
    U.step_next = step_next;
#ifdef G2048_MLP_PHASE
    U.phase = reinterpret_cast<long long*>(workspace + (int64_t)grid * SLAB + WS_TAIL);
#endif
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    ReduceArgs R{};
    R.slab = workspace;
    R.nslab = grid;
    R.grad = grad_out;
    R.loss = loss_out;
    R.step_next = step_next;
    R.step = reinterpret_cast<unsigned long long*>(step_dev);
    R.adam = exp_avg != nullptr;
    R.p[0] = const_cast<float*>(online->w1);
    R.p[1] = const_cast<float*>(online->b1);
    R.p[2] = const_cast<float*>(online->w2);
    R.p[3] = const_cast<float*>(online->b2);
    R.sync_every = exp_avg ? sync_every : 0;
    R.tp[0] = const_cast<float*>(target->w1);
    R.tp[1] = const_cast<float*>(target->b1);
    R.tp[2] = const_cast<float*>(target->w2);
    R.tp[3] = const_cast<float*>(target->b2);
    R.m = exp_avg;
    R.v = exp_avg_sq;
    R.lr = lr;
    R.b1 = beta1;
    R.b2 = beta2;
    R.eps = eps;
    if (dense64_one_launch()) {
        Update1Args A1;
        A1.U = U;
        A1.R = R;
        A1.arrive = reinterpret_cast<unsigned int*>(step_next + 1);
        hipLaunchKernelGGL(k_mlp_update1, dim3(grid), dim3(NT), 0, st, A1);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? G2048_OK
                               : g2048_fail(G2048_EHIP, "k_mlp_update1: %s", hipGetErrorString(e));
    }
    hipLaunchKernelGGL(k_mlp_update, dim3(grid), dim3(NT), 0, st, U);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_mlp_update: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(k_mlp_reduce, dim3(RCHUNKS), dim3(64 * RW), 0, st, R);
    e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "k_mlp_reduce: %s", hipGetErrorString(e));
}
