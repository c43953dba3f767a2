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

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"

namespace {

constexpr int S = 64, NT = 256, H = 64;
constexpr int XS = 17, W1S = 17, HS = 65, W2S = 65;
// torch order: 0.weight [64][16], 0.bias [64], 2.weight [4][64], 2.bias [4]
constexpr int P_W1 = 0, P_B1 = 1024, P_W2 = 1088, P_B2 = 1344, P_N = 1348;
constexpr int SLAB = 1352;  // params + loss, padded

struct MlpW {
    const float *w1, *b1, *w2, *b2;
};

struct Lds {
    float x[S * XS];
    float w1[H * W1S];
    float b1[H];
    float w2[4 * W2S];
    float b2[4];
    float h[S * HS];
    float q[S * 4];
    float a[S], y[S], g[S];
};

__device__ __forceinline__ void stage_weights(const MlpW& W, Lds& L) {
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

__device__ __forceinline__ void stage_boards(Lds& L, const uint8_t* rows, const int64_t* idx,
                                             int64_t b0, int64_t n) {
    const int t = threadIdx.x;  // 64 boards x 4 words
    const int s = t >> 2, w = t & 3;
    const int64_t b = b0 + s;
    uint32_t v = 0;
    if (b < n) v = reinterpret_cast<const uint32_t*>(rows)[(idx ? idx[b] : b) * 4 + w];
    float* dst = L.x + s * XS + w * 4;
    dst[0] = (float)(v & 0xFFu);
    dst[1] = (float)((v >> 8) & 0xFFu);
    dst[2] = (float)((v >> 16) & 0xFFu);
    dst[3] = (float)(v >> 24);
}

// weights + boards staged (caller syncs); leaves h (post-ReLU) and q in LDS, ends with a sync
__device__ __forceinline__ void forward_tile(Lds& L) {
    const int t = threadIdx.x;
    {
        const int j = t & 63, s0 = (t >> 6) * 16;
        float w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = L.w1[j * W1S + i];
        const float bb = L.b1[j];
#pragma unroll 4
        for (int ss = 0; ss < 16; ++ss) {
            const int s = s0 + ss;
            float v = bb;
#pragma unroll
            for (int i = 0; i < 16; ++i) v = fmaf(w[i], L.x[s * XS + i], v);
            L.h[s * HS + j] = fmaxf(v, 0.f);
        }
    }
    __syncthreads();
    {
        const int s = t >> 2, a = t & 3;
        float v = L.b2[a];
#pragma unroll 16
        for (int j = 0; j < H; ++j) v = fmaf(L.w2[a * W2S + j], L.h[s * HS + j], v);
        L.q[t] = v;
    }
    __syncthreads();
}

struct FwdArgs {
    MlpW W;
    const uint8_t* rows;
    const int64_t* idx;
    int64_t n;
    float* q;
};

__global__ __launch_bounds__(NT) void k_mlp_forward(FwdArgs A) {
    __shared__ Lds L;
    const int64_t b0 = (int64_t)blockIdx.x * S;
    stage_weights(A.W, L);
    stage_boards(L, A.rows, A.idx, b0, A.n);
    __syncthreads();
    forward_tile(L);
    const int t = threadIdx.x;
    if (b0 + (t >> 2) < A.n) A.q[b0 * 4 + t] = L.q[t];
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
    __shared__ Lds L;
    __shared__ float qon[S * 4];
    __shared__ int64_t sidx[S];
    const int t = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * S;
    if (t < S) {
        const int64_t b = b0 + t;
        int64_t j = 0;
        if (b < A.batch) {
            if (A.idx_in) {
                j = A.idx_in[b];
            } else {  // same draw as k_sample (domain 3)
                const unsigned long long ep = *A.epoch;
                const uint4 u = g2048::philox10(
                    make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32), (uint32_t)ep,
                               (uint32_t)(ep >> 32) | (g2048::DOMAIN_SAMPLE << 30)),
                    A.seed_lo, A.seed_hi);
                j = (int64_t)__umul64hi(((unsigned long long)u.y << 32) | u.x, *A.count);
            }
            A.idx_out[b] = j;
        }
        sidx[t] = j;
    }
    stage_weights(A.on, L);
    __syncthreads();
    stage_boards(L, A.s2, sidx, 0, S);
    __syncthreads();
    forward_tile(L);
    qon[t] = L.q[t];
    stage_weights(A.tg, L);  // forward_tile ended with a sync: the online weights are dead
    __syncthreads();
    forward_tile(L);
    if (t < S && b0 + t < A.batch) {
#pragma clang fp contract(off)
        const float* qo = qon + t * 4;
        const float* qt = L.q + t * 4;
        float next;
        if (A.double_dqn) {
            int a = 0;
            float best = qo[0];
            for (int k = 1; k < 4; ++k)
                if (qo[k] > best) { best = qo[k]; a = k; }
            next = qt[a];
        } else {
            next = fmaxf(fmaxf(qt[0], qt[1]), fmaxf(qt[2], qt[3]));
        }
        const int64_t j = sidx[t];
        const float disc = (float)(1 - (int)A.d[j]) * A.gamma;
        A.y[b0 + t] = (float)A.r[j] + disc * next;
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
    __shared__ Lds L;
    const int t = threadIdx.x;
    if (A.step && blockIdx.x == 0 && t == 0) *A.step += 1ull;
    stage_weights(A.W, L);
    float gW1[4] = {0, 0, 0, 0}, gB1 = 0.f, gW2 = 0.f, gB2 = 0.f, gLoss = 0.f;
    const int64_t ntiles = (A.batch + S - 1) / S;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b0 = tile * S;
        __syncthreads();
        stage_boards(L, A.rows, A.idx, b0, A.batch);
        if (t < S) {
            const int64_t b = b0 + t;
            const bool ok = b < A.batch;
            L.a[t] = ok ? (float)A.actions[A.idx[b]] : 0.f;
            L.y[t] = ok ? A.y[b] : 0.f;
            L.g[t] = ok ? 1.f : 0.f;
        }
        __syncthreads();
        forward_tile(L);
        if (t < S) {  // loss and dq = 2 (q - y) at the taken action
            const float d = (L.q[t * 4 + (int)L.a[t]] - L.y[t]) * L.g[t];
            gLoss = fmaf(d, d, gLoss);
            L.g[t] = 2.f * d;
        }
        __syncthreads();
        {  // dW2[a][j] / db2[a]: thread (a = t>>6, j = t&63)
            const int a = t >> 6, j = t & 63;
            float gw = 0.f, gb = 0.f;
#pragma unroll 8
            for (int s = 0; s < S; ++s) {
                const float g = (int)L.a[s] == a ? L.g[s] : 0.f;
                gw = fmaf(g, L.h[s * HS + j], gw);
                gb += g;
            }
            gW2 += gw;
            if (j == 0) gB2 += gb;
        }
        __syncthreads();
        {  // dh = dq * W2[a] * relu'(h), in place
            const int j = t & 63, s0 = (t >> 6) * 16;
#pragma unroll 4
            for (int ss = 0; ss < 16; ++ss) {
                const int s = s0 + ss;
                const float hv = L.h[s * HS + j];
                L.h[s * HS + j] = hv > 0.f ? L.g[s] * L.w2[(int)L.a[s] * W2S + j] : 0.f;
            }
        }
        __syncthreads();
        {  // dW1[j][i0..i0+3]: thread (j = t>>2, i0 = 4*(t&3)); db1 by threads j < 64
            const int j = t >> 2, i0 = (t & 3) * 4;
#pragma unroll 8
            for (int s = 0; s < S; ++s) {
                const float dh = L.h[s * HS + j];
#pragma unroll
                for (int u = 0; u < 4; ++u) gW1[u] = fmaf(dh, L.x[s * XS + i0 + u], gW1[u]);
            }
            if (t < H) {
                float v = 0.f;
#pragma unroll 8
                for (int s = 0; s < S; ++s) v += L.h[s * HS + t];
                gB1 += v;
            }
        }
    }
    float* slab = A.slab + (int64_t)blockIdx.x * SLAB;
    {
        const int j = t >> 2, i0 = (t & 3) * 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) slab[P_W1 + j * 16 + i0 + u] = gW1[u];
    }
    if (t < H) slab[P_B1 + t] = gB1;
    slab[P_W2 + t] = gW2;  // t = a*64 + j
    if ((t & 63) == 0) slab[P_B2 + (t >> 6)] = gB2;
    __syncthreads();
    L.q[t] = gLoss;  // reuse as scratch (threads >= 64 hold 0)
    __syncthreads();
    if (t == 0) {
        float v = 0.f;
        for (int i = 0; i < S; ++i) v += L.q[i];
        slab[P_N] = v;
    }
}

// block = 64 slab positions x 4 waves (wave w sums slabs w, w+4, ...), fixed-order combine
__global__ __launch_bounds__(256) void k_mlp_reduce(const float* slab, int nslab, float* grad,
                                                    float* loss) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pos = blockIdx.x * 64 + lane;
    float v = 0.f;
    if (pos <= P_N) {
        int g = wave;
        for (; g + 28 < nslab; g += 32) {
            float r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) r[u] = slab[(int64_t)(g + 4 * u) * SLAB + pos];
#pragma unroll
            for (int u = 0; u < 8; ++u) v += r[u];
        }
        for (; g < nslab; g += 4) v += slab[(int64_t)g * SLAB + pos];
    }
    part[wave][lane] = v;
    __syncthreads();
    if (wave == 0 && pos <= P_N) {
        const float sum = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
        if (pos == P_N) {
            if (loss) *loss = sum;
        } else {
            grad[pos] = sum;
        }
    }
}

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
    hipLaunchKernelGGL(k_mlp_forward, dim3((unsigned)((n + S - 1) / S)), dim3(NT), 0,
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
    hipLaunchKernelGGL(k_mlp_targets, dim3((unsigned)((batch + S - 1) / S)), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "dense64_targets: %s", hipGetErrorString(e));
}

extern "C" G2048_API int64_t g2048_dense64_train_workspace(int64_t batch) {
    const int64_t ntiles = (batch + S - 1) / S;
    return (ntiles < 256 ? ntiles : 256) * SLAB;
}

extern "C" G2048_API int g2048_dense64_train_grad(const g2048_dense64_params* p,
                                                  const uint8_t* rows, const uint8_t* actions,
                                                  const int64_t* idx, const float* y, int64_t batch,
                                                  float* workspace, float* grad_out,
                                                  float* loss_out, uint64_t* step_dev,
                                                  void* stream) {
    if (!ok_params(p) || !rows || !actions || !idx || !y || !workspace || !grad_out || batch <= 0)
        return g2048_fail(G2048_EINVAL, "dense64_train_grad: NULL argument or batch <= 0");
    const int64_t ntiles = (batch + S - 1) / S;
    const int grid = (int)(ntiles < 256 ? ntiles : 256);
    TrainArgs A{mlp_w(p), rows, actions, idx, y, batch, workspace,
                reinterpret_cast<unsigned long long*>(step_dev)};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_mlp_train, dim3(grid), dim3(NT), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return g2048_fail(G2048_EHIP, "k_mlp_train: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(k_mlp_reduce, dim3((P_N + 64) / 64), dim3(256), 0, st, workspace, grid,
                       grad_out, loss_out);
    e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "k_mlp_reduce: %s", hipGetErrorString(e));
}
