// g2048_learn64.hip -- the Double-DQN update of the dense 16 -> 64 -> 4 Q-net in float64, the
// reference's precision (src/configs/double_dqn_dense.py:15 `.double()`; BASELINE configs[2] at
// width 64), fused: sampler + Q_target(s') + Q_online(s') -> y + Q_online(s) -> MSE(sum) ->
// gradient in ONE launch per 64-row tile, then a fixed-order slab reduction with torch's Adam
// (float64) and the target sync applied in place.  train_step: src/dqn_lib.py:119-164; the
// target sync: :227-228.
//
// Tile = 64 minibatch rows per 256-thread workgroup, VALU float64 (57 TF of f64 vector FMA
// against 74 TF of f64 MFMA with VGPR accumulators, and at 1 280 MAC per row the update is
// latency-bound, not FLOP-bound).  Every output element has one owner thread and every sum runs in a fixed order,
// so the update is run-to-run bitwise reproducible:
//   h[s][j] = relu(b1[j] + W1[j] . x[s])        thread (j = t & 63, rows 16 (t >> 6) ..)
//   Q[s][a] = b2[a] + W2[a] . h[s]              thread (s = t >> 2, a = t & 3)
//   dW2[a][j], db2[a]: thread (a = t >> 6, j = t & 63) over the tile's rows of action a
//   dh[s][j] = (h > 0) dq_s W2[a_s][j]          in place over h
//   dW1[j][4q .. 4q+3] += sum_s dh[s][j] x[s][.]  thread (j = t & 63, q = t >> 6); db1[j]
// Gradient accumulators persist in registers across a workgroup's tiles and are written once,
// in torch's parameter order, to the workgroup's slab (+ its loss).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"

namespace {

constexpr int NT = 256;
constexpr int S = 64;        // rows per tile
constexpr int XS = 17;       // doubles per x row in LDS (odd: the row-strided reads spread)
constexpr int HS = 65;       // doubles per h row
constexpr int P_W1 = 0, P_B1 = 1024, P_W2 = 1088, P_B2 = 1344, P_N = 1348;
constexpr int SLAB = P_N + 4;  // + the loss at P_N (doubles; rows 32-byte aligned)
constexpr int MAX_SLABS = 256;

struct Net64 {
    double *w1, *b1, *w2, *b2;
};

struct alignas(16) Smem {
    double x[S * XS];    // s' then s of the tile, as exponent doubles
    double h[S * HS];    // relu(layer 1) -> dh
    double w2[2][4 * 64];
    double b1[2][64];
    double b2[2][4];
    double qa[S * 4];    // Q_target(s')
    double qb[S * 4];    // Q_online(s') then Q_online(s)
    double y[S];
    double dq[S];
    double loss[S];
    int act[S];
};

__device__ __forceinline__ int64_t sample_row(int64_t b, unsigned long long ep,
                                              unsigned long long count, uint32_t lo, uint32_t hi) {
    // the draw of k_sample / the fp32 learners (domain 3): uniform over [0, count)
    const uint4 u = g2048::philox10(
        make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32), (uint32_t)ep,
                   (uint32_t)(ep >> 32) | (g2048::DOMAIN_SAMPLE << 30)),
        lo, hi);
    return (int64_t)__umul64hi(((unsigned long long)u.y << 32) | u.x, count);
}

__device__ __forceinline__ void put_row(double* xr, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        xr[4 * k + 0] = (double)(w[k] & 0xFFu);
        xr[4 * k + 1] = (double)((w[k] >> 8) & 0xFFu);
        xr[4 * k + 2] = (double)((w[k] >> 16) & 0xFFu);
        xr[4 * k + 3] = (double)(w[k] >> 24);
    }
}

// Q = relu(x W1^T + b1) W2^T + b2 for the tile in LDS (x rows visible) -> q[S][4]; h left in
// LDS.  w1r: this thread's row W1[j][0..15] (registers).  Ends with a sync.
__device__ __forceinline__ void forward(Smem& M, const double (&w1r)[16], int net, double* q) {
    const int t = threadIdx.x, j = t & 63, rq = t >> 6;
    const double bj = M.b1[net][j];
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr) {
        const int s = rq * 16 + rr;
        const double* xr = M.x + s * XS;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = fma(w1r[k], xr[k], acc);
        const double pre = acc + bj;
        M.h[s * HS + j] = pre > 0.0 ? pre : 0.0;
    }
    __syncthreads();
    const int s = t >> 2, a = t & 3;
    const double* hr = M.h + s * HS;
    const double* w2 = M.w2[net] + a * 64;
    double acc = 0.0;
#pragma unroll 8
    for (int jj = 0; jj < 64; ++jj) acc = fma(w2[jj], hr[jj], acc);
    q[s * 4 + a] = acc + M.b2[net][a];
    __syncthreads();
}

struct UpdArgs64 {
    Net64 on, tg;
    const uint4 *s, *s2;
    const uint8_t *a, *d;
    const int32_t* r;
    const unsigned long long* count;
    const unsigned long long* step;
    const int64_t* idx_in;
    int64_t batch;
    uint32_t seed_lo, seed_hi;
    float gamma;
    int double_dqn;
    int64_t* idx_out;
    double* y_out;
    double* slab;
    unsigned long long* step_next;
};

// A slab element: a plain store, or (COH) a device-scope sc1 store through the XCD's L2 to the
// coherent level, read back by the same launch's reducers with sc1 loads (as g2048_mlp.hip's
// slab_put: buffer forms, so the reducers' loads batch).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int AUX_SC1 = 16;  // gfx950 buffer cache-policy word: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const double* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
// sl: the workgroup's slab (wave-uniform: the resource stays in SGPRs; a per-lane base would
// need a waterfall loop over the lanes' resources); e: the element
template <bool COH>
__device__ __forceinline__ void slab_put(double* sl, int e, double v) {
    if constexpr (COH)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), slab_rsrc(sl),
                                              (uint32_t)e * 8u, 0u, AUX_SC1);
    else
        sl[e] = v;
}

// a workgroup's tiles and its gradient slab (k_dense64_update_f64, and the first half of
// k_dense64_update1_f64; COH: the slab written through to the coherent level)
template <bool COH>
__device__ __forceinline__ void update_tiles64(const UpdArgs64& A) {
    __shared__ Smem M;
    const int t = threadIdx.x, j = t & 63, qd = t >> 6;
    const unsigned long long ep = A.idx_in ? 0ull : *A.step;
    const unsigned long long count = A.idx_in ? 0ull : *A.count;
    if (blockIdx.x == 0 && t == 0) *A.step_next = *A.step + 1ull;
    // stage: W2, b1, b2 of both nets in LDS; this thread's W1 rows in registers
    const Net64 nets[2] = {A.tg, A.on};  // net 0 = target, net 1 = online
    double w1t[16], w1o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        w1t[k] = A.tg.w1[j * 16 + k];
        w1o[k] = A.on.w1[j * 16 + k];
    }
    for (int i = t; i < 2 * 256; i += NT) M.w2[i >> 8][i & 255] = nets[i >> 8].w2[i & 255];
    if (t < 128) M.b1[t >> 6][t & 63] = nets[t >> 6].b1[t & 63];
    if (t < 8) M.b2[t >> 2][t & 3] = nets[t >> 2].b2[t & 3];
    double w2o[4];  // W2_online[a][j] for dh
#pragma unroll
    for (int a = 0; a < 4; ++a) w2o[a] = A.on.w2[a * 64 + j];
    // gradient accumulators (fixed order across the workgroup's tiles)
    double g_w1[4] = {0.0, 0.0, 0.0, 0.0}, g_b1 = 0.0, g_w2 = 0.0, g_b2 = 0.0, g_loss = 0.0;
    const int64_t ntiles = (A.batch + S - 1) / S;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t b = tile * S + t;
        uint4 sv = make_uint4(0u, 0u, 0u, 0u);
        double rj = 0.0;
        float disc = 0.f;
        bool ok = false;
        __syncthreads();  // the previous tile is done with M
        if (t < S) {
            uint4 s2v = make_uint4(0u, 0u, 0u, 0u);
            int aj = 0;
            ok = b < A.batch;
            if (ok) {
                const int64_t row =
                    A.idx_in ? A.idx_in[b] : sample_row(b, ep, count, A.seed_lo, A.seed_hi);
                A.idx_out[b] = row;
                s2v = A.s2[row];
                sv = A.s[row];
                aj = A.a[row];
                rj = (double)A.r[row];
                // (1 - dones) * discount_factor: float32 in torch (src/dqn_lib.py:131)
                disc = (float)(1 - (int)A.d[row]) * A.gamma;
            }
            put_row(M.x + t * XS, s2v);
            M.act[t] = aj;
        }
        __syncthreads();
        forward(M, w1t, 0, M.qa);  // Q_target(s')
        forward(M, w1o, 1, M.qb);  // Q_online(s')
        if (t < S) {
            const double* qo = M.qb + t * 4;
            const double* qt = M.qa + t * 4;
            double next;
            if (A.double_dqn) {
                const uint32_t as = g2048::argmax4_torch(qo[0], qo[1], qo[2], qo[3]);
                next = qt[as];
            } else {
                next = g2048::qmax4_torch(qt[0], qt[1], qt[2], qt[3]);
            }
            double y;
            {
#pragma clang fp contract(off)
                y = rj + (double)disc * next;
            }
            M.y[t] = y;
            if (ok) A.y_out[b] = y;
            put_row(M.x + t * XS, sv);
        }
        __syncthreads();
        forward(M, w1o, 1, M.qb);  // Q_online(s), h = its hidden layer
        if (t < S) {
            double dq = 0.0, l = 0.0;
            if (ok) {
#pragma clang fp contract(off)
                const double e = M.qb[t * 4 + M.act[t]] - M.y[t];
                dq = 2.0 * e;  // d sum (q - y)^2 / dq
                l = e * e;
            }
            M.dq[t] = dq;
            M.loss[t] = l;
        }
        __syncthreads();
        // layer 2: dW2[a][j], db2[a] (thread (a = qd, j))
        {
            double acc = 0.0, accb = 0.0;
            for (int s = 0; s < S; ++s) {
                if (M.act[s] == qd) {
                    acc = fma(M.dq[s], M.h[s * HS + j], acc);
                    accb += M.dq[s];
                }
            }
            g_w2 += acc;
            if (j == 0) g_b2 += accb;
        }
        if (t == 0) {
            double l = 0.0;
            for (int s = 0; s < S; ++s) l += M.loss[s];
            g_loss += l;
        }
        __syncthreads();  // h is overwritten with dh below
#pragma unroll 4
        for (int rr = 0; rr < 16; ++rr) {
            const int s = qd * 16 + rr;
            double& hv = M.h[s * HS + j];
            const double w = M.act[s] == 0 ? w2o[0] : M.act[s] == 1 ? w2o[1]
                           : M.act[s] == 2 ? w2o[2] : w2o[3];
            hv = hv > 0.0 ? M.dq[s] * w : 0.0;
        }
        __syncthreads();
        // layer 1: dW1[j][4 qd + i], db1[j]
        {
            double acc[4] = {0.0, 0.0, 0.0, 0.0}, accb = 0.0;
            for (int s = 0; s < S; ++s) {
                const double dh = M.h[s * HS + j];
                const double* xr = M.x + s * XS + 4 * qd;
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = fma(dh, xr[i], acc[i]);
                accb += dh;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) g_w1[i] += acc[i];
            if (qd == 0) g_b1 += accb;
        }
    }
    // slab in torch order: 0.weight [64][16], 0.bias [64], 2.weight [4][64], 2.bias [4], loss
    double* sl = A.slab + (int64_t)blockIdx.x * SLAB;
#pragma unroll
    for (int i = 0; i < 4; ++i) slab_put<COH>(sl, P_W1 + j * 16 + 4 * qd + i, g_w1[i]);
    if (qd == 0) slab_put<COH>(sl, P_B1 + j, g_b1);
    slab_put<COH>(sl, P_W2 + qd * 64 + j, g_w2);
    if (j == 0) slab_put<COH>(sl, P_B2 + qd, g_b2);
    if (t == 0) slab_put<COH>(sl, P_N, g_loss);
}

__global__ __launch_bounds__(NT) void k_dense64_update_f64(UpdArgs64 A) { update_tiles64<false>(A); }

constexpr int RW = 16;  // waves per reduction block
static_assert(MAX_SLABS <= RW * 16, "reduction covers at most RW*16 slabs");

struct RedArgs64 {
    const double* slab;
    int nslab;
    double* grad;
    double* loss;
    const unsigned long long* step_next;
    unsigned long long* step;
    double* p[4];
    double* tp[4];
    unsigned long long sync_every;
    double* m;
    double* v;
    double lr, b1, b2, eps;
    int adam;
};

// The fixed-order sum of slab position chunk*64 + lane: partials p_w = 0 + slab[w] + slab[w + 16]
// + ... (w = 0 .. 15, all of a wave's loads in flight at once), then p_0 + ... + p_15 by wave 0,
// which writes the gradient / loss and (adam) applies the update (step t) to the parameter in
// place; wave 0's Adam operands are loaded with the slabs.  The calling block's NW waves take the
// partials w = wave, wave + NW, ...: k_dense64_reduce_f64 (16 waves) and k_dense64_update1_f64's
// reducers (4 waves, COH: sc1 loads of slabs written in the same launch) sum in exactly this order.
template <int NW, bool COH>
__device__ __forceinline__ void reduce_positions64(const RedArgs64& A, int chunk,
                                                   unsigned long long t, double (*part)[64]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pos = chunk * 64 + lane;
    const int k = pos < P_B1 ? 0 : pos < P_W2 ? 1 : pos < P_B2 ? 2 : 3;
    const int base[4] = {P_W1, P_B1, P_W2, P_B2};
    const bool adam = A.adam && wave == 0 && pos < P_N;
    double am = 0.0, av = 0.0, ap = 0.0;
    if (adam) {
        am = A.m[pos];
        av = A.v[pos];
        ap = A.p[k][pos - base[k]];
    }
    constexpr int PW = RW / NW;
    // unconditional loads from clamped (valid) addresses, zeroed after (batched, not branched)
    const bool okp = pos <= P_N;
    const int pc = okp ? pos : P_N;
    double v[PW][16];
#pragma unroll
    for (int i = 0; i < PW; ++i)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int g = wave + NW * i + RW * u;
            const bool ok = okp && g < A.nslab;
            const int64_t e = (int64_t)(g < A.nslab ? g : 0) * SLAB + pc;
            double x;
            if constexpr (COH)
                x = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                   slab_rsrc(A.slab), (uint32_t)(e * 8), 0u, AUX_SC1));
            else
                x = A.slab[e];
            v[i][u] = ok ? x : 0.0;
        }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        double r = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) r += v[i][u];
        part[wave + NW * i][lane] = r;
    }
    __syncthreads();
    if (wave == 0 && pos <= P_N) {
        double sum = part[0][lane];
        for (int j = 1; j < RW; ++j) sum += part[j][lane];
        if (pos == P_N) {
            if (A.loss) *A.loss = sum;
        } else {
            if (A.grad) A.grad[pos] = sum;
            if (adam) {
                const double np = g2048::adam64((double)t, A.lr, A.b1, A.b2, A.eps, sum, am, av, ap);
                A.m[pos] = am;
                A.v[pos] = av;
                A.p[k][pos - base[k]] = np;
                if (A.sync_every && t % A.sync_every == 0ull) A.tp[k][pos - base[k]] = np;
            }
        }
    }
}

constexpr int RCHUNKS = (P_N + 1 + 63) / 64;  // 64-position chunks of the slab (loss included)

__global__ __launch_bounds__(64 * RW) void k_dense64_reduce_f64(RedArgs64 A) {
    __shared__ double part[RW][64];
    reduce_positions64<RW, false>(A, blockIdx.x, A.adam ? *A.step_next : 0ull, part);
    if (A.step && blockIdx.x == 0 && threadIdx.x == 0) *A.step = *A.step_next;
}

// The whole float64 update in ONE launch, as k_mlp_update1 (g2048_mlp.hip): every workgroup
// writes its slab with sc1 stores, waits for them and counts its arrival; the last
// min(RCHUNKS, grid) to arrive reduce (after every arrival, sc1 loads) in k_dense64_reduce_f64's
// order with t = *step + 1; the last reducer returns the counters (workspace tail, zeroed before
// first use) to 0.
struct Upd1Args64 {
    UpdArgs64 U;
    RedArgs64 R;
    unsigned int* arrive;  // [0] arrivals, [1] reducers done, [2] error count
};

__global__ __launch_bounds__(NT) void k_dense64_update1_f64(Upd1Args64 A) {
    const unsigned long long t_next = *A.U.step + 1ull;
    update_tiles64<true>(A.U);
    __shared__ unsigned int s_arrival;
    __shared__ double part[RW][64];
    const unsigned grid = gridDim.x;
    __builtin_amdgcn_s_waitcnt(0);  // this wave's slab stores are complete
    __syncthreads();
    if (threadIdx.x == 0)
        s_arrival = __hip_atomic_fetch_add(&A.arrive[0], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned a = s_arrival;
    const unsigned nred = grid < (unsigned)RCHUNKS ? grid : (unsigned)RCHUNKS;
    if (a >= grid) {  // a workspace that was not zeroed
        if (threadIdx.x == 0) atomicAdd(&A.arrive[2], 1u);
        return;
    }
    if (a < grid - nred) return;
    const unsigned me = a - (grid - nred);
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
        reduce_positions64<NT / 64, true>(A.R, (int)c, t_next, part);
        __syncthreads();
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

extern "C" G2048_API int64_t g2048_dense64_update_f64_workspace(int64_t batch) {
    // slabs (<= 256 workgroups) + the next-step word + the one-launch form's u32 counters
    // (arrivals, reducers done, errors, pad), in doubles
    const int64_t tiles = (batch + S - 1) / S;
    const int64_t grid = tiles < MAX_SLABS ? tiles : MAX_SLABS;
    return grid * SLAB + 1 + 2;
}

extern "C" G2048_API int g2048_dense64_update_f64(
    const g2048_dense64_params_f64* online, const g2048_dense64_params_f64* target,
    g2048_replay* rb, const int64_t* idx_in, int64_t batch, uint64_t seed, uint64_t* step_dev,
    float gamma, int double_dqn, int64_t* idx_out, double* y_out, double* workspace,
    double* grad_out, double* loss_out, double* exp_avg, double* exp_avg_sq, double lr,
    double beta1, double beta2, double eps, uint64_t sync_every, void* stream) {
    if (!online || !target || !rb || batch <= 0 || !step_dev || !idx_out || !y_out || !workspace)
        return g2048_fail(G2048_EINVAL, "dense64_update_f64: NULL argument or batch <= 0");
    if (!online->w1 || !online->b1 || !online->w2 || !online->b2 || !target->w1 || !target->b1 ||
        !target->w2 || !target->b2)
        return g2048_fail(G2048_EINVAL, "dense64_update_f64: NULL parameter pointer");
    const bool adam = exp_avg && exp_avg_sq;
    if (!adam && !grad_out)
        return g2048_fail(G2048_EINVAL,
                          "dense64_update_f64: need exp_avg and exp_avg_sq (Adam) or grad_out");
    uint8_t *s = nullptr, *s2 = nullptr, *a = nullptr, *d = nullptr;
    int32_t* r = nullptr;
    uint64_t* count = nullptr;
    if (g2048_replay_views(rb, &s, &s2, &a, &r, &d, &count) != G2048_OK) return G2048_EINVAL;
    const int64_t tiles = (batch + S - 1) / S;
    const int grid = (int)(tiles < MAX_SLABS ? tiles : MAX_SLABS);
    UpdArgs64 U;
    U.on = Net64{online->w1, online->b1, online->w2, online->b2};
    U.tg = Net64{target->w1, target->b1, target->w2, target->b2};
    U.s = reinterpret_cast<const uint4*>(s);
    U.s2 = reinterpret_cast<const uint4*>(s2);
    U.a = a;
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
    U.step_next = reinterpret_cast<unsigned long long*>(workspace + (int64_t)grid * SLAB);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    RedArgs64 R;
    R.slab = workspace;
    R.nslab = grid;
    R.grad = grad_out;
    R.loss = loss_out;
    R.step_next = U.step_next;
    R.step = reinterpret_cast<unsigned long long*>(step_dev);
    double* ps[4] = {online->w1, online->b1, online->w2, online->b2};
    double* ts[4] = {target->w1, target->b1, target->w2, target->b2};
    for (int k = 0; k < 4; ++k) {
        R.p[k] = ps[k];
        R.tp[k] = ts[k];
    }
    R.sync_every = adam ? sync_every : 0ull;
    R.m = exp_avg;
    R.v = exp_avg_sq;
    R.lr = lr;
    R.b1 = beta1;
    R.b2 = beta2;
    R.eps = eps;
    R.adam = adam ? 1 : 0;
    // G2048_DENSE64_ONE_LAUNCH=1: the one-launch form (measured slower, as in g2048_mlp.hip)
    const char* one = getenv("G2048_DENSE64_ONE_LAUNCH");
    if (one && one[0] == '1') {
        Upd1Args64 A1;
        A1.U = U;
        A1.R = R;
        A1.arrive = reinterpret_cast<unsigned int*>(U.step_next + 1);
        hipLaunchKernelGGL(k_dense64_update1_f64, dim3(grid), dim3(NT), 0, st, A1);
    } else {
        hipLaunchKernelGGL(k_dense64_update_f64, dim3(grid), dim3(NT), 0, st, U);
        hipLaunchKernelGGL(k_dense64_reduce_f64, dim3(RCHUNKS), dim3(64 * RW), 0, st, R);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "dense64_update_f64: %s", hipGetErrorString(e));
}
