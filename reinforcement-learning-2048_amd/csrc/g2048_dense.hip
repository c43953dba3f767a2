// g2048_dense.hip -- the forward of the reference's dense Q-net (src/configs/double_dqn_dense.py:
// 7-15: Linear(16,512) ReLU Linear(512,512) ReLU Linear(512,256) ReLU Linear(256,4)) on board rows,
// in float32 or float64: the `model(state)` of epsilon_greedy_policy (src/dqn_lib.py:20-24) for a
// Trainer whose learner trains that net on the torch path.  Two forms:
//   all rows:      Q[b] of rows[idx ? idx[b] : b], b < n;
//   greedy rows:   Q only of the env's boards whose next eps-greedy step takes the greedy branch
//                  (the step kernel's own Philox draw and eps rule) -- the only rows the policy
//                  evaluates the model on.  Early in the schedule (eps ~ 1) that is almost none.
// A row's Q does not depend on which rows share its tile (every output element sums its k in one
// fixed order), so the greedy rows are bitwise the all-rows forward's.
//
// Per tile of TB rows (64 in f32, 32 in f64: RB = TB / 16 row blocks), 8 waves (two per SIMD);
// wave w owns output columns [w N/8, (w+1) N/8) of a layer, in 16-wide blocks, on
// v_mfma_{f32,f64}_16x16x4, for all RB row blocks at once, so every weight fragment read from L2
// feeds RB MFMAs (a 16-row tile re-read the 1.6 MB (f32) of weights per 16 rows and ran at 0.43 of
// the f32 MFMA spec).  Activations stay in one LDS buffer [TB][512 + pad], each layer overwriting
// its own input (a barrier between the last read and the first write).  The weights stream from
// L2 as B fragments, one run of E k-steps ahead.  The K order is permuted within each 4E-wide k
// chunk so that every lane's A and B operands of E k-steps are E consecutive elements -- 32 bytes
// (E = 8 in f32, 4 in f64; 4 in f32's first layer, K = 16), so the four lanes of a B row read one
// 128-byte line: k-step E q + u, lane k-group lk <-> k = 4E q + E lk + u.  The last layer (N = 4)
// runs on VALU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048.h"
#include "g2048_board.hpp"
#include "g2048_common.hpp"

namespace {

constexpr int NT = 512;  // 8 waves: two per SIMD, so one wave's operand waits hide under the other's MFMAs
constexpr int NW = NT / 64;
constexpr int MAX_WG = 256;
constexpr int H1 = 512, H2 = 512, H3 = 256;
// rows per tile: as many 16-row blocks as one LDS activation buffer [TB][H1 + pad] holds
template <typename T>
constexpr int tile_rows() {
    return sizeof(T) == 4 ? 64 : 32;
}

template <typename T>
struct DenseNet {
    const T *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4;
};

// E consecutive elements (16-byte aligned) as 16-byte accesses
template <int E>
__device__ __forceinline__ void ldE(const float* p, float (&v)[E]) {
#pragma unroll
    for (int h = 0; h < E / 4; ++h) {
        const float4 x = reinterpret_cast<const float4*>(p)[h];
        v[4 * h] = x.x, v[4 * h + 1] = x.y, v[4 * h + 2] = x.z, v[4 * h + 3] = x.w;
    }
}
template <int E>
__device__ __forceinline__ void ldE(const double* p, double (&v)[E]) {
#pragma unroll
    for (int h = 0; h < E / 2; ++h) {
        const double2 x = reinterpret_cast<const double2*>(p)[h];
        v[2 * h] = x.x, v[2 * h + 1] = x.y;
    }
}

// k-steps per operand run: a lane's A and B operands of E consecutive k-steps are E consecutive
// elements (32 bytes, so the 4 lanes of a B row fill a 128-byte line), fewer when K is short
template <typename T, int K>
constexpr int run_of() {
    return sizeof(T) == 4 && K >= 64 ? 8 : 4;
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d4v __attribute__((ext_vector_type(4)));
template <typename T>
struct Acc;
template <>
struct Acc<float> {
    typedef f4v type;
    static __device__ __forceinline__ f4v mfma(float a, float b, f4v c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // lane l, register r of a 16x16 result tile: row, column
    static __device__ __forceinline__ int row(int l, int r) { return 4 * (l >> 4) + r; }
};
template <>
struct Acc<double> {
    typedef d4v type;
    static __device__ __forceinline__ d4v mfma(double a, double b, d4v c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int l, int r) { return 4 * r + (l >> 4); }
};

// LDS row strides (elements): K + pad so that the 16 rows of a 16-byte read start 4 banks apart
template <typename T>
constexpr int stride_of(int k) {
    return k + (sizeof(T) == 4 ? 4 : 2);
}

template <typename T>
struct alignas(16) Smem {
    static constexpr int TB = tile_rows<T>();
    T x[TB * stride_of<T>(16)];
    T h[TB * stride_of<T>(H1)];  // every hidden layer's output, written over its input
};

// One layer: out[r][j] = relu(sum_k in[r][k] W[j][k] + bias[j]) for the tile's TB rows (row
// stride SI in, SO out); wave w computes columns w N/8 .. ; K % 16 == 0, N % 128 == 0.
// kInPlace: out overwrites in (a barrier after the K loop).  Ends with a barrier.
template <typename T, int K, int N, int SI, int SO, bool kInPlace>
__device__ __forceinline__ void layer(const T* in, T* out, const T* __restrict__ W,
                                      const T* __restrict__ bias) {
    typedef typename Acc<T>::type AccT;
    constexpr int RB = tile_rows<T>() / 16;  // 16-row blocks per tile
    constexpr int CB = N / (16 * NW);        // 16-wide column blocks per wave
    constexpr int E = run_of<T, K>();        // k-steps per operand run
    constexpr int NQ = K / (4 * E);          // runs of E k-steps
    const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lk = l >> 4;
    AccT acc[RB][CB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[rb][c] = AccT{0, 0, 0, 0};
    // k-step E q + u of lane k-group lk is k = 4 E q + E lk + u; lane's B rows:
    // W[(w CB + c) 16 + lr][4 E q + E lk .. + E - 1]
    const T* wr = W + (size_t)(w * CB * 16 + lr) * K + E * lk;
    const T* ar = in + lr * SI + E * lk;
    T bq[2][CB][E];
#pragma unroll
    for (int c = 0; c < CB; ++c) ldE<E>(wr + (size_t)c * 16 * K, bq[0][c]);
    // one run of B fragments in flight ahead of the MFMAs; the loop is unrolled by two (static
    // buffer indices), not fully: fully unrolled, the scheduler hoisted later runs' loads and
    // the kernel spilled
    auto run = [&](int q, T (&cur)[CB][E], T (&nxt)[CB][E]) {
        if (q + 1 < NQ) {
#pragma unroll
            for (int c = 0; c < CB; ++c) ldE<E>(wr + (size_t)c * 16 * K + 4 * E * (q + 1), nxt[c]);
        }
        // row block by row block: one block's A operands live at a time
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            T av[E];
            ldE<E>(ar + rb * 16 * SI + 4 * E * q, av);
#pragma unroll
            for (int u = 0; u < E; ++u)
#pragma unroll
                for (int c = 0; c < CB; ++c) acc[rb][c] = Acc<T>::mfma(av[u], cur[c][u], acc[rb][c]);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    static_assert(NQ % 2 == 0 || NQ == 1, "runs in pairs");
    if constexpr (NQ == 1) {
        run(0, bq[0], bq[1]);
    } else {
#pragma unroll 1
        for (int q = 0; q < NQ; q += 2) {
            run(q, bq[0], bq[1]);
            run(q + 1, bq[1], bq[0]);
        }
    }
    if constexpr (kInPlace) __syncthreads();  // every wave's last read of in
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int j = (w * CB + c) * 16 + lr;
        const T bj = bias[j];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const T z = acc[rb][c][r] + bj;
                out[(rb * 16 + Acc<T>::row(l, r)) * SO + j] = z > T(0) ? z : T(0);
            }
    }
    __syncthreads();
}

// The tile's TB rows (in S.x) through the net; Q of row b -> q[qrow[b] * 4 + a] for b < nb.
template <typename T>
__device__ __forceinline__ void forward_tile(Smem<T>& S, const DenseNet<T>& P, T* q, int nb,
                                             const int32_t* qrow) {
    constexpr int TB = tile_rows<T>(), SX = stride_of<T>(16), SH = stride_of<T>(H1);
    __syncthreads();  // S.x written
    layer<T, 16, H1, SX, SH, false>(S.x, S.h, P.w1, P.b1);
    layer<T, H1, H2, SH, SH, true>(S.h, S.h, P.w2, P.b2);
    layer<T, H2, H3, SH, SH, true>(S.h, S.h, P.w3, P.b3);
    // Linear(256, 4) on VALU: thread (row b, action a, part p) sums NP consecutive k in two
    // chains; the parts are combined in a fixed order through lane shuffles
    constexpr int PARTS = NT / (TB * 4), NP = H3 / PARTS;
    const int t = threadIdx.x, part = t % PARTS, a = (t / PARTS) & 3, b = t / (4 * PARTS);
    const T* hr = S.h + b * SH + NP * part;
    const T* wr = P.w4 + a * H3 + NP * part;
    T e = T(0), o = T(0);
#pragma unroll 8
    for (int k = 0; k < NP; k += 2) {
        e = fma(wr[k], hr[k], e);
        o = fma(wr[k + 1], hr[k + 1], o);
    }
    T v = e + o;
#pragma unroll
    for (int m = 1; m < PARTS; m *= 2) v = v + __shfl_xor(v, m);
    if (part == 0 && b < nb) q[(int64_t)qrow[b] * 4 + a] = v + P.b4[a];
    __syncthreads();  // S.h / S.x free for the next tile
}

template <typename T>
struct FwdArgs {
    DenseNet<T> net;
    const uint4* rows;
    const int64_t* idx;
    int64_t n;
    T* q;
    const uint64_t* clock;  // null: every row
    const uint32_t* ep;
    uint64_t board_offset;
    uint32_t seed_lo, seed_hi;
    const double* eps_dev;
    double eps, eps_decay, eps_min;
    int64_t chunk;
};

template <typename T>
__device__ __forceinline__ void put_row(T* xr, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) xr[4 * k + j] = (T)((w[k] >> (8 * j)) & 0xFFu);
}

// The rows [c0, c1) of workgroup w: per window of NT rows the selected ones (all, or the greedy
// branch's) are queued (ballot + prefix) and run in TB-row tiles; fewer than TB left over carry
// into the next window (the k_conv64_forward scheme).  The queue holds row offsets from c0.
template <typename T>
__global__ __launch_bounds__(NT) void k_dense_forward(FwdArgs<T> A) {
    constexpr int TB = tile_rows<T>();
    __shared__ Smem<T> S;
    __shared__ int32_t queue[NT + TB];
    __shared__ int32_t qrow[TB];
    __shared__ int32_t wcnt[NW];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * A.chunk;
    const int64_t c1 = c0 + A.chunk < A.n ? c0 + A.chunk : A.n;
    int qn = 0;
    for (int64_t w0 = c0; w0 < c1; w0 += NT) {
        const bool last = w0 + NT >= c1;
        const int64_t i = w0 + t;
        bool g = i < c1;
        if (g && A.clock) {
            const uint4 u = g2048::draw(A.seed_lo, A.seed_hi, A.board_offset + (uint64_t)i,
                                        g2048::DOMAIN_STEP, A.clock[i >> 6]);
            const uint32_t e = A.eps_decay > 0.0 ? A.ep[4 * i] : 0u;
            g = !g2048::explores(u.y, g2048::step_eps(A.eps_decay, A.eps_min, A.eps_dev, A.eps, e));
        }
        const uint64_t bal = __ballot(g);
        if (lane == 0) wcnt[wv] = __popcll(bal);
        __syncthreads();
        int base = qn;
        for (int ww = 0; ww < wv; ++ww) base += wcnt[ww];
        if (g) queue[base + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)(i - c0);
        for (int ww = 0; ww < NW; ++ww) qn += wcnt[ww];
        __syncthreads();
        const int nt = last ? (qn + TB - 1) / TB : qn / TB;
        for (int j = 0; j < nt; ++j) {
            const int nb = qn - j * TB < TB ? qn - j * TB : TB;
            if (t < TB) {
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                int32_t row = 0;
                if (t < nb) {
                    const int64_t b = c0 + queue[j * TB + t];
                    v = A.rows[A.idx ? A.idx[b] : b];
                    row = (int32_t)b;
                }
                put_row(S.x + t * stride_of<T>(16), v);
                qrow[t] = row;
            }
            forward_tile<T>(S, A.net, A.q, nb, qrow);
        }
        // carry the remainder (< TB rows) to the front of the queue
        const int rem = qn - nt * TB;
        __syncthreads();
        const int32_t keep = t < rem ? queue[nt * TB + t] : 0;
        __syncthreads();
        if (t < rem) queue[t] = keep;
        qn = rem;
    }
}

template <typename T>
DenseNet<T> net_of(const g2048_densenet_params* p) {
    return DenseNet<T>{(const T*)p->w1, (const T*)p->b1, (const T*)p->w2, (const T*)p->b2,
                       (const T*)p->w3, (const T*)p->b3, (const T*)p->w4, (const T*)p->b4};
}

template <typename T>
int launch(const g2048_densenet_params* p, FwdArgs<T>& F, void* stream, const char* what) {
    F.net = net_of<T>(p);
    const int64_t tiles = (F.n + tile_rows<T>() - 1) / tile_rows<T>();
    const int grid = (int)(tiles < MAX_WG ? tiles : MAX_WG);
    F.chunk = (F.n + grid - 1) / grid;
    hipLaunchKernelGGL(k_dense_forward<T>, dim3(grid), dim3(NT), 0,
                       reinterpret_cast<hipStream_t>(stream), F);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "%s: %s", what, hipGetErrorString(e));
}

bool params_ok(const g2048_densenet_params* p) {
    return p && p->w1 && p->b1 && p->w2 && p->b2 && p->w3 && p->b3 && p->w4 && p->b4;
}

}  // namespace

extern "C" G2048_API int g2048_densenet_forward(const g2048_densenet_params* p, int dtype,
                                                const uint8_t* rows, const int64_t* idx, int64_t n,
                                                void* q_out, void* stream) {
    if (!params_ok(p) || !rows || !q_out || n < 0 || (dtype != G2048_F32 && dtype != G2048_F64))
        return g2048_fail(G2048_EINVAL, "densenet_forward: NULL argument, n < 0 or bad dtype");
    if (n == 0) return G2048_OK;
    if (n > INT32_MAX) return g2048_fail(G2048_EINVAL, "densenet_forward: n > 2^31 - 1");
    if (dtype == G2048_F32) {
        FwdArgs<float> F{};
        F.rows = reinterpret_cast<const uint4*>(rows);
        F.idx = idx;
        F.n = n;
        F.q = static_cast<float*>(q_out);
        return launch(p, F, stream, "densenet_forward");
    }
    FwdArgs<double> F{};
    F.rows = reinterpret_cast<const uint4*>(rows);
    F.idx = idx;
    F.n = n;
    F.q = static_cast<double*>(q_out);
    return launch(p, F, stream, "densenet_forward");
}

extern "C" G2048_API int g2048_densenet_forward_greedy(const g2048_densenet_params* p, int dtype,
                                                       g2048_env* env, const double* eps_dev,
                                                       double eps, double eps_decay_episodes,
                                                       double eps_min, void* q_out, void* stream) {
    if (!params_ok(p) || !env || !q_out || (dtype != G2048_F32 && dtype != G2048_F64))
        return g2048_fail(G2048_EINVAL, "densenet_forward_greedy: NULL argument or bad dtype");
    uint8_t* board = nullptr;
    uint32_t* ep = nullptr;
    uint64_t* clock = nullptr;
    uint64_t seed = 0, offset = 0;
    if (g2048_env_views(env, &board, nullptr, &ep, &clock) != G2048_OK ||
        g2048_env_rng(env, &seed, &offset) != G2048_OK)
        return G2048_EINVAL;
    const int64_t n = g2048_env_size(env);
    if (n <= 0) return g2048_fail(G2048_EINVAL, "densenet_forward_greedy: empty env");
    if (n > INT32_MAX) return g2048_fail(G2048_EINVAL, "densenet_forward_greedy: n > 2^31 - 1");
    auto fill = [&](auto& F) {
        F.rows = reinterpret_cast<const uint4*>(board);
        F.n = n;
        F.clock = clock;
        F.ep = ep;
        F.board_offset = offset;
        F.seed_lo = (uint32_t)seed;
        F.seed_hi = (uint32_t)(seed >> 32);
        F.eps_dev = eps_dev;
        F.eps = eps;
        F.eps_decay = eps_decay_episodes > 0.0 ? eps_decay_episodes : 0.0;
        F.eps_min = eps_min;
    };
    if (dtype == G2048_F32) {
        FwdArgs<float> F{};
        fill(F);
        F.q = static_cast<float*>(q_out);
        return launch(p, F, stream, "densenet_forward_greedy");
    }
    FwdArgs<double> F{};
    fill(F);
    F.q = static_cast<double*>(q_out);
    return launch(p, F, stream, "densenet_forward_greedy");
}
