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
#include <stdlib.h>

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

template <typename T, int TB = tile_rows<T>()>
struct alignas(16) Smem {
    T x[TB * stride_of<T>(16)];
    T h[TB * stride_of<T>(H1)];  // every hidden layer's output, written over its input
};

// One layer: out[r][j] = relu(sum_k in[r][k] W[j][k] + bias[j]) for the tile's TB rows (row
// stride SI in, SO out); wave w computes columns w N/8 .. ; K % 16 == 0, N % 128 == 0.
// kInPlace: out overwrites in (a barrier after the K loop).  Ends with a barrier.
template <typename T, int K, int N, int SI, int SO, bool kInPlace, int TB = tile_rows<T>()>
__device__ __forceinline__ void layer(const T* in, T* out, const T* __restrict__ W,
                                      const T* __restrict__ bias) {
    typedef typename Acc<T>::type AccT;
    constexpr int RB = TB / 16;  // 16-row blocks per tile
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

// The tile's TB rows (in x, row stride SX) through the net (activations in h, row stride SH);
// Q of row b -> q[qrow[b] * 4 + a] for b < nb.  A row's Q does not depend on TB (every output
// element sums its k in one fixed order), so a 16-row tile run in a 32-row tile's buffers
// (k_dense_forward's remainder tiles) gives the rows the same bits.
// TBL: the tile size whose thread layout the last (VALU) layer uses -- a 16-row remainder tile
// in a 32-row kernel keeps the 32-row tile's split of the k-sum (PARTS), so its rows' Q are
// bitwise those of a full tile.
template <typename T, int TB, int TBL = TB>
__device__ __forceinline__ void forward_tile(T* x, T* h, const DenseNet<T>& P, T* q, int nb,
                                             const int32_t* qrow) {
    constexpr int SX = stride_of<T>(16), SH = stride_of<T>(H1);
    __syncthreads();  // x written
    layer<T, 16, H1, SX, SH, false, TB>(x, h, P.w1, P.b1);
    layer<T, H1, H2, SH, SH, true, TB>(h, h, P.w2, P.b2);
    layer<T, H2, H3, SH, SH, true, TB>(h, h, P.w3, P.b3);
    // Linear(256, 4) on VALU: thread (row b, action a, part p) sums NP consecutive k in two
    // chains; the parts are combined in a fixed order through lane shuffles
    constexpr int PARTS = NT / (TBL * 4), NP = H3 / PARTS;
    const int t = threadIdx.x, part = t % PARTS, a = (t / PARTS) & 3, b = t / (4 * PARTS);
    const T* hr = h + b * SH + NP * part;
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
    __syncthreads();  // h / x free for the next tile
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
    // two nets in one launch (the update's Double-DQN target side): workgroups [0, nb1) run `net`
    // into q, workgroups [nb1, 2 nb1) the same rows through net2 into q2 (nb1 = 0: one net)
    DenseNet<T> net2;
    T* q2;
    int nb1;
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
// TB: rows per tile (tile_rows<T>() for the rollout; the update's target-side forwards run
// 32-row tiles in float32 too, so B = 8192 rows fill all 256 CUs)
template <typename T, int TB = tile_rows<T>()>
__global__ __launch_bounds__(NT) void k_dense_forward(FwdArgs<T> A) {
    __shared__ Smem<T, TB> S;
    __shared__ int32_t queue[NT + TB];
    __shared__ int32_t qrow[TB];
    __shared__ int32_t wcnt[NW];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const bool second = A.nb1 > 0 && (int)blockIdx.x >= A.nb1;  // workgroup-uniform
    const int64_t c0 = (int64_t)(second ? (int)blockIdx.x - A.nb1 : (int)blockIdx.x) * A.chunk;
    const int64_t c1 = c0 + A.chunk < A.n ? c0 + A.chunk : A.n;
    const DenseNet<T> net = second ? A.net2 : A.net;
    T* const q = second ? A.q2 : A.q;
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
            // a remainder of <= 16 rows in a 32-row kernel runs as a 16-row tile: half the
            // MFMAs for the same weight stream (the update's target-side forwards at batches
            // whose 32-row tiles would spill into a partial second round, e.g. B = 5000)
            if constexpr (TB == 32) {
                if (nb <= 16) {
                    forward_tile<T, 16, 32>(S.x, S.h, net, q, nb, qrow);
                    continue;
                }
            }
            forward_tile<T, TB>(S.x, S.h, net, q, nb, qrow);
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


// ================================================================== the update (train_step)
// One Double-DQN update of the reference dense net (src/configs/double_dqn_dense.py:7-15, trained
// by src/dqn_lib.py:119-164, + the target sync of :227-228) in float32 or float64, five launches:
//   k_dense_sample   the minibatch rows (Philox, the fused learners' draw, or idx_in) + the next
//                    update counter
//   k_dense_forward  Q_online(s') and Q_target(s') of the sampled rows in one launch (the rollout
//                    forward, half the workgroups per net; vanilla DQN: Q_target(s') alone)
//   k_dense_rows     per TR-row tile: y (Double / vanilla DQN), Q_online(s) with H1 / H2 stored,
//                    MSE(sum) -> dq; dW4 / db4 (VALU); dZ3 = dq W4[a] relu'(h3) (stored);
//                    dZ2 = (dZ3 W3) relu'(h2) (stored) and dZ1 = (dZ2 W2) relu'(h1) on MFMA --
//                    the forward's tile, the weights read row-major as B fragments; dW1 = dZ1^T X
//                    and the column sums of dZ1..3 (bias gradients) per workgroup -> its slab
//   k_dense_wgrad    dW2 = dZ2^T H1, dW3 = dZ3^T H2: K = B GEMMs split in NSPLIT row ranges, one
//                    128 x 128 block per workgroup, operands staged through LDS -> partials
//   k_dense_reduce   fixed-order sums of the partials and the slabs -> the gradient in torch
//                    order; Adam (+ target sync) on the device update counter
// Every sum has a fixed order: an update is run-to-run bitwise reproducible.
constexpr int TR = 32;                  // rows per k_dense_rows tile (two 16-row MFMA blocks)
constexpr int NP_W1 = 512 * 16, NP_W2 = 512 * 512, NP_W3 = 256 * 512, NP_W4 = 4 * 256;
constexpr int P_W1 = 0, P_B1 = P_W1 + NP_W1, P_W2 = P_B1 + 512, P_B2 = P_W2 + NP_W2,
              P_W3 = P_B2 + 512, P_B3 = P_W3 + NP_W3, P_W4 = P_B3 + 256, P_B4 = P_W4 + NP_W4,
              P_ALL = P_B4 + 4;  // 403 716
// k_dense_rows slab per workgroup: dW1 | db1 | db2 | db3 | dW4 | db4 | loss
constexpr int S_W1 = 0, S_B1 = S_W1 + NP_W1, S_B2 = S_B1 + 512, S_B3 = S_B2 + 512,
              S_W4 = S_B3 + 256, S_B4 = S_W4 + NP_W4, S_LOSS = S_B4 + 4, SLAB_R = S_LOSS + 4;
// k_dense_wgrad: dW2 (4 x 4 blocks of 128 x 128) + dW3 (2 x 4), each over NSPLIT row ranges
constexpr int WG_BLK = 128, WG_KC = 16, WG_TILES = 16 + 8;
// row ranges of the weight-gradient GEMMs (runtime: G2048_DENSE_NSPLIT for tuning, at most
// MAX_NSPLIT, which sizes the workspace)
constexpr int NSPLIT_DEFAULT = 10, MAX_NSPLIT = 16;
constexpr int PART = NP_W2 + NP_W3;  // one split's partial dW2 | dW3

template <typename T>
struct RowArgs {
    DenseNet<T> net;
    const uint4* s;  // replay ring sections
    const uint8_t *a, *d;
    const int32_t* r;
    const int64_t* idx;     // [B] sampled rows
    const T *q2on, *q2tg;   // [B][4]
    float gamma;
    int double_dqn;
    int64_t batch;
    T* y_out;               // [B]
    T *h1, *h2, *z2, *z3;   // [B][512], [B][512], [B][512], [B][256]
    T* slab;                // [grid][SLAB_R]
};

template <typename T>
struct alignas(16) RowSmem {
    T x[TR * stride_of<T>(16)];
    T h[TR * stride_of<T>(H1)];
    T q[TR * 4];
    T y[TR];
    T dq[TR];
    T part[2 * H3];         // b3 column-sum halves
    T loss[64];
    int act[TR];
    uint16_t m1[TR * (H1 / 16)], m2[TR * (H2 / 16)];
};

// A forward layer of k_dense_rows: layer() plus the stores the backward needs -- the output rows
// < nb to gout [B][N] (row b0 + r), and relu'(z) as bits in mask (u16 per row and 16 columns)
template <typename T, int K, int N, int SI, int SO, bool kInPlace>
__device__ __forceinline__ void layer_st(const T* in, T* out, const T* __restrict__ W,
                                         const T* __restrict__ bias, T* gout, uint16_t* mask,
                                         int64_t b0, int nb) {
    typedef typename Acc<T>::type AccT;
    constexpr int RB = TR / 16, CB = N / (16 * NW), E = run_of<T, K>(), NQ = K / (4 * E);
    const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lk = l >> 4;
    AccT acc[RB][CB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[rb][c] = AccT{0, 0, 0, 0};
    const T* wr = W + (size_t)(w * CB * 16 + lr) * K + E * lk;
    const T* ar = in + lr * SI + E * lk;
    T bq[2][CB][E];
#pragma unroll
    for (int c = 0; c < CB; ++c) ldE<E>(wr + (size_t)c * 16 * K, bq[0][c]);
    auto run = [&](int q, T (&cur)[CB][E], T (&nxt)[CB][E]) {
        if (q + 1 < NQ) {
#pragma unroll
            for (int c = 0; c < CB; ++c) ldE<E>(wr + (size_t)c * 16 * K + 4 * E * (q + 1), nxt[c]);
        }
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
    if constexpr (NQ == 1) {
        run(0, bq[0], bq[1]);
    } else {
#pragma unroll 1
        for (int q = 0; q < NQ; q += 2) {
            run(q, bq[0], bq[1]);
            run(q + 1, bq[1], bq[0]);
        }
    }
    if constexpr (kInPlace) __syncthreads();
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int blk = w * CB + c, j = blk * 16 + lr;
        const T bj = bias[j];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rb * 16 + Acc<T>::row(l, r);
                const T z = acc[rb][c][r] + bj;
                const T v = z > T(0) ? z : T(0);
                out[row * SO + j] = v;
                if (gout && row < nb) gout[(b0 + row) * N + j] = v;
                if (mask) {
                    const uint64_t bal = __ballot(z > T(0));
                    if (lr == 0) mask[row * (N / 16) + blk] = (uint16_t)(bal >> (16 * lk));
                }
            }
    }
    __syncthreads();
}

// A backward layer: out[r][k] = relu'(h_l)[r][k] * sum_j in[r][j] W[j][k] (W row-major [K][N]:
// the forward's weight, whose rows are the contraction here, so a B fragment is 16 consecutive
// elements of a weight row per four lanes); the output rows < nb also go to gout [B][N] (null:
// not stored), and every lane adds its outputs into cs[c] (the bias gradient's column sums).
template <typename T, int K, int N, int SI, int SO, bool kInPlace>
__device__ __forceinline__ void layer_bwd(const T* in, T* out, const T* __restrict__ W,
                                          const uint16_t* mask, T* gout, int64_t b0, int nb,
                                          T (&cs)[N / (16 * NW)]) {
    typedef typename Acc<T>::type AccT;
    constexpr int RB = TR / 16, CB = N / (16 * NW), NS = K / 4;
    const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lk = l >> 4;
    AccT acc[RB][CB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[rb][c] = AccT{0, 0, 0, 0};
    const T* wr = W + (size_t)lk * N + w * CB * 16 + lr;  // + 4 s N + 16 c
    const T* ar = in + lr * SI + lk;                        // + rb 16 SI + 4 s
    T bq[3][CB];
    auto ldb = [&](T (&b)[CB], int s) {
#pragma unroll
        for (int c = 0; c < CB; ++c) b[c] = wr[(size_t)4 * s * N + 16 * c];
    };
    ldb(bq[0], 0);
    ldb(bq[1], 1);
    auto step = [&](int s, T (&cur)[CB], T (&nx2)[CB]) {
        if (s + 2 < NS) ldb(nx2, s + 2);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const T av = ar[rb * 16 * SI + 4 * s];
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[rb][c] = Acc<T>::mfma(av, cur[c], acc[rb][c]);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    static_assert(NS % 3 == 1 || NS % 3 == 2 || NS % 3 == 0, "steps");
#pragma unroll 1
    for (int s = 0; s + 3 <= NS; s += 3) {
        step(s, bq[0], bq[2]);
        step(s + 1, bq[1], bq[0]);
        step(s + 2, bq[2], bq[1]);
    }
    if constexpr (NS % 3 >= 1) step(NS - NS % 3, bq[0], bq[2]);
    if constexpr (NS % 3 == 2) step(NS - 1, bq[1], bq[0]);
    if constexpr (kInPlace) __syncthreads();
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int blk = w * CB + c, j = blk * 16 + lr;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rb * 16 + Acc<T>::row(l, r);
                const bool m = (mask[row * (N / 16) + blk] >> lr) & 1u;
                const T v = m ? acc[rb][c][r] : T(0);
                out[row * SO + j] = v;
                if (gout && row < nb) gout[(b0 + row) * N + j] = v;
                cs[c] += v;
            }
    }
    __syncthreads();
}

__device__ __forceinline__ int64_t sample_row_d(int64_t b, unsigned long long ep,
                                                unsigned long long count, uint32_t lo, uint32_t hi) {
    const uint4 u = g2048::philox10(
        make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32), (uint32_t)ep,
                   (uint32_t)(ep >> 32) | (g2048::DOMAIN_SAMPLE << 30)),
        lo, hi);
    return (int64_t)__umul64hi(((unsigned long long)u.y << 32) | u.x, count);
}

struct SampleArgs {
    const int64_t* idx_in;
    int64_t* idx_out;
    int64_t batch;
    const unsigned long long* count;
    const unsigned long long* step;
    unsigned long long* step_next;
    uint32_t seed_lo, seed_hi;
};

__global__ __launch_bounds__(256) void k_dense_sample(SampleArgs A) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const unsigned long long ep = *A.step;
    if (b == 0) *A.step_next = ep + 1ull;
    if (b >= A.batch) return;
    A.idx_out[b] = A.idx_in ? A.idx_in[b] : sample_row_d(b, ep, *A.count, A.seed_lo, A.seed_hi);
}

// one tile per workgroup (grid = the batch's tiles), so no accumulator lives across tiles: every
// per-tile gradient term goes to the workgroup's slab as soon as it is complete
template <typename T>
__global__ __launch_bounds__(NT) void k_dense_rows(RowArgs<T> A) {
    __shared__ RowSmem<T> S;
    constexpr int SX = stride_of<T>(16), SH = stride_of<T>(H1);
    constexpr int CB2 = H2 / (16 * NW), CB1 = H1 / (16 * NW);
    const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lk = l >> 4;
    typedef typename Acc<T>::type AccT;
    const int64_t b0 = (int64_t)blockIdx.x * TR;
    const int nb = A.batch - b0 < TR ? (int)(A.batch - b0) : TR;
    T* sl = A.slab + (int64_t)blockIdx.x * SLAB_R;
    if (t < TR) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        int act = -1;
        T yv = T(0);
        if (t < nb) {
            const int64_t b = b0 + t, row = A.idx[b];
            v = A.s[row];
            act = A.a[row];
            const T* qo = A.q2on + b * 4;
            const T* qt = A.q2tg + b * 4;
            T next;
            if (A.double_dqn)
                next = qt[g2048::argmax4_torch(qo[0], qo[1], qo[2], qo[3])];
            else
                next = g2048::qmax4_torch(qt[0], qt[1], qt[2], qt[3]);
            const float disc = (float)(1 - (int)A.d[row]) * A.gamma;
            {
#pragma clang fp contract(off)
                yv = (T)A.r[row] + (T)disc * next;
            }
            A.y_out[b] = yv;
        }
        put_row(S.x + t * SX, v);
        S.act[t] = act;
        S.y[t] = yv;
    }
    __syncthreads();
    layer_st<T, 16, H1, SX, SH, false>(S.x, S.h, A.net.w1, A.net.b1, A.h1, S.m1, b0, nb);
    layer_st<T, H1, H2, SH, SH, true>(S.h, S.h, A.net.w2, A.net.b2, A.h2, S.m2, b0, nb);
    layer_st<T, H2, H3, SH, SH, true>(S.h, S.h, A.net.w3, A.net.b3, nullptr, nullptr, b0, nb);
    {  // Q (Linear(256, 4) on VALU, forward_tile's order) -> S.q
        constexpr int PARTS = NT / (TR * 4), NPP = H3 / PARTS;
        const int part = t % PARTS, a = (t / PARTS) & 3, b = t / (4 * PARTS);
        const T* hr = S.h + b * SH + NPP * part;
        const T* wr = A.net.w4 + a * H3 + NPP * part;
        T e = T(0), o = T(0);
#pragma unroll 8
        for (int k = 0; k < NPP; k += 2) {
            e = fma(wr[k], hr[k], e);
            o = fma(wr[k + 1], hr[k + 1], o);
        }
        T v = e + o;
#pragma unroll
        for (int m = 1; m < PARTS; m *= 2) v = v + __shfl_xor(v, m);
        if (part == 0) S.q[b * 4 + a] = v + A.net.b4[a];
    }
    __syncthreads();
    if (t < TR) {  // MSE(sum): dq = 2 (q[a] - y)
        T dq = T(0), ls = T(0);
        const int act = S.act[t];
        if (act >= 0) {
#pragma clang fp contract(off)
            const T e = S.q[t * 4 + act] - S.y[t];
            dq = T(2) * e;
            ls = e * e;
        }
        S.dq[t] = dq;
        S.loss[t] = ls;
    }
    __syncthreads();
    {  // dW4[a][k0, k0 + 1], db4[a] over the tile's rows (h3 in S.h[:, 0:256])
        const int a = t >> 7, k0 = (t & 127) * 2;
        T g4a = T(0), g4b = T(0), gb = T(0);
#pragma unroll 4
        for (int r = 0; r < TR; ++r) {
            const T g = S.act[r] == a ? S.dq[r] : T(0);
            g4a = fma(g, S.h[r * SH + k0], g4a);
            g4b = fma(g, S.h[r * SH + k0 + 1], g4b);
            gb += g;
        }
        sl[S_W4 + a * H3 + k0] = g4a;
        sl[S_W4 + a * H3 + k0 + 1] = g4b;
        if (k0 == 0) sl[S_B4 + a] = gb;
    }
    if (t == 0) {
        T v = T(0);
        for (int i = 0; i < TR; ++i) v += S.loss[i];
        sl[S_LOSS] = v;
    }
    // dZ3 = dq W4[a] relu'(h3), over h3 in place: thread (column j, half h of the rows)
    {
        const int j = t & (H3 - 1), h = t >> 8;
        T z3v[TR / 2];
#pragma unroll
        for (int i = 0; i < TR / 2; ++i) {
            const int r = h * (TR / 2) + i, act = S.act[r];
            const T hv = S.h[r * SH + j];
            z3v[i] = (act >= 0 && hv > T(0)) ? S.dq[r] * A.net.w4[act * H3 + j] : T(0);
        }
        __syncthreads();  // every read of h3 done
        T cs = T(0);
#pragma unroll
        for (int i = 0; i < TR / 2; ++i) {
            const int r = h * (TR / 2) + i;
            S.h[r * SH + j] = z3v[i];
            if (r < nb) A.z3[(b0 + r) * H3 + j] = z3v[i];
            cs += z3v[i];
        }
        S.part[t] = cs;  // t = h * 256 + j
    }
    __syncthreads();
    if (t < H3) sl[S_B3 + t] = S.part[t] + S.part[H3 + t];
    // column sums of a backward layer's output: a lane holds its rows' sums of the columns
    // (w CB + c) 16 + lr; the four lane groups lk are added in a fixed tree (xor 16, then 32)
    auto colsums = [&](auto& cs, int off) {
        constexpr int CB = sizeof(cs) / sizeof(cs[0]);
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            T v = cs[c];
            v = v + __shfl_xor(v, 16);
            v = v + __shfl_xor(v, 32);
            if (lk == 0) sl[off + (w * CB + c) * 16 + lr] = v;
        }
    };
    {
        T cs2[CB2];
#pragma unroll
        for (int c = 0; c < CB2; ++c) cs2[c] = T(0);
        layer_bwd<T, H3, H2, SH, SH, true>(S.h, S.h, A.net.w3, S.m2, A.z2, b0, nb, cs2);
        colsums(cs2, S_B2);
    }
    {
        T cs1[CB1];
#pragma unroll
        for (int c = 0; c < CB1; ++c) cs1[c] = T(0);
        layer_bwd<T, H2, H1, SH, SH, true>(S.h, S.h, A.net.w2, S.m1, nullptr, b0, nb, cs1);
        colsums(cs1, S_B1);
    }
    // dW1 = dZ1^T X over the tile's rows: M = j (wave w: 16-row blocks 4w .. 4w+3), N = the 16
    // cells, K = rows
    AccT gw1[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) gw1[mt] = AccT{0, 0, 0, 0};
#pragma unroll
    for (int s4 = 0; s4 < TR / 4; ++s4) {
        const T bx = S.x[(4 * s4 + lk) * SX + lr];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            const T az = S.h[(4 * s4 + lk) * SH + 16 * (4 * w + mt) + lr];
            gw1[mt] = Acc<T>::mfma(az, bx, gw1[mt]);
        }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            sl[S_W1 + (16 * (4 * w + mt) + Acc<T>::row(l, r)) * 16 + lr] = gw1[mt][r];
}

// dW2 = dZ2^T H1 and dW3 = dZ3^T H2 over one row range: workgroup -> (tile, split); wave w ->
// rows 32 (w & 3) .. of the 128 x 128 block (two 16-row MFMA blocks), columns 64 (w >> 2) ..
// (four), operands staged through LDS in chunks of WG_KC batch rows, the next chunk's global
// loads in flight while the current one is multiplied.
template <typename T>
struct WgradArgs {
    const T *z2, *h1, *z3, *h2;
    int64_t batch, rows_per_split;
    T* part;  // [nsplit][PART]
};

template <typename T>
__global__ __launch_bounds__(NT) void k_dense_wgrad(WgradArgs<T> A) {
    typedef typename Acc<T>::type AccT;
    constexpr int LS = WG_BLK + (sizeof(T) == 4 ? 4 : 2);  // LDS row stride
    __shared__ __attribute__((aligned(16))) T As[2][WG_KC * LS];
    __shared__ __attribute__((aligned(16))) T Bs[2][WG_KC * LS];
    const int t = threadIdx.x, l = t & 63, w = t >> 6, lr = l & 15, lk = l >> 4;
    const int tile = blockIdx.x % WG_TILES, split = blockIdx.x / WG_TILES;
    // tile -> (matrix, 128-row block of M, 128-column block of N)
    const bool w2 = tile < 16;
    const int mblk = w2 ? tile >> 2 : (tile - 16) >> 2, nblk = tile & 3;
    const T* Az = w2 ? A.z2 : A.z3;
    const T* Bh = w2 ? A.h1 : A.h2;
    const int M = w2 ? 512 : 256, N = 512;
    const int64_t r0 = (int64_t)split * A.rows_per_split;
    const int64_t r1 = r0 + A.rows_per_split < A.batch ? r0 + A.rows_per_split : A.batch;
    // each thread stages 4 consecutive elements of one chunk row of A and of B
    const int lrow = t >> 5, lcol = (t & 31) * 4;
    T ra[4], rbv[4];
    auto gload = [&](int64_t c0) {
        const int64_t row = c0 + lrow;
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[e] = rbv[e] = T(0);
        if (row < r1) {
            const T* pa = Az + row * M + mblk * WG_BLK + lcol;
            const T* pb = Bh + row * N + nblk * WG_BLK + lcol;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                ra[e] = pa[e];
                rbv[e] = pb[e];
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            As[buf][lrow * LS + lcol + e] = ra[e];
            Bs[buf][lrow * LS + lcol + e] = rbv[e];
        }
    };
    AccT acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = AccT{0, 0, 0, 0};
    const int m0 = 32 * (w & 3), n0 = 64 * (w >> 2);
    int buf = 0;
    if (r0 < r1) {
        gload(r0);
        lstore(0);
    }
    __syncthreads();
    for (int64_t c0 = r0; c0 < r1; c0 += WG_KC) {
        const bool more = c0 + WG_KC < r1;
        if (more) gload(c0 + WG_KC);
#pragma unroll
        for (int ks = 0; ks < WG_KC / 4; ++ks) {
            const int kr = 4 * ks + lk;
            T av[2], bv[4];
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i] = As[buf][kr * LS + m0 + 16 * i + lr];
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = Bs[buf][kr * LS + n0 + 16 * j + lr];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = Acc<T>::mfma(av[i], bv[j], acc[i][j]);
        }
        if (more) {
            lstore(buf ^ 1);
            buf ^= 1;
        }
        __syncthreads();
    }
    T* out = A.part + (int64_t)split * PART + (w2 ? 0 : NP_W2);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mblk * WG_BLK + m0 + 16 * i + Acc<T>::row(l, r);
                const int n = nblk * WG_BLK + n0 + 16 * j + lr;
                out[(int64_t)m * N + n] = acc[i][j][r];
            }
}

// The gradient in torch order (w1 b1 w2 b2 w3 b3 w4 b4) from k_dense_rows' slabs (fixed slab
// order) and k_dense_wgrad's partials (fixed split order), then Adam (+ target sync).  Blocks
// [0, NB_SLABP): 64 slab-sourced parameters each, wave v summing slabs v, v + 8, ... and the eight
// wave partials added in wave order; the other blocks: one partial-sourced parameter per thread.
constexpr int N_SLABP = NP_W1 + 512 + 512 + 256 + NP_W4 + 4;  // + the loss
constexpr int NB_SLABP = (N_SLABP + 1 + 63) / 64;

template <typename T>
struct DRedArgs {
    const T* slab;
    int nslab;
    const T* part;
    int nsplit;
    T* p[8];   // online parameters (torch order)
    T* tp[8];  // target parameters
    T* grad;   // [P_ALL] (nullable)
    T* loss;   // (nullable)
    T *m, *v;  // Adam state (null: gradient only)
    double lr, b1, b2, eps;
    unsigned long long sync_every;
    const unsigned long long* step_next;
    unsigned long long* step;
};

// slab offset of the i-th slab-sourced parameter (w1, b1, b2, b3, w4, b4 in that order; then the
// loss), and its torch-order index
__device__ __forceinline__ void slab_param(int i, int& soff, int& pidx) {
    if (i < NP_W1) { soff = S_W1 + i; pidx = P_W1 + i; return; }
    i -= NP_W1;
    if (i < 512) { soff = S_B1 + i; pidx = P_B1 + i; return; }
    i -= 512;
    if (i < 512) { soff = S_B2 + i; pidx = P_B2 + i; return; }
    i -= 512;
    if (i < 256) { soff = S_B3 + i; pidx = P_B3 + i; return; }
    i -= 256;
    if (i < NP_W4) { soff = S_W4 + i; pidx = P_W4 + i; return; }
    i -= NP_W4;
    if (i < 4) { soff = S_B4 + i; pidx = P_B4 + i; return; }
    soff = S_LOSS;
    pidx = -1;  // the loss
}

template <typename T>
__device__ __forceinline__ void dense_apply(const DRedArgs<T>& A, int pidx, T g,
                                            unsigned long long t) {
    if (A.grad) A.grad[pidx] = g;
    if (!A.m) return;
    int k = 0;
    const int ends[8] = {P_B1, P_W2, P_B2, P_W3, P_B3, P_W4, P_B4, P_ALL};
#pragma unroll
    for (int j = 0; j < 7; ++j) k += pidx >= ends[j] ? 1 : 0;
    const int begins[8] = {P_W1, P_B1, P_W2, P_B2, P_W3, P_B3, P_W4, P_B4};
    T* p = A.p[k] + (pidx - begins[k]);
    T np;
    if constexpr (sizeof(T) == 8) {
        double m = A.m[pidx], v = A.v[pidx];
        np = g2048::adam64((double)t, A.lr, A.b1, A.b2, A.eps, g, m, v, *p);
        A.m[pidx] = m;
        A.v[pidx] = v;
    } else {
        const g2048::AdamCoef c = g2048::adam_coef((double)t, A.lr, A.b1, A.b2, A.eps);
        np = g2048::adam_apply(c, g, A.m + pidx, A.v + pidx, *p);
    }
    *p = np;
    if (A.sync_every && t % A.sync_every == 0ull) A.tp[k][pidx - begins[k]] = np;
}

template <typename T>
__global__ __launch_bounds__(NT) void k_dense_reduce(DRedArgs<T> A) {
    __shared__ T red[NW][64];
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    // the update counter (sampler epoch, Adam's t) is committed here with or without Adam (a
    // data-parallel step reads it as t after the all-reduce); every block reads step_next
    const unsigned long long tt = *A.step_next;
    if (blockIdx.x == 0 && t == 0) *A.step = tt;
    if ((int)blockIdx.x < NB_SLABP) {
        const int i = blockIdx.x * 64 + l;
        int soff = 0, pidx = 0;
        if (i <= N_SLABP) slab_param(i, soff, pidx);
        T acc = T(0);
        if (i <= N_SLABP) {
            const T* p = A.slab + soff;
            int g = w;
            for (; g + 8 * 3 < A.nslab; g += 8 * 4) {  // four loads in flight, ascending order
                const T v0 = p[(int64_t)g * SLAB_R], v1 = p[(int64_t)(g + 8) * SLAB_R];
                const T v2 = p[(int64_t)(g + 16) * SLAB_R], v3 = p[(int64_t)(g + 24) * SLAB_R];
                acc = acc + v0;
                acc = acc + v1;
                acc = acc + v2;
                acc = acc + v3;
            }
            for (; g < A.nslab; g += 8) acc = acc + p[(int64_t)g * SLAB_R];
        }
        red[w][l] = acc;
        __syncthreads();
        if (w == 0 && i <= N_SLABP) {
            T s = red[0][l];
#pragma unroll
            for (int v = 1; v < NW; ++v) s = s + red[v][l];
            if (pidx < 0) {
                if (A.loss) *A.loss = s;
            } else {
                dense_apply(A, pidx, s, tt);
            }
        }
        return;
    }
    const int64_t i = (int64_t)(blockIdx.x - NB_SLABP) * NT + t;  // index into dW2 | dW3
    if (i >= PART) return;
    T acc = T(0);
    const T* p = A.part + i;
#pragma unroll 4
    for (int s = 0; s < A.nsplit; ++s) acc = acc + p[(int64_t)s * PART];
    dense_apply(A, i < NP_W2 ? P_W2 + (int)i : P_W3 + (int)(i - NP_W2), acc, tt);
}

template <typename T>
int64_t update_workspace_elems(int64_t batch) {
    const int64_t grid = (batch + TR - 1) / TR;  // k_dense_rows: one tile per workgroup
    // q2on | q2tg | step word (32) | h1 | h2 | z2 | z3 | slabs | partials
    return 8 * batch + 32 + batch * (512 + 512 + 512 + 256) + grid * SLAB_R +
           (int64_t)MAX_NSPLIT * PART;
}

template <typename T>
int update_launch(const g2048_densenet_params* on, const g2048_densenet_params* tg,
                  g2048_replay* rb, const int64_t* idx_in, int64_t batch, uint64_t seed,
                  uint64_t* step_dev, float gamma, int double_dqn, int64_t* idx_out, T* y_out,
                  T* ws, T* grad_out, T* loss_out, T* m, T* v, double lr, double b1, double b2,
                  double eps, uint64_t sync_every, hipStream_t st) {
    uint8_t *s = nullptr, *s2 = nullptr, *a = nullptr, *d = nullptr;
    int32_t* r = nullptr;
    uint64_t* count = nullptr;
    if (g2048_replay_views(rb, &s, &s2, &a, &r, &d, &count) != G2048_OK) return G2048_EINVAL;
    T* q2on = ws;
    T* q2tg = q2on + 4 * batch;
    unsigned long long* step_next = reinterpret_cast<unsigned long long*>(q2tg + 4 * batch);
    T* h1 = q2tg + 4 * batch + 32;
    T* h2 = h1 + batch * 512;
    T* z2 = h2 + batch * 512;
    T* z3 = z2 + batch * 512;
    T* slab = z3 + batch * 256;
    const int grid = (int)((batch + TR - 1) / TR);  // k_dense_rows: one tile per workgroup
    T* part = slab + (int64_t)grid * SLAB_R;

    SampleArgs SA{idx_in, idx_out, batch, reinterpret_cast<const unsigned long long*>(count),
                  reinterpret_cast<const unsigned long long*>(step_dev), step_next,
                  (uint32_t)seed, (uint32_t)(seed >> 32)};
    hipLaunchKernelGGL(k_dense_sample, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, st, SA);
    // the target-side forwards on the sampled s' rows (the rollout forward kernel).  Double DQN:
    // Q_online(s') and Q_target(s') in ONE launch, half the workgroups per net, each on
    // tile_rows<T>() rows (64 in float32): every workgroup streams one net's weights through L2
    // for twice the rows of the 32-row tiles two launches needed to fill the CUs, so the weight
    // traffic per row halves.  Vanilla DQN: Q_target(s') alone, 32-row tiles over every CU.
    {
        FwdArgs<T> F{};
        F.rows = reinterpret_cast<const uint4*>(s2);
        F.idx = idx_out;
        F.n = batch;
        if (double_dqn) {
            constexpr int TBM = tile_rows<T>();
            F.net = net_of<T>(on);
            F.q = q2on;
            F.net2 = net_of<T>(tg);
            F.q2 = q2tg;
            const int64_t ft = (batch + TBM - 1) / TBM;
            int g1 = (int)(ft < MAX_WG ? ft : MAX_WG);
            F.chunk = (batch + g1 - 1) / g1;
            // 2 g1 workgroups of one TBM-row tile each would fill the CUs one and a fraction
            // times (f64, 4096 < B <= 6144; B = 5000: 314 tiles on 256 CUs, the second round 58
            // tiles deep): half the CUs per net instead, each on a TBM-row tile plus a <= 16-row
            // remainder tile (k_dense_forward), one round
            const char* nos = getenv("G2048_DENSE_FWD_ONE_TILE");  // 1: round 5's layout (A/B)
            if (TBM == 32 && 2 * ft > MAX_WG && 2 * ft < 2 * MAX_WG && !(nos && nos[0] == '1')) {
                const int64_t ch = (batch + MAX_WG / 2 - 1) / (MAX_WG / 2);
                if (ch <= TBM + 16) {
                    g1 = MAX_WG / 2;
                    F.chunk = ch;
                }
            }
            F.nb1 = g1;
            hipLaunchKernelGGL((k_dense_forward<T, TBM>), dim3(2 * g1), dim3(NT), 0, st, F);
        } else {
            F.net = net_of<T>(tg);
            F.q = q2tg;
            const int64_t ft = (batch + TR - 1) / TR;
            const int fg = (int)(ft < MAX_WG ? ft : MAX_WG);
            F.chunk = (batch + fg - 1) / fg;
            hipLaunchKernelGGL((k_dense_forward<T, TR>), dim3(fg), dim3(NT), 0, st, F);
        }
    }
    RowArgs<T> R{};
    R.net = net_of<T>(on);
    R.s = reinterpret_cast<const uint4*>(s);
    R.a = a;
    R.d = d;
    R.r = r;
    R.idx = idx_out;
    R.q2on = q2on;
    R.q2tg = q2tg;
    R.gamma = gamma;
    R.double_dqn = double_dqn;
    R.batch = batch;
    R.y_out = y_out;
    R.h1 = h1;
    R.h2 = h2;
    R.z2 = z2;
    R.z3 = z3;
    R.slab = slab;
    hipLaunchKernelGGL(k_dense_rows<T>, dim3(grid), dim3(NT), 0, st, R);
    int nsplit = NSPLIT_DEFAULT;
    if (const char* e = getenv("G2048_DENSE_NSPLIT")) {
        const int v = atoi(e);
        if (v >= 1 && v <= MAX_NSPLIT) nsplit = v;
    }
    WgradArgs<T> WG{z2, h1, z3, h2, batch, 0, part};
    WG.rows_per_split = ((batch + nsplit - 1) / nsplit + WG_KC - 1) / WG_KC * WG_KC;
    hipLaunchKernelGGL(k_dense_wgrad<T>, dim3(WG_TILES * nsplit), dim3(NT), 0, st, WG);
    DRedArgs<T> D{};
    D.slab = slab;
    D.nslab = grid;
    D.part = part;
    D.nsplit = nsplit;
    const void* ps[8] = {on->w1, on->b1, on->w2, on->b2, on->w3, on->b3, on->w4, on->b4};
    const void* ts[8] = {tg->w1, tg->b1, tg->w2, tg->b2, tg->w3, tg->b3, tg->w4, tg->b4};
    for (int k = 0; k < 8; ++k) {
        D.p[k] = const_cast<T*>(static_cast<const T*>(ps[k]));
        D.tp[k] = const_cast<T*>(static_cast<const T*>(ts[k]));
    }
    D.grad = grad_out;
    D.loss = loss_out;
    D.m = m;
    D.v = v;
    D.lr = lr;
    D.b1 = b1;
    D.b2 = b2;
    D.eps = eps;
    D.sync_every = m ? sync_every : 0ull;
    D.step_next = step_next;
    D.step = reinterpret_cast<unsigned long long*>(step_dev);
    const int nb_part = (PART + NT - 1) / NT;
    hipLaunchKernelGGL(k_dense_reduce<T>, dim3(NB_SLABP + nb_part), dim3(NT), 0, st, D);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "densenet_update: %s", hipGetErrorString(e));
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

extern "C" G2048_API int64_t g2048_densenet_update_workspace(int64_t batch, int dtype) {
    if (batch <= 0 || (dtype != G2048_F32 && dtype != G2048_F64)) return 0;
    return dtype == G2048_F32 ? update_workspace_elems<float>(batch)
                              : update_workspace_elems<double>(batch);
}

extern "C" G2048_API int g2048_densenet_update(
    const g2048_densenet_params* online, const g2048_densenet_params* target, int dtype,
    g2048_replay* rb, const int64_t* idx_in, int64_t batch, uint64_t seed, uint64_t* step_dev,
    float gamma, int double_dqn, int64_t* idx_out, void* y_out, void* workspace, void* grad_out,
    void* loss_out, void* exp_avg, void* exp_avg_sq, double lr, double beta1, double beta2,
    double eps, uint64_t sync_every, void* stream) {
    if (!params_ok(online) || !params_ok(target) || !rb || batch <= 0 || !step_dev || !idx_out ||
        !y_out || !workspace || (dtype != G2048_F32 && dtype != G2048_F64))
        return g2048_fail(G2048_EINVAL, "densenet_update: NULL argument, batch <= 0 or bad dtype");
    if (batch > INT32_MAX) return g2048_fail(G2048_EINVAL, "densenet_update: batch > 2^31 - 1");
    const bool adam = exp_avg && exp_avg_sq;
    if (!adam && !grad_out)
        return g2048_fail(G2048_EINVAL,
                          "densenet_update: need exp_avg and exp_avg_sq (Adam) or grad_out");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (dtype == G2048_F32)
        return update_launch<float>(online, target, rb, idx_in, batch, seed, step_dev, gamma,
                                    double_dqn, idx_out, static_cast<float*>(y_out),
                                    static_cast<float*>(workspace), static_cast<float*>(grad_out),
                                    static_cast<float*>(loss_out), static_cast<float*>(exp_avg),
                                    static_cast<float*>(exp_avg_sq), lr, beta1, beta2, eps,
                                    sync_every, st);
    return update_launch<double>(online, target, rb, idx_in, batch, seed, step_dev, gamma,
                                 double_dqn, idx_out, static_cast<double*>(y_out),
                                 static_cast<double*>(workspace), static_cast<double*>(grad_out),
                                 static_cast<double*>(loss_out), static_cast<double*>(exp_avg),
                                 static_cast<double*>(exp_avg_sq), lr, beta1, beta2, eps,
                                 sync_every, st);
}
