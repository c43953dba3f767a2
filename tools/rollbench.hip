// rollbench.hip -- cost components of the K-steps-per-launch random rollout (k_rollout) on gfx950.
// Standalone (hipcc, no torch): the same per-step board arithmetic as g2048_board.hpp with parts
// switched off by template flags, timed with hipEvents at 64k and 1k boards, K = 64.
//   F_PHILOX  Philox4x32-10 block per step (else a 3-op counter hash)
//   F_HALF    one Philox block per TWO steps (words x,z for even steps, y,w for odd)
//   F_STORE   ring append (s, s', a, r, d) per step (else one checksum store at the end)
//   F_BOARD   legal mask + move + spawn + reset (else the board is only xor-ed with the draw)
//   F_SOFF    ring offsets uniform (row * n scalar + lane constant) instead of per-lane t % rows
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rollbench tools/rollbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../reinforcement-learning-2048_amd/csrc/g2048_board.hpp"

using namespace g2048;

enum { F_PHILOX = 1, F_STORE = 2, F_BOARD = 4, F_SOFF = 8, F_HALF = 16 };

struct Ring {
    uint4* s;
    uint4* s2;
    uint8_t* a;
    int32_t* r;
    uint8_t* d;
    uint32_t rows;
};

template <int F>
__global__ __launch_bounds__(256) void k_roll(uint4* board, uint4* meta, int64_t n, Ring R, int K,
                                              uint32_t seed_lo, uint32_t seed_hi,
                                              uint32_t* sink) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = board[i];
    Board b{v.x, v.y, v.z, v.w};
    uint4 m = meta[i];
    uint64_t t = (uint64_t)m.z | ((uint64_t)m.w << 32);
    const uint64_t gid = (uint64_t)i;
    uint32_t acc = 0;
    // uniform ring row (F_SOFF): every board of the env shares t
    uint32_t row = __builtin_amdgcn_readfirstlane((uint32_t)t) % R.rows;
    uint4 hold = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < K; ++s) {
        uint4 u;
        if constexpr (F & F_HALF) {
            if ((s & 1) == 0) hold = draw(seed_lo, seed_hi, gid, DOMAIN_STEP, t >> 1);
            u = (s & 1) ? make_uint4(hold.y, hold.w, hold.y << 16, hold.w << 16)
                        : make_uint4(hold.x, hold.z, hold.x << 16, hold.z << 16);
        } else if constexpr (F & F_PHILOX) {
            u = draw(seed_lo, seed_hi, gid, DOMAIN_STEP, t);
        } else {
            const uint32_t h = ((uint32_t)t * 0x9E3779B9u) ^ ((uint32_t)gid * 0x85EBCA6Bu);
            u = make_uint4(h, h * 3u, h ^ 0x5bd1e995u, h + 0x27d4eb2fu);
        }
        const Board s_old = b;
        uint32_t r = 0, done = 0;
        const uint32_t act = u.x >> 30;
        if constexpr (F & F_BOARD) {
            const uint32_t legal = legal_mask(b);
            done = legal == 0u;
            if (!done && ((legal >> act) & 1u)) {
                r = apply_move(b, act);
                spawn(b, u.z, u.w, 0x80000000u);
            }
            m.x += r;
            m.y += 1u;
            if (done) {
                b = fresh_board(u, 0x80000000u);
                m.x = 0u;
                m.y = 0u;
            }
        } else {
            b.r0 ^= u.x;
            b.r1 ^= u.y;
            b.r2 ^= u.z;
            b.r3 ^= u.w;
        }
        if constexpr (F & F_STORE) {
            int64_t slot;
            if constexpr (F & F_SOFF) {
                slot = (int64_t)row * n + i;
                row = row + 1u == R.rows ? 0u : row + 1u;
            } else {
                slot = (int64_t)((uint32_t)t % R.rows) * n + i;
            }
            R.s[slot] = make_uint4(s_old.r0, s_old.r1, s_old.r2, s_old.r3);
            R.s2[slot] = make_uint4(b.r0, b.r1, b.r2, b.r3);
            R.a[slot] = (uint8_t)act;
            R.r[slot] = (int32_t)r;
            R.d[slot] = (uint8_t)done;
        } else {
            acc += r + done + b.r0;
        }
        ++t;
    }
    board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    m.z = (uint32_t)t;
    m.w = (uint32_t)(t >> 32);
    meta[i] = m;
    if (!(F & F_STORE) && acc == 0x12345678u) sink[0] = acc;
}


// ---------------------------------------------------------------- candidate lean step
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}
template <bool kX3>
__device__ __forceinline__ uint4 philox_x3(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u;
        const uint64_t p1 = (uint64_t)c.z * 0xCD9E8D57u;
        if constexpr (kX3)
            c = make_uint4(xor3((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1,
                           xor3((uint32_t)(p0 >> 32), c.w, k1), (uint32_t)p0);
        else
            c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1,
                           (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
// terminal test without the 4-direction mask: full board and no equal neighbour
__device__ __forceinline__ bool is_done(const Board& b) {
    const uint32_t z = z80(b.r0) | z80(b.r1) | z80(b.r2) | z80(b.r3);
    const uint32_t H = z80(b.r0 ^ (b.r0 >> 8)) | z80(b.r1 ^ (b.r1 >> 8)) |
                       z80(b.r2 ^ (b.r2 >> 8)) | z80(b.r3 ^ (b.r3 >> 8));
    const uint32_t V = z80(b.r0 ^ b.r1) | z80(b.r1 ^ b.r2) | z80(b.r2 ^ b.r3);
    return (z | (H & 0x00808080u) | V) == 0u;
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
enum { N_X3 = 1, N_DONE = 2, N_BUF = 4, N_HALF = 8 };

template <int F>
__global__ __launch_bounds__(256) void k_new(uint4* board, uint4* meta, int64_t n, Ring R, int K,
                                             uint32_t seed_lo, uint32_t seed_hi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = board[i];
    Board b{v.x, v.y, v.z, v.w};
    uint4 m = meta[i];
    const uint32_t t0 = __builtin_amdgcn_readfirstlane(m.z);
    const uint32_t gid_lo = (uint32_t)i, gid_hi = (uint32_t)((uint64_t)i >> 32);
    uint32_t row = t0 % R.rows;
    const uint32_t nn = (uint32_t)n;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(R.s, 0, (int)(16u * nn * R.rows), 0x00020000);
    const auto rs2 = __builtin_amdgcn_make_buffer_rsrc(R.s2, 0, (int)(16u * nn * R.rows), 0x00020000);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(R.a, 0, (int)(nn * R.rows), 0x00020000);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(R.r, 0, (int)(4u * nn * R.rows), 0x00020000);
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(R.d, 0, (int)(nn * R.rows), 0x00020000);
    uint4 hold = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < K; ++s) {
        const uint32_t t = t0 + (uint32_t)s;
        uint32_t wa, wb;
        if constexpr (F & N_HALF) {
            if ((t & 1u) == 0u || s == 0)
                hold = philox_x3<(F & N_X3) != 0>(make_uint4(t >> 1, 0u, gid_lo, gid_hi | (1u << 30)),
                                                  seed_lo, seed_hi);
            wa = (t & 1u) ? hold.z : hold.x;
            wb = (t & 1u) ? hold.w : hold.y;
        } else {
            hold = philox_x3<(F & N_X3) != 0>(make_uint4(t, 0u, gid_lo, gid_hi), seed_lo, seed_hi);
            wa = hold.x;
            wb = hold.w;
        }
        const Board s_old = b;
        const uint32_t act = wa >> 30;
        uint32_t r = 0;
        bool done;
        if constexpr (F & N_DONE) {
            Board nb = b;
            const uint32_t sc = apply_move(nb, act);
            const bool moved = ((nb.r0 ^ b.r0) | (nb.r1 ^ b.r1) | (nb.r2 ^ b.r2) | (nb.r3 ^ b.r3)) != 0u;
            done = is_done(b);
            if (moved) {
                b = nb;
                r = sc;
                spawn(b, wa << 2, wb, 0x80000000u);
            }
        } else {
            const uint32_t legal = legal_mask(b);
            done = legal == 0u;
            if (!done && ((legal >> act) & 1u)) {
                r = apply_move(b, act);
                spawn(b, wa << 2, wb, 0x80000000u);
            }
        }
        m.x += r;
        m.y += 1u;
        if constexpr (F & N_BUF) {
            const uint32_t so = row * nn;
            __builtin_amdgcn_raw_buffer_store_b128(v4u{s_old.r0, s_old.r1, s_old.r2, s_old.r3}, rs, (uint32_t)i * 16u, so * 16u, 0);
            __builtin_amdgcn_raw_buffer_store_b128(v4u{b.r0, b.r1, b.r2, b.r3}, rs2, (uint32_t)i * 16u, so * 16u, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)act, ra, (uint32_t)i, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(r, rr, (uint32_t)i * 4u, so * 4u, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)done, rd, (uint32_t)i, so, 0);
        } else {
            const int64_t slot = (int64_t)row * n + i;
            R.s[slot] = make_uint4(s_old.r0, s_old.r1, s_old.r2, s_old.r3);
            R.s2[slot] = make_uint4(b.r0, b.r1, b.r2, b.r3);
            R.a[slot] = (uint8_t)act;
            R.r[slot] = (int32_t)r;
            R.d[slot] = (uint8_t)done;
        }
        row = row + 1u == R.rows ? 0u : row + 1u;
        if (done) {
            b = fresh_board(make_uint4(wa << 2, 0u, wa, wb), 0x80000000u);
            m.x = 0u;
            m.y = 0u;
        }
    }
    board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    m.z = t0 + (uint32_t)K;
    meta[i] = m;
}

template <int F>
void run_new(const char* name, int64_t n, int K, uint4* board, uint4* meta, Ring R) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 5; ++w)
        hipLaunchKernelGGL(k_new<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u);
    const int reps = 20;
    (void)hipEventRecord(a, 0);
    for (int w = 0; w < reps; ++w)
        hipLaunchKernelGGL(k_new<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / reps;
    printf("%-28s n=%-7lld K=%d  %8.2f us/launch  %7.3f us/step  %7.1f GB/s (38 B/step)\n", name,
           (long long)n, K, us, us / K, (double)n * K * 38.0 / us * 1e-3);
}


// ---------------------------------------------------------------- lean step v2 (branch-free)
__device__ __forceinline__ void spawn_bf(Board& b, uint32_t u_cell, uint32_t u_val, uint32_t th,
                                         bool on) {
    const uint32_t z0 = z80(b.r0), z1 = z80(b.r1), z2 = z80(b.r2), z3 = z80(b.r3);
    const uint32_t p1 = __popc(z0), p2 = p1 + __popc(z1), p3 = p2 + __popc(z2);
    const uint32_t n = p3 + __popc(z3);
    uint32_t k = __umulhi(u_cell, n);
    const uint32_t row = (uint32_t)(k >= p1) + (uint32_t)(k >= p2) + (uint32_t)(k >= p3);
    uint32_t z = row == 0u ? z0 : row == 1u ? z1 : row == 2u ? z2 : z3;
    k -= row == 0u ? 0u : row == 1u ? p1 : row == 2u ? p2 : p3;
    uint32_t byte = 0;
    const uint32_t c01 = __popc(z & 0x8080u);
    if (k >= c01) { k -= c01; z >>= 16; byte = 2; }
    byte += (uint32_t)(k >= ((z >> 7) & 1u));
    set_cell(b, row * 4u + byte, on ? (u_val < th ? 2u : 1u) : 0u);
}

template <int F>
__device__ __forceinline__ void lean_step(Board& b, uint2& m, uint32_t wa, uint32_t wb,
                                          uint32_t& r_out, uint32_t& d_out, uint32_t& a_out) {
    Board nb = b;
    const uint32_t act = wa >> 30;
    const uint32_t sc = apply_move(nb, act);
    const bool moved = ((nb.r0 ^ b.r0) | (nb.r1 ^ b.r1) | (nb.r2 ^ b.r2) | (nb.r3 ^ b.r3)) != 0u;
    const bool done = is_done(b);
    if constexpr (F & 1) {
        // an unmoved board is its own slide: spawn a 0 exponent (no-op) instead of selecting
        spawn_bf(nb, wa << 2, moved ? wb : 0xFFFFFFFFu, 0x80000000u, moved);
        b = nb;
    } else {
        spawn_bf(nb, wa << 2, wb, 0x80000000u, true);
        b.r0 = moved ? nb.r0 : b.r0;
        b.r1 = moved ? nb.r1 : b.r1;
        b.r2 = moved ? nb.r2 : b.r2;
        b.r3 = moved ? nb.r3 : b.r3;
    }
    m.x += sc;
    m.y += 1u;
    r_out = sc;
    d_out = done;
    a_out = act;
}

template <int F>
__global__ __launch_bounds__(256) void k_new2(uint4* board, uint4* meta, int64_t n, Ring R, int K,
                                              uint32_t seed_lo, uint32_t seed_hi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = board[i];
    Board b{v.x, v.y, v.z, v.w};
    const uint4 m4 = meta[i];
    uint2 m = make_uint2(m4.x, m4.y);
    uint32_t t = __builtin_amdgcn_readfirstlane(m4.z) & ~1u;  // even start (experiment)
    const uint32_t gid_lo = (uint32_t)i, gid_hi = (uint32_t)((uint64_t)i >> 32);
    uint32_t row = t % R.rows;
    const uint32_t nn = (uint32_t)n;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(R.s, 0, (int)(16u * nn * R.rows), 0x00020000);
    const auto rs2 = __builtin_amdgcn_make_buffer_rsrc(R.s2, 0, (int)(16u * nn * R.rows), 0x00020000);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(R.a, 0, (int)(nn * R.rows), 0x00020000);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(R.r, 0, (int)(4u * nn * R.rows), 0x00020000);
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(R.d, 0, (int)(nn * R.rows), 0x00020000);
    const uint32_t vo16 = (uint32_t)i * 16u, vo4 = (uint32_t)i * 4u, vo1 = (uint32_t)i;
    auto emit = [&](const Board& so, uint32_t r, uint32_t d, uint32_t a) {
        const uint32_t so_ = row * nn;
        __builtin_amdgcn_raw_buffer_store_b128(v4u{so.r0, so.r1, so.r2, so.r3}, rs, vo16, so_ * 16u, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v4u{b.r0, b.r1, b.r2, b.r3}, rs2, vo16, so_ * 16u, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)a, ra, vo1, so_, 0);
        __builtin_amdgcn_raw_buffer_store_b32(r, rr, vo4, so_ * 4u, 0);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)d, rd, vo1, so_, 0);
        row = row + 1u == R.rows ? 0u : row + 1u;
    };
    auto half = [&](uint32_t wa, uint32_t wb) {
        const Board so = b;
        uint32_t r, d, a;
        lean_step<F>(b, m, wa, wb, r, d, a);
        emit(so, r, d, a);
        if constexpr (F & 4) {
            const Board fb = fresh_board(make_uint4(wa << 2, 0u, wa, wb), 0x80000000u);
            b.r0 = d ? fb.r0 : b.r0;
            b.r1 = d ? fb.r1 : b.r1;
            b.r2 = d ? fb.r2 : b.r2;
            b.r3 = d ? fb.r3 : b.r3;
            m.x = d ? 0u : m.x;
            m.y = d ? 0u : m.y;
        } else {
            if (d) {
                b = fresh_board(make_uint4(wa << 2, 0u, wa, wb), 0x80000000u);
                m = make_uint2(0u, 0u);
            }
        }
    };
    if constexpr (F & 2) {  // software-pipelined: the next pair's block under this pair's steps
        uint4 h = philox_x3<true>(make_uint4(t >> 1, 0u, gid_lo, gid_hi | (1u << 30)), seed_lo,
                                  seed_hi);
        for (int s = 0; s < K; s += 2, t += 2) {
            const uint4 hn = philox_x3<true>(
                make_uint4((t >> 1) + 1u, 0u, gid_lo, gid_hi | (1u << 30)), seed_lo, seed_hi);
            half(h.x, h.y);
            half(h.z, h.w);
            h = hn;
        }
    } else {
        for (int s = 0; s < K; s += 2, t += 2) {
            const uint4 h = philox_x3<true>(make_uint4(t >> 1, 0u, gid_lo, gid_hi | (1u << 30)),
                                            seed_lo, seed_hi);
            half(h.x, h.y);
            half(h.z, h.w);
        }
    }
    board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    meta[i] = make_uint4(m.x, m.y, t, 0u);
}

template <int F>
void run_new2(const char* name, int64_t n, int K, uint4* board, uint4* meta, Ring R) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int w = 0; w < 5; ++w)
        hipLaunchKernelGGL(k_new2<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u);
    const int reps = 20;
    (void)hipEventRecord(a, 0);
    for (int w = 0; w < reps; ++w)
        hipLaunchKernelGGL(k_new2<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / reps;
    printf("%-28s n=%-7lld K=%d  %8.2f us/launch  %7.3f us/step  %7.1f GB/s (38 B/step)\n", name,
           (long long)n, K, us, us / K, (double)n * K * 38.0 / us * 1e-3);
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

template <int F>
void run(const char* name, int64_t n, int K, uint4* board, uint4* meta, Ring R, uint32_t* sink) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 5; ++w)
        hipLaunchKernelGGL(k_roll<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u, sink);
    const int reps = 20;
    CK(hipEventRecord(a, 0));
    for (int w = 0; w < reps; ++w)
        hipLaunchKernelGGL(k_roll<F>, dim3(grid), dim3(256), 0, 0, board, meta, n, R, K, 1u, 2u, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)n * K * 38.0;
    printf("%-28s n=%-7lld K=%d  %8.2f us/launch  %7.3f us/step  %7.1f GB/s (38 B/step)\n", name,
           (long long)n, K, us, us / K, bytes / us * 1e-3);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const int K = 64;
    const int64_t nmax = 65536;
    const int64_t nalloc = 2 * nmax;
    uint4 *board, *meta;
    Ring R;
    uint32_t* sink;
    R.rows = K;
    CK(hipMalloc(&board, 16 * nalloc));
    CK(hipMalloc(&meta, 16 * nalloc));
    CK(hipMemset(board, 0, 16 * nalloc));
    CK(hipMemset(meta, 0, 16 * nalloc));
    CK(hipMalloc(&R.s, 16 * nalloc * K));
    CK(hipMalloc(&R.s2, 16 * nalloc * K));
    CK(hipMalloc(&R.a, nalloc * K));
    CK(hipMalloc(&R.r, 4 * nalloc * K));
    CK(hipMalloc(&R.d, nalloc * K));
    CK(hipMalloc(&sink, 64));
    for (int64_t n : {nmax, (int64_t)1024, 2 * nmax}) {
        run<F_PHILOX | F_STORE | F_BOARD>("full", n, K, board, meta, R, sink);
        run<F_PHILOX | F_STORE | F_BOARD | F_SOFF>("full, uniform offsets", n, K, board, meta, R, sink);
        run<F_HALF | F_STORE | F_BOARD | F_SOFF>("half philox, uniform offs", n, K, board, meta, R, sink);
        run<F_STORE | F_BOARD | F_SOFF>("no philox", n, K, board, meta, R, sink);
        run<F_PHILOX | F_BOARD>("no stores", n, K, board, meta, R, sink);
        run<F_BOARD>("board only", n, K, board, meta, R, sink);
        run<F_PHILOX>("philox only", n, K, board, meta, R, sink);
        run<F_PHILOX | F_STORE | F_SOFF>("philox + stores", n, K, board, meta, R, sink);
        run<F_STORE | F_SOFF>("stores only", n, K, board, meta, R, sink);
        run_new<0>("new: base", n, K, board, meta, R);
        run_new<N_X3>("new: xor3", n, K, board, meta, R);
        run_new<N_DONE>("new: done-test", n, K, board, meta, R);
        run_new<N_BUF>("new: buffer stores", n, K, board, meta, R);
        run_new<N_HALF>("new: half philox", n, K, board, meta, R);
        run_new<N_X3 | N_HALF>("new: xor3+half", n, K, board, meta, R);
        run_new<N_X3 | N_DONE | N_BUF | N_HALF>("new: all", n, K, board, meta, R);
        run_new2<0>("new2: branch-free, unroll2", n, K, board, meta, R);
        run_new2<1>("new2: + spawn-0 select", n, K, board, meta, R);
        run_new2<3>("new2: + sw-pipelined philox", n, K, board, meta, R);
        run_new2<5>("new2: + branch-free reset", n, K, board, meta, R);
        run_new2<7>("new2: + both", n, K, board, meta, R);
    }
    return 0;
}
