// g2048_board.hpp -- per-lane 2048 board arithmetic for gfx950 (device-only).
//
// A board is four u32 "rows" held in VGPRs; byte c of row r is the log2 exponent of cell (r, c)
// (0 = empty).  All four moves are reduced to "slide every row toward byte 0":
//   left = identity, right = byte-reverse, up = 4x4 byte transpose, down = transpose + reverse;
// the transpose is 8 v_perm_b32, the reverse one v_perm_b32 per row with a per-lane selector, so
// lanes taking different actions run the same instruction stream (no divergence).
// The legal-move mask is computed without sliding at all: packed-byte (SWAR) zero / equality tests
// give 16-bit occupancy masks whose shifts expose "a tile can move into a hole" and "two equal
// neighbours can merge".
//
// Reference semantics (ribal-aladeeb/reinforcement-learning-2048):
//   slide/merge/score  src/board.py:92-126 (score += value of each NEW tile, :114)
//   direction mapping  src/board.py:147-183
//   legal mask         src/board.py:128-135
//   spawn distribution src/board.py:41-51 (uniform empty cell, row-major; 2 or 4, p(4)=0.5)
// Checked bit-for-bit against the oracle and the reference's exhaustive 65 536-row LUT in
// tests/test_env_gpu.py.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// 0x80 in every non-zero byte of x, 0 elsewhere (exact, no cross-byte carries).
__device__ __forceinline__ uint32_t nz_bytes(uint32_t x) {
    return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// bit c set iff byte c of x is non-zero.
__device__ __forceinline__ uint32_t nz4(uint32_t x) {
    return (((nz_bytes(x) >> 7) * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ uint32_t z4(uint32_t x) { return (~nz4(x)) & 0xFu; }

struct Board {
    uint32_t r0, r1, r2, r3;
};

__device__ __forceinline__ Board transpose(const Board& b) {
    const uint32_t a = perm(b.r1, b.r0, 0x05010400u);  // r0b0 r1b0 r0b1 r1b1
    const uint32_t c = perm(b.r1, b.r0, 0x07030602u);  // r0b2 r1b2 r0b3 r1b3
    const uint32_t d = perm(b.r3, b.r2, 0x05010400u);  // r2b0 r3b0 r2b1 r3b1
    const uint32_t e = perm(b.r3, b.r2, 0x07030602u);  // r2b2 r3b2 r2b3 r3b3
    Board t;
    t.r0 = perm(d, a, 0x05040100u);
    t.r1 = perm(d, a, 0x07060302u);
    t.r2 = perm(e, c, 0x05040100u);
    t.r3 = perm(e, c, 0x07060302u);
    return t;
}

// 16-bit empty-cell mask, bit 4r + c.
__device__ __forceinline__ uint32_t empty_mask(const Board& b) {
    return z4(b.r0) | (z4(b.r1) << 4) | (z4(b.r2) << 8) | (z4(b.r3) << 12);
}

// Legal-move mask (bit 0 up, 1 down, 2 left, 3 right) == src/board.py:128-135.
__device__ __forceinline__ uint32_t legal_mask(const Board& b) {
    const uint32_t n0 = nz4(b.r0), n1 = nz4(b.r1), n2 = nz4(b.r2), n3 = nz4(b.r3);
    const uint32_t N = n0 | (n1 << 4) | (n2 << 8) | (n3 << 12);
    const uint32_t Z = (~N) & 0xFFFFu;
    // a tile next to a hole in the move direction
    const uint32_t left = Z & (N >> 1) & 0x7777u;
    const uint32_t right = N & (Z >> 1) & 0x7777u;
    const uint32_t up = Z & (N >> 4) & 0x0FFFu;
    const uint32_t down = N & (Z >> 4) & 0x0FFFu;
    // equal non-zero neighbours: horizontal (c, c+1) and vertical (r, r+1)
    const uint32_t H = ((z4(b.r0 ^ (b.r0 >> 8)) & n0) | ((z4(b.r1 ^ (b.r1 >> 8)) & n1) << 4) |
                        ((z4(b.r2 ^ (b.r2 >> 8)) & n2) << 8) |
                        ((z4(b.r3 ^ (b.r3 >> 8)) & n3) << 12)) & 0x7777u;
    const uint32_t V = (z4(b.r0 ^ b.r1) & n0) | ((z4(b.r1 ^ b.r2) & n1) << 4) |
                       ((z4(b.r2 ^ b.r3) & n2) << 8);
    return ((up | V) != 0u) | (((down | V) != 0u) << 1) | (((left | H) != 0u) << 2) |
           (((right | H) != 0u) << 3);
}

// Slide one row toward byte 0, merging equal neighbours once, leftmost first; adds the value
// of every new tile to `score` (src/board.py:92-126).
__device__ __forceinline__ uint32_t slide_row(uint32_t x, uint32_t& score) {
    // 1) compact the non-zero bytes to the front with one v_perm_b32; selector byte k = index of
    //    the k-th non-zero byte, or 4 (= a byte of the zero hi operand) when there is none.
    uint32_t m = nz4(x);
    const uint32_t s0 = min((uint32_t)(__ffs(m) - 1), 4u);
    m &= m - 1u;
    const uint32_t s1 = min((uint32_t)(__ffs(m) - 1), 4u);
    m &= m - 1u;
    const uint32_t s2 = min((uint32_t)(__ffs(m) - 1), 4u);
    m &= m - 1u;
    const uint32_t s3 = min((uint32_t)(__ffs(m) - 1), 4u);
    const uint32_t c = perm(0u, x, s0 | (s1 << 8) | (s2 << 16) | (s3 << 24));
    // 2) merge pass over the compacted [a b c d]
    const uint32_t a = c & 0xFFu, b = (c >> 8) & 0xFFu, e = (c >> 16) & 0xFFu, d = c >> 24;
    const bool ab = (a == b) & (a != 0u);
    const bool bc = (b == e) & (b != 0u) & !ab;          // b+c merge (only if a,b did not)
    const bool cd = (e == d) & (e != 0u) & (ab | !((b == e) & (b != 0u)));
    const uint32_t o0 = a + (uint32_t)ab;
    const uint32_t o1 = ab ? (e + (uint32_t)cd) : (b + (uint32_t)bc);
    const uint32_t o2 = ab ? (cd ? 0u : d) : (bc ? d : (e + (uint32_t)cd));
    const uint32_t o3 = (ab | bc | cd) ? 0u : d;
    score += (ab ? (2u << (a & 31u)) : 0u) + (bc ? (2u << (b & 31u)) : 0u) +
             (cd ? (2u << (e & 31u)) : 0u);
    return o0 | (o1 << 8) | (o2 << 16) | (o3 << 24);
}

// Apply action a (0 up, 1 down, 2 left, 3 right) WITHOUT spawning; returns the merge gain.
__device__ __forceinline__ uint32_t apply_move(Board& b, uint32_t act) {
    const bool vert = act < 2u;
    const uint32_t sel = (act & 1u) ? 0x00010203u : 0x03020100u;  // byte reverse or identity
    Board t = transpose(b);
    Board o;
    o.r0 = vert ? t.r0 : b.r0;
    o.r1 = vert ? t.r1 : b.r1;
    o.r2 = vert ? t.r2 : b.r2;
    o.r3 = vert ? t.r3 : b.r3;
    uint32_t score = 0;
    o.r0 = perm(0u, slide_row(perm(0u, o.r0, sel), score), sel);
    o.r1 = perm(0u, slide_row(perm(0u, o.r1, sel), score), sel);
    o.r2 = perm(0u, slide_row(perm(0u, o.r2, sel), score), sel);
    o.r3 = perm(0u, slide_row(perm(0u, o.r3, sel), score), sel);
    t = transpose(o);
    b.r0 = vert ? t.r0 : o.r0;
    b.r1 = vert ? t.r1 : o.r1;
    b.r2 = vert ? t.r2 : o.r2;
    b.r3 = vert ? t.r3 : o.r3;
    return score;
}

// Index of the k-th (0-based) set bit of a 16-bit mask (k < popcount(m)).
__device__ __forceinline__ uint32_t kth_bit16(uint32_t m, uint32_t k) {
    uint32_t pos = 0;
    uint32_t c = __popc(m & 0xFFu);
    if (k >= c) { k -= c; m >>= 8; pos += 8; }
    c = __popc(m & 0xFu);
    if (k >= c) { k -= c; m >>= 4; pos += 4; }
    c = __popc(m & 0x3u);
    if (k >= c) { k -= c; m >>= 2; pos += 2; }
    c = m & 1u;
    if (k >= c) { pos += 1; }
    return pos;
}

__device__ __forceinline__ void set_cell(Board& b, uint32_t pos, uint32_t e) {
    const uint32_t v = e << ((pos & 3u) * 8u);
    const uint32_t row = pos >> 2;
    b.r0 |= row == 0u ? v : 0u;
    b.r1 |= row == 1u ? v : 0u;
    b.r2 |= row == 2u ? v : 0u;
    b.r3 |= row == 3u ? v : 0u;
}

// One spawn (src/board.py:41-51): uniform empty cell in row-major order via
// k = floor(u_cell * n / 2^32); exponent 2 (a "4") iff u_val < p4_thresh.
__device__ __forceinline__ void spawn(Board& b, uint32_t u_cell, uint32_t u_val,
                                      uint32_t p4_thresh) {
    const uint32_t Z = empty_mask(b);
    const uint32_t n = __popc(Z);
    if (n == 0u) return;
    const uint32_t k = __umulhi(u_cell, n);
    set_cell(b, kth_bit16(Z, k), u_val < p4_thresh ? 2u : 1u);
}

__device__ __forceinline__ uint32_t max_exp(const Board& b) {
    uint32_t m = 0;
    const uint32_t rows[4] = {b.r0, b.r1, b.r2, b.r3};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m = max(m, max(max(rows[r] & 0xFFu, (rows[r] >> 8) & 0xFFu),
                       max((rows[r] >> 16) & 0xFFu, rows[r] >> 24)));
    }
    return m;
}

// ------------------------------------------------------------------ Philox4x32-10
// Same rounds, constants and counter layout as rocRAND's philox4x32_10 engine: the block for
// (seed, subsequence s, offset 4t) is philox10({t_lo, t_hi, s_lo, s_hi}, {seed_lo, seed_hi}).
__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

enum : uint32_t { DOMAIN_STEP = 0u, DOMAIN_AUTORESET = 1u, DOMAIN_RESET = 2u, DOMAIN_SAMPLE = 3u };

__device__ __forceinline__ uint4 draw(uint32_t seed_lo, uint32_t seed_hi, uint64_t gid,
                                      uint32_t domain, uint64_t t) {
    return philox10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid,
                               (uint32_t)(gid >> 32) | (domain << 30)),
                    seed_lo, seed_hi);
}

__device__ __forceinline__ Board fresh_board(uint4 u, uint32_t p4_thresh) {
    Board b{0u, 0u, 0u, 0u};
    spawn(b, u.x, u.y, p4_thresh);
    spawn(b, u.z, u.w, p4_thresh);
    return b;
}

// ------------------------------------------------------------------ policy (src/dqn_lib.py:16-30)
// compat: Qn = Q - min(Q)*max(Q) - min(Q) (the reference's operator precedence, F5),
// a = argmax(avail * Qn) with the first index winning ties; no FMA contraction so the products
// round exactly like torch's separate kernels.
template <typename T>
__device__ __forceinline__ uint32_t greedy_compat(T q0, T q1, T q2, T q3, uint32_t legal) {
#pragma clang fp contract(off)
    T mn = q0, mx = q0;
    mn = q1 < mn ? q1 : mn; mx = q1 > mx ? q1 : mx;
    mn = q2 < mn ? q2 : mn; mx = q2 > mx ? q2 : mx;
    mn = q3 < mn ? q3 : mn; mx = q3 > mx ? q3 : mx;
    const T prod = mn * mx;
    const T v0 = (T)(legal & 1u) * ((q0 - prod) - mn);
    const T v1 = (T)((legal >> 1) & 1u) * ((q1 - prod) - mn);
    const T v2 = (T)((legal >> 2) & 1u) * ((q2 - prod) - mn);
    const T v3 = (T)((legal >> 3) & 1u) * ((q3 - prod) - mn);
    uint32_t a = 0;
    T best = v0;
    if (v1 > best) { a = 1; best = v1; }
    if (v2 > best) { a = 2; best = v2; }
    if (v3 > best) { a = 3; best = v3; }
    return a;
}

// fixed: argmax of Q over legal moves only (first index on ties), 0 if no move is legal.
template <typename T>
__device__ __forceinline__ uint32_t greedy_fixed(T q0, T q1, T q2, T q3, uint32_t legal) {
    const T qs[4] = {q0, q1, q2, q3};
    uint32_t a = 0;
    bool found = false;
    T best = q0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const bool ok = (legal >> j) & 1u;
        const bool take = ok && (!found || qs[j] > best);
        a = take ? j : a;
        best = take ? qs[j] : best;
        found = found || ok;
    }
    return a;
}

}  // namespace g2048
