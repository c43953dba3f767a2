// g2048_board.hpp -- per-lane 2048 board arithmetic for gfx950 (device-only).
//
// A board is four u32 words in VGPRs; byte c of word r is the log2 exponent of cell (r, c)
// (0 = empty).  Every move is computed LINE-PARALLEL: the four cells along the move direction
// become four words L0..L3 whose byte j belongs to line j, so one VALU op advances all four
// rows (or columns) at once:
//   up    L_k = row k              down  L_k = row 3-k
//   left  L_k = column k           right L_k = column 3-k     (columns = 8-v_perm_b32 transpose)
// and the slide is "compact the non-empty bytes toward L0, then merge equal neighbours once,
// front first" on whole words: zero/equality tests are packed-byte (SWAR) adds, byte masks are
// expanded with v_perm_b32's sign-replicate selectors, selects are v_bfi_b32.  Lanes taking
// different actions run one instruction stream (no divergence).
//
// Reference semantics (ribal-aladeeb/reinforcement-learning-2048):
//   slide/merge/score  src/board.py:92-126 (score += value of each NEW tile, :114)
//   direction mapping  src/board.py:147-183
//   legal mask         src/board.py:128-135
//   spawn distribution src/board.py:41-51 (uniform empty cell, row-major; 2 or 4, p(4)=0.5)
// Checked bit-for-bit against the reference's exhaustive 65 536-row LUT (all four directions),
// its recorded trajectories and the CPU oracle in tests/test_env_gpu.py.
//
// Domain: exponents < 128 (tiles < 2^128; a 4x4 game cannot pass 2^17); the merge-score
// reward is exact while merged tiles stay <= 2^30.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2048 {

constexpr uint32_t K7F = 0x7F7F7F7Fu;
constexpr uint32_t K80 = 0x80808080u;

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
// 0x80 in every non-zero / zero byte (bytes < 0x80: x + 0x7F never carries across bytes).
__device__ __forceinline__ uint32_t nz80(uint32_t x) { return (x + K7F) & K80; }
__device__ __forceinline__ uint32_t z80(uint32_t x) { return ~(x + K7F) & K80; }
// 0x80 byte flags -> 0xFF byte masks: v_perm selectors 8/10/9/11 replicate bit 15/47/31/63 of
// {hi, lo}, i.e. the flags of bytes 0/1/2/3 once lo = f << 8 and hi = f.
__device__ __forceinline__ uint32_t expand80(uint32_t f) { return perm(f, f << 8, 0x0B090A08u); }
// per-bit select (v_bfi_b32): bits of a where m, else b
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    return (a & m) | (b & ~m);
}

__device__ __forceinline__ uint32_t or3_v(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_or3_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

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

// Legal-move mask (bit 0 up, 1 down, 2 left, 3 right) == src/board.py:128-135, without sliding:
// a move is legal iff some tile has a hole next to it in the move direction, or two equal
// non-empty neighbours lie along it.
__device__ __forceinline__ uint32_t legal_mask(const Board& b) {
    const uint32_t n0 = nz80(b.r0), n1 = nz80(b.r1), n2 = nz80(b.r2), n3 = nz80(b.r3);
    // within a row: hole at c, tile at c+1 (left) / tile at c, hole at c+1 (right)
    const uint32_t s0 = n0 >> 8, s1 = n1 >> 8, s2 = n2 >> 8, s3 = n3 >> 8;
    const uint32_t L = (~n0 & s0) | (~n1 & s1) | (~n2 & s2) | (~n3 & s3);
    const uint32_t R = ((n0 & ~s0) | (n1 & ~s1) | (n2 & ~s2) | (n3 & ~s3)) & 0x00808080u;
    const uint32_t H = ((z80(b.r0 ^ (b.r0 >> 8)) & n0) | (z80(b.r1 ^ (b.r1 >> 8)) & n1) |
                        (z80(b.r2 ^ (b.r2 >> 8)) & n2) | (z80(b.r3 ^ (b.r3 >> 8)) & n3)) &
                       0x00808080u;
    // across rows: hole in row r, tile in row r+1 (up) / the reverse (down); equal pairs
    const uint32_t U = (~n0 & n1) | (~n1 & n2) | (~n2 & n3);
    const uint32_t D = (n0 & ~n1) | (n1 & ~n2) | (n2 & ~n3);
    const uint32_t V = (z80(b.r0 ^ b.r1) & n0) | (z80(b.r1 ^ b.r2) & n1) | (z80(b.r2 ^ b.r3) & n2);
    return (uint32_t)((U | V) != 0u) | ((uint32_t)((D | V) != 0u) << 1) |
           ((uint32_t)((L | H) != 0u) << 2) | ((uint32_t)((R | H) != 0u) << 3);
}

// 2^x0 + 2^x1 + 2^x2 + 2^x3 over the bytes x_k of x (each < 32): one SDWA shift per byte, whose
// byte-select operand does the extraction (hipcc spends a v_lshrrev per byte otherwise).
template <int K>
__device__ __forceinline__ uint32_t pow2_byte(uint32_t x, uint32_t one) {
    uint32_t d;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
            : "=v"(d) : "v"(x), "v"(one));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(d) : "v"(x), "v"(one));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
            : "=v"(d) : "v"(x), "v"(one));
    else
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
            : "=v"(d) : "v"(x), "v"(one));
    return d;
}

__device__ __forceinline__ uint32_t pow2_bytes(uint32_t x) {
    const uint32_t one = 1u;
    return pow2_byte<0>(x, one) + pow2_byte<1>(x, one) + pow2_byte<2>(x, one) +
           pow2_byte<3>(x, one);
}

// Slide the four lines toward L0 (byte j of L_k = k-th cell of line j); returns the merge gain.
// zany: 0x80 flags of the empty cells of the lines as given (non-zero iff a cell is empty);
// pairs: 0x80 flags of the equal non-empty neighbours after compaction -- for a full board (no
// compaction) the equal neighbours along the lines, which is_done needs for this axis.
__device__ __forceinline__ uint32_t slide_lines(uint32_t& l0, uint32_t& l1, uint32_t& l2,
                                                uint32_t& l3, uint32_t& zany, uint32_t& pairs) {
    // 1) stable compaction, back to front: [c d] then [b c d] then [a b c d]
    const uint32_t z2 = z80(l2), z3 = z80(l3);
    uint32_t m = expand80(z2);
    l2 = bsel(m, l3, l2);
    l3 &= ~m;
    const uint32_t z1 = z80(l1);
    m = expand80(z1);
    l1 = bsel(m, l2, l1);
    l2 = bsel(m, l3, l2);
    l3 &= ~m;
    const uint32_t z0 = z80(l0);
    zany = or3_v(z0, z1, z2 | z3);
    m = expand80(z0);
    l0 = bsel(m, l1, l0);
    l1 = bsel(m, l2, l1);
    l2 = bsel(m, l3, l2);
    l3 &= ~m;
    // 2) merges, front first; each tile merges at most once
    const uint32_t ab = z80(l0 ^ l1) & nz80(l0);
    const uint32_t bc_raw = z80(l1 ^ l2) & nz80(l1);
    const uint32_t cd_raw = z80(l2 ^ l3) & nz80(l2);
    const uint32_t bc = bc_raw & ~ab;
    const uint32_t cd = cd_raw & (ab | ~bc_raw);
    pairs = or3_v(ab, bc_raw, cd_raw);
    const uint32_t AB = expand80(ab), BC = expand80(bc), CD = expand80(cd);
    const uint32_t c1 = l2 + (cd >> 7);  // merged c+d (when that merge happens)
    const uint32_t b1 = l1 + (bc >> 7);  // merged b+c
    const uint32_t o0 = l0 + (ab >> 7);  // merged a+b
    const uint32_t o1 = bsel(AB, c1, b1);
    const uint32_t o2 = bsel(AB, l3 & ~CD, bsel(BC, l3, c1));
    const uint32_t o3 = l3 & ~(AB | BC | CD);
    // 3) score = sum of 2^e over the merged tiles.  A line merges a+b or b+c, never both (bc
    //    excludes ab), so their merged bytes share one word: 8 candidate bytes, and a zero byte
    //    (no merge) gives 2^0 = 1, taken off at the end.
    const uint32_t e01 = (o0 & AB) | (b1 & BC), e2 = c1 & CD;
    const uint32_t s = (pow2_bytes(e01) + pow2_bytes(e2)) -
                       (8u - (uint32_t)(__popc(ab | bc) + __popc(cd)));
    l0 = o0;
    l1 = o1;
    l2 = o2;
    l3 = o3;
    return s;
}

__device__ __forceinline__ uint32_t slide_lines(uint32_t& l0, uint32_t& l1, uint32_t& l2,
                                                uint32_t& l3) {
    uint32_t zany, pairs;
    return slide_lines(l0, l1, l2, l3, zany, pairs);
}

// Apply action a (0 up, 1 down, 2 left, 3 right) WITHOUT spawning; returns the merge gain.
// done_flags (optional): zero iff the board as given is terminal and not empty -- full, with no
// equal neighbours along the move's lines (the slide's own pair flags: a full board does not
// compact) nor across them (adjacent bytes within the line words); see is_done.
__device__ __forceinline__ uint32_t apply_move(Board& b, uint32_t act,
                                               uint32_t* done_flags = nullptr) {
    const bool horiz = act >= 2u, rev = (act & 1u) != 0u;
    const Board t = transpose(b);
    const uint32_t a0 = horiz ? t.r0 : b.r0, a1 = horiz ? t.r1 : b.r1;
    const uint32_t a2 = horiz ? t.r2 : b.r2, a3 = horiz ? t.r3 : b.r3;
    uint32_t l0 = rev ? a3 : a0, l1 = rev ? a2 : a1, l2 = rev ? a1 : a2, l3 = rev ? a0 : a3;
    uint32_t zany, pairs;
    const uint32_t score = slide_lines(l0, l1, l2, l3, zany, pairs);
    if (done_flags) {
        const uint32_t across = z80(a0 ^ (a0 >> 8)) | z80(a1 ^ (a1 >> 8)) |
                                z80(a2 ^ (a2 >> 8)) | z80(a3 ^ (a3 >> 8));
        *done_flags = or3_v(zany, pairs, across & 0x00808080u);
    }
    Board o;
    o.r0 = rev ? l3 : l0;
    o.r1 = rev ? l2 : l1;
    o.r2 = rev ? l1 : l2;
    o.r3 = rev ? l0 : l3;
    const Board ot = transpose(o);
    b = horiz ? ot : o;
    return score;
}

// Index of the k-th (0-based) set bit of a 4-bit mask (k < popcount(m)).
__device__ __forceinline__ uint32_t kth_bit4(uint32_t m, uint32_t k) {
    uint32_t pos = 0;
    const uint32_t c = __popc(m & 0x3u);
    if (k >= c) { k -= c; m >>= 2; pos = 2; }
    return pos + (k >= (m & 1u));
}

__device__ __forceinline__ void set_cell(Board& b, uint32_t pos, uint32_t e) {
    const uint32_t v = e << ((pos & 3u) * 8u);
    const uint32_t row = pos >> 2;
    b.r0 |= row == 0u ? v : 0u;
    b.r1 |= row == 1u ? v : 0u;
    b.r2 |= row == 2u ? v : 0u;
    b.r3 |= row == 3u ? v : 0u;
}

__device__ __forceinline__ bool cell_empty(const Board& b, uint32_t pos) {
    const uint32_t row = pos >> 2;
    const uint32_t w = row == 0u ? b.r0 : row == 1u ? b.r1 : row == 2u ? b.r2 : b.r3;
    return ((w >> ((pos & 3u) * 8u)) & 0xFFu) == 0u;
}

__device__ __forceinline__ bool has_empty(const Board& b) {
    return (z80(b.r0) | z80(b.r1) | z80(b.r2) | z80(b.r3)) != 0u;
}

// The k-th (0-based) empty cell in row-major order, k = floor(u_cell * n / 2^32) for the n > 0
// empty cells, ORed with exponent e (e = 0 leaves the board as it is).  Binary search over the
// board's halves {r0, r1} / {r2, r3}, then the row, then the byte pair, then the byte; the tile is
// placed with one 64-bit shift into the chosen half.
__device__ __forceinline__ void spawn_at(Board& b, uint32_t u_cell, uint32_t e) {
    const uint32_t z0 = z80(b.r0), z1 = z80(b.r1), z2 = z80(b.r2), z3 = z80(b.r3);
    const uint32_t p1 = __popc(z0), p2 = p1 + __popc(z1), p3 = p2 + __popc(z2);
    const uint32_t n = p3 + __popc(z3);
    uint32_t k = __umulhi(u_cell, n);
    const bool hi = k >= p2;  // rows 2-3
    const uint32_t za = hi ? z2 : z0, zb = hi ? z3 : z1;
    const uint32_t c1 = hi ? p3 - p2 : p1;
    k = hi ? k - p2 : k;
    const bool w1 = k >= c1;  // the half's second row
    k = w1 ? k - c1 : k;
    uint32_t z = w1 ? zb : za;
    const uint32_t c2 = __popc(z & 0x8080u);
    const bool h2 = k >= c2;  // bytes 2-3
    k = h2 ? k - c2 : k;
    z = h2 ? z >> 16 : z;
    const bool b1 = k >= ((z >> 7) & 1u);
    const uint32_t sh = (w1 ? 32u : 0u) | (h2 ? 16u : 0u) | (b1 ? 8u : 0u);
    const uint64_t v = (uint64_t)e << sh;
    b.r0 |= hi ? 0u : (uint32_t)v;
    b.r1 |= hi ? 0u : (uint32_t)(v >> 32);
    b.r2 |= hi ? (uint32_t)v : 0u;
    b.r3 |= hi ? (uint32_t)(v >> 32) : 0u;
}

// One spawn (src/board.py:41-51): the k-th empty cell in row-major order with
// k = floor(u_cell * n / 2^32); exponent 2 (a "4") iff u_val < p4_thresh.
__device__ __forceinline__ void spawn(Board& b, uint32_t u_cell, uint32_t u_val,
                                      uint32_t p4_thresh) {
    if (!has_empty(b)) return;
    spawn_at(b, u_cell, u_val < p4_thresh ? 2u : 1u);
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
// a ^ b ^ k in ONE v_bitop3_b32 (truth table 0x96).  hipcc emits two v_xor_b32 when k is a
// scalar operand (the key schedule always is); inline asm keeps it to one VALU op.  The "s"
// constraint makes a non-uniform k a compile error instead of a silent readfirstlane.
__device__ __forceinline__ uint32_t xor3_sk(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "s"(k));
    return d;
}


// Same rounds, constants and counter layout as rocRAND's philox4x32_10 engine: the block for
// (seed, subsequence s, offset 4t) is philox10({t_lo, t_hi, s_lo, s_hi}, {seed_lo, seed_hi}).
// The key (k0, k1) must be wave-uniform (it is the env / sampler seed everywhere).
__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // one v_mad_u64_u32 per product instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
        const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u;
        const uint64_t p1 = (uint64_t)c.z * 0xCD9E8D57u;
        c = make_uint4(xor3_sk((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1,
                       xor3_sk((uint32_t)(p0 >> 32), c.w, k1), (uint32_t)p0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Domain bits 30-31 of the subsequence word: step draws of the action-given / eps-greedy modes
// (one block per step), random-policy draws (one block per two steps), explicit resets, sampler.
enum : uint32_t { DOMAIN_STEP = 0u, DOMAIN_RANDOM = 1u, DOMAIN_RESET = 2u, DOMAIN_SAMPLE = 3u };

__device__ __forceinline__ uint4 draw(uint32_t seed_lo, uint32_t seed_hi, uint64_t gid,
                                      uint32_t domain, uint64_t t) {
    return philox10(make_uint4((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)gid,
                               (uint32_t)(gid >> 32) | (domain << 30)),
                    seed_lo, seed_hi);
}

// eps of a board's next eps-greedy step (src/dqn_lib.py:184-188): eps_decay > 0 selects the
// per-board schedule max((D - episodes) / D, eps_min), else *eps_dev or eps.  Shared by the step
// kernels and the greedy-only forward (g2048_qnet.hip), which must agree on every draw.
__device__ __forceinline__ double step_eps(double eps_decay, double eps_min, const double* eps_dev,
                                           double eps, uint32_t episodes) {
    if (eps_decay > 0.0) return fmax((eps_decay - (double)episodes) / eps_decay, eps_min);
    return eps_dev ? *eps_dev : eps;
}

// The random branch of epsilon_greedy_policy (src/dqn_lib.py:20, np.random.rand() < eps) with
// word y of the step's Philox block as the uniform.
__device__ __forceinline__ bool explores(uint32_t uy, double eps) {
    return (double)uy * (1.0 / 4294967296.0) < eps;
}

// Two spawns on an empty board (src/board.py:18-20) from ONE Philox block: (u.z, u.w) for the
// first, (u.z << 4, u.x << 2) for the second -- the words a terminal step leaves unused, so the
// auto-reset reuses the step's own block.  With 16 empty cells the first is cell u.z >> 28; the
// second is the k-th of the remaining 15.
__device__ __forceinline__ Board fresh_board(uint4 u, uint32_t p4_thresh) {
    const uint32_t ca = u.z >> 28;
    const uint32_t k2 = __umulhi(u.z << 4, 15u);
    const uint32_t cb = k2 + (uint32_t)(k2 >= ca);
    Board b{0u, 0u, 0u, 0u};
    set_cell(b, ca, u.w < p4_thresh ? 2u : 1u);
    set_cell(b, cb, (u.x << 2) < p4_thresh ? 2u : 1u);
    return b;
}

// ------------------------------------------------------------------ terminal test
// The random policy's step (ABI v3, include/g2048.h) lives in g2048_roll.hpp.
// No legal move (src/dqn_lib.py:17-18: max(available_moves) == 0) without the 4-direction mask:
// a board with both an empty and a non-empty cell always has one (some tile borders a hole), so
// it is terminal iff it is full with no equal neighbours, or empty.
__device__ __forceinline__ bool is_done(const Board& b) {
    const uint32_t z = z80(b.r0) | z80(b.r1) | z80(b.r2) | z80(b.r3);
    const uint32_t H = z80(b.r0 ^ (b.r0 >> 8)) | z80(b.r1 ^ (b.r1 >> 8)) |
                       z80(b.r2 ^ (b.r2 >> 8)) | z80(b.r3 ^ (b.r3 >> 8));
    const uint32_t V = z80(b.r0 ^ b.r1) | z80(b.r1 ^ b.r2) | z80(b.r2 ^ b.r3);
    // one compare: min(no-move witnesses, any tile) == 0
    return min(z | (H & 0x00808080u) | V, b.r0 | b.r1 | b.r2 | b.r3) == 0u;
}

// ------------------------------------------------------------------ policy (src/dqn_lib.py:16-30)
// compat: Qn = Q - min(Q)*max(Q) - min(Q) (the reference's operator precedence, F5),
// a = argmax(avail * Qn) with the first index winning ties; no FMA contraction so the products
// round exactly like torch's separate kernels.  Non-finite Q follows torch: torch.min/torch.max
// are NaN once any element is NaN, 0 * inf and inf - inf are NaN, and torch.argmax ranks NaN
// above every number (the first NaN wins).
template <typename T>
__device__ __forceinline__ bool is_nan(T x) {
    return __builtin_isnan(x);
}

// torch.argmax over 4 values: first NaN if any, else the first maximum.
template <typename T>
__device__ __forceinline__ uint32_t argmax4_torch(T v0, T v1, T v2, T v3) {
    uint32_t a = 0;
    T best = v0;
    bool bn = is_nan(v0);
    if (!bn && (is_nan(v1) || v1 > best)) { a = 1; best = v1; bn = is_nan(v1); }
    if (!bn && (is_nan(v2) || v2 > best)) { a = 2; best = v2; bn = is_nan(v2); }
    if (!bn && (is_nan(v3) || v3 > best)) { a = 3; }
    return a;
}

// torch.max over 4 values (src/dqn_lib.py:29, the Q-sum of the episode log): NaN if any is NaN.
template <typename T>
__device__ __forceinline__ T qmax4_torch(T q0, T q1, T q2, T q3) {
    const T m = q0 > q1 ? q0 : q1, n = q2 > q3 ? q2 : q3;
    const T mx = m > n ? m : n;
    return (is_nan(q0) || is_nan(q1) || is_nan(q2) || is_nan(q3)) ? (T)__builtin_nan("") : mx;
}

template <typename T>
__device__ __forceinline__ uint32_t greedy_compat(T q0, T q1, T q2, T q3, uint32_t legal) {
#pragma clang fp contract(off)
    T mn = q0, mx = q0;
    mn = q1 < mn ? q1 : mn; mx = q1 > mx ? q1 : mx;
    mn = q2 < mn ? q2 : mn; mx = q2 > mx ? q2 : mx;
    mn = q3 < mn ? q3 : mn; mx = q3 > mx ? q3 : mx;
    if (is_nan(q0) || is_nan(q1) || is_nan(q2) || is_nan(q3)) {
        mn = (T)__builtin_nan("");
        mx = mn;
    }
    const T prod = mn * mx;
    const T v0 = (T)(legal & 1u) * ((q0 - prod) - mn);
    const T v1 = (T)((legal >> 1) & 1u) * ((q1 - prod) - mn);
    const T v2 = (T)((legal >> 2) & 1u) * ((q2 - prod) - mn);
    const T v3 = (T)((legal >> 3) & 1u) * ((q3 - prod) - mn);
    return argmax4_torch(v0, v1, v2, v3);
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
