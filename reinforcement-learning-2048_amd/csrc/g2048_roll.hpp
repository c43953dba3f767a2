// g2048_roll.hpp -- the random-policy step of the rollout kernel (k_rollout_lean), rewritten for
// the instruction budget of ONE wave per SIMD (64k boards on 256 CUs).  Measured on gfx950
// (tools/opcost.hip, tools/pairbench.hip): with one wave per SIMD every VALU op costs one issue
// turn of ~5.1-5.9 shader cycles whatever it computes, v_mad_u64_u32 / v_lshlrev_b64 / v_mov
// cost 8-10, SALU ops 8-10; a second wave per SIMD adds throughput only for plain VOP2 ops.  So the
// step is bound by its instruction count, and this file minimises it.  The single-step kernel
// and the general k_rollout use the same functions; the oracle restates them (oracle2048.c) and
// tests/test_fullsize_gpu.py + tools/rollexp.hip compare the kernels on every output.
//
// Direction handling without selects: a 4x4 byte board in four row words goes to the four LINE
// words of the move (byte j = line j, word k = k-th cell along the move, see g2048_board.hpp) by
// an 8-v_perm_b32 network whose four selectors are PER LANE:
//     a = perm(r1, r0, SA)  c = perm(r1, r0, SC)  d = perm(r3, r2, SA)  e = perm(r3, r2, SC)
//     L0 = perm(d, a, S0)   L1 = perm(e, c, S0)   L2 = perm(d, a, S2)   L3 = perm(e, c, S2)
// With the selectors of kDirNet one network is the identity (up), the word reversal (down), the
// transpose (left) or the transpose with reversed word order (right); the inverse map (line words
// back to rows) is the same network with the second selector quad.  The lane fetches its action's
// eight selectors from an LDS table (two ds_read_b128) instead of spending 16 v_cndmask on
// horiz / rev selects around two fixed transposes.
#pragma once

#include "g2048_board.hpp"

namespace g2048 {

// Region markers for ISA accounting (tools/isa_regions.py, built with -DG2048_ISA_MARKS only; they
// pin the instruction order, so the timed library is built without them).
// A marker names the region that follows it and takes the values the previous region produced as
// "+v" operands, so those are computed before it and their users come after it.
#ifdef G2048_ISA_MARKS
#define G2048_MARK(x, ...) asm volatile(";; region " #x : __VA_ARGS__)
#else
#define G2048_MARK(x, ...)
#endif

// 255 in a register the compiler cannot see through (lean_step's k255), set once per kernel
__device__ __forceinline__ uint32_t opaque_255() {
    uint32_t k = 255u;
    asm volatile("" : "+v"(k));
    return k;
}

// [action][0] forward {SA, SC, S0, S2}, [action][1] inverse; actions 0 up, 1 down, 2 left, 3 right
// (src/board.py:147-183).  Up, down and left are involutions (inverse == forward).
__device__ __constant__ const uint32_t kDirNet[4][2][4] = {
    {{0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u},
     {0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u}},
    {{0x07060504u, 0x03020100u, 0x07060504u, 0x03020100u},
     {0x07060504u, 0x03020100u, 0x07060504u, 0x03020100u}},
    {{0x06020400u, 0x07030501u, 0x05040100u, 0x07060302u},
     {0x06020400u, 0x07030501u, 0x05040100u, 0x07060302u}},
    {{0x05010703u, 0x04000602u, 0x05040100u, 0x07060302u},
     {0x02060004u, 0x03070105u, 0x01000504u, 0x03020706u}},
};

__device__ __forceinline__ void dir_net(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                        const uint4& S, uint32_t& l0, uint32_t& l1, uint32_t& l2,
                                        uint32_t& l3) {
    const uint32_t a = perm(r1, r0, S.x), c = perm(r1, r0, S.y);
    const uint32_t d = perm(r3, r2, S.x), e = perm(r3, r2, S.y);
    l0 = perm(d, a, S.z);
    l1 = perm(e, c, S.z);
    l2 = perm(d, a, S.w);
    l3 = perm(e, c, S.w);
}

// 0xFF in every byte of x that is zero, from D = 0x80808080 - x (bit 7 of byte j set iff byte j
// of x is 0; bytes < 0x80, so no borrow crosses a byte): v_perm_b32's sign-replicate selectors
// 8/10/9/11 read bits 15/47/31/63 of {D, D << 8} = bit 7 of bytes 0/1/2/3 of D.  The other bits
// of D are never read, so D needs no mask.
__device__ __forceinline__ uint32_t zmask(uint32_t D) { return perm(D, D << 8, 0x0B090A08u); }

// (a ^ b) + c in one VALU op
__device__ __forceinline__ uint32_t xad(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// sum over the bytes b of x of (byte b of f) << (byte b of x): one SDWA shift per byte, whose
// byte-select operands do both extractions
template <int K>
__device__ __forceinline__ uint32_t shl_byte(uint32_t x, uint32_t f) {
    uint32_t d;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0"
            : "=v"(d) : "v"(x), "v"(f));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1"
            : "=v"(d) : "v"(x), "v"(f));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2"
            : "=v"(d) : "v"(x), "v"(f));
    else
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3"
            : "=v"(d) : "v"(x), "v"(f));
    return d;
}

__device__ __forceinline__ uint32_t shl_bytes(uint32_t x, uint32_t f) {
    return shl_byte<0>(x, f) + shl_byte<1>(x, f) + shl_byte<2>(x, f) + shl_byte<3>(x, f);
}

// lanes set in the wave mask `on` take a, the others b (v_cndmask_b32 with an SGPR-pair mask).
// Opaque to the compiler: plain selects on `done` in the auto-reset block were turned back into
// a lane-masked branch whose phi copies cost a v_mov per value.
__device__ __forceinline__ uint32_t sel_lanes(uint64_t on, uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(d) : "v"(b), "v"(a), "s"(on));
    return d;
}

// The merge gain: sum over the bytes b of (f01_b << e01_b) + (f2_b << e2_b), f = 0x01 per merging
// line -- eight SDWA shifts whose byte-select operands do the extractions, summed with three
// v_add3.  One asm block: after an inline-asm result hipcc pads its consumer with an s_nop (it
// cannot rule out a transcendental op, whose result needs a wait state); inside the block the
// shifts (dst_sel DWORD) need none.
__device__ __forceinline__ uint32_t merge_gain(uint32_t e01, uint32_t f01, uint32_t e2, uint32_t f2) {
    uint32_t g, t0, t1, t2, t3, t4, t5, t6;
    asm("v_lshlrev_b32_sdwa %1, %8, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_lshlrev_b32_sdwa %2, %8, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_lshlrev_b32_sdwa %3, %8, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_lshlrev_b32_sdwa %4, %8, %9 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_lshlrev_b32_sdwa %5, %10, %11 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_lshlrev_b32_sdwa %6, %10, %11 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_lshlrev_b32_sdwa %7, %10, %11 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_add3_u32 %1, %1, %2, %3\n\t"
        "v_lshlrev_b32_sdwa %2, %10, %11 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_add3_u32 %4, %4, %5, %6\n\t"
        "v_add3_u32 %0, %1, %4, %7\n\t"
        "v_add_u32 %0, %0, %2"
        : "=&v"(g), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6)
        : "v"(e01), "v"(f01), "v"(e2), "v"(f2));
    return g;
}

// 0x80 flags of the equal non-empty neighbours along the compacted lines: ab (cells 0, 1), bc
// (1, 2), cd (2, 3) -- the later cell non-empty implies the earlier one is.  v_xad: bit 7 of
// (x ^ y) + 0x7F is set iff the bytes differ, of y + 0x7F iff y != 0; bitop3 0x08 = ~S0 & S1 & S2
// (table index S0*4 + S1*2 + S2).  One asm block (see merge_gain).
__device__ __forceinline__ void pair_flags(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                           uint32_t& ab, uint32_t& bc, uint32_t& cd) {
    uint32_t x0, x1, x2;
    asm("v_xad_u32 %3, %6, %7, %10\n\t"
        "v_xad_u32 %4, %7, %8, %10\n\t"
        "v_xad_u32 %5, %8, %9, %10\n\t"
        "v_add_u32 %0, %7, %10\n\t"
        "v_add_u32 %1, %8, %10\n\t"
        "v_add_u32 %2, %9, %10\n\t"
        "v_bitop3_b32 %0, %3, %0, %11 bitop3:0x08\n\t"
        "v_bitop3_b32 %1, %4, %1, %11 bitop3:0x08\n\t"
        "v_bitop3_b32 %2, %5, %2, %11 bitop3:0x08"
        : "=&v"(ab), "=&v"(bc), "=&v"(cd), "=&v"(x0), "=&v"(x1), "=&v"(x2)
        : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(K7F), "v"(K80));
}

// Equal neighbours ACROSS the lines: 0x80 flags of the bytes j < 3 of any line word equal to byte
// j + 1 (v_xad: bit 7 of (x ^ y) + 0x7F is set iff the bytes differ).  One asm block (see
// merge_gain).
__device__ __forceinline__ uint32_t across_pairs(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3) {
    uint32_t r, a0, a1, a2, a3;
    asm("v_alignbit_b32 %1, %6, %5, 8\n\t"
        "v_alignbit_b32 %2, %7, %6, 8\n\t"
        "v_alignbit_b32 %3, %8, %7, 8\n\t"
        "v_lshrrev_b32 %4, 8, %8\n\t"
        "v_xad_u32 %1, %5, %1, %9\n\t"
        "v_xad_u32 %2, %6, %2, %9\n\t"
        "v_xad_u32 %3, %7, %3, %9\n\t"
        "v_xad_u32 %4, %8, %4, %9\n\t"
        "v_bitop3_b32 %1, %1, %2, %3 bitop3:0x80\n\t"
        "v_bitop3_b32 %0, %1, %4, %10 bitop3:0x2a"  // ~(S0 & S1) & S2 (table index S0*4 + S1*2 + S2)
        : "=v"(r), "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
        : "v"(l0), "v"(l1), "v"(l2), "v"(l3), "v"(K7F), "v"(0x00808080u));
    return r;
}

// The moved flags of a step: 0x80 per line with a hole before a tile along it -- bit 7 of
// (D0 & ~D1) | (D1 & ~D2) | (D2 & N3), N3 = L3 + 0x7F7F7F7F (bit 7: cell 3 holds a tile) -- or with a
// merge (P = ab | bc | cd, 0x80 flags).  Three bitop3 (table index S0*4 + S1*2 + S2): 0x74 =
// (S0 & ~S1) | (S1 & ~S2), 0xF8 = S0 | (S1 & S2), 0xEA = (S0 & S1) | S2.  One asm block: written
// in C, hipcc rewrites ~D as L + 0x7F per word (nine ops instead of three).
__device__ __forceinline__ uint32_t moved_flags(uint32_t D0, uint32_t D1, uint32_t D2, uint32_t N3,
                                                uint32_t P) {
    uint32_t mv, x;
    asm("v_bitop3_b32 %1, %2, %3, %4 bitop3:0x74\n\t"
        "v_bitop3_b32 %1, %1, %4, %5 bitop3:0xf8\n\t"
        "v_bitop3_b32 %0, %1, %6, %7 bitop3:0xea"
        : "=v"(mv), "=&v"(x)
        : "v"(D0), "v"(D1), "v"(D2), "v"(N3), "v"(K80), "v"(P));
    return mv;
}

// 0xFF in every byte of a 0x01-flag word: f * 255 (bytes <= 1, so no carries) in one
// v_mul_lo_u32.  k255 = 255 held opaque in a register: hipcc rewrites a multiply by the
// constant as (f << 8) - f, two ops.
__device__ __forceinline__ uint32_t expand01(uint32_t f, uint32_t k255) { return f * k255; }

// The spawn slot of a step.  E_j = line j's empty cells after the move = its empty cells before
// (the compaction masks M0..M2: 0xFF per empty byte; cell 3 from N3 = L3 + 0x7F7F7F7F, bit 7 set
// for a tile) + its merges (f01 + f_cd, each frees a cell) -- at most 4 per byte, no carries --
// and S = E * 0x01010101 (byte j: empties in lines 0..j; byte 3: their total).  Then
//   n  = total mod 16 -- 0 for the empty board as for a full one (neither moves, so neither spawns)
//   k  = floor((w << 3) * n / 2^32), the rank of the chosen empty cell
//   j8 = 8 j*, j* = the number of lines j < 3 with S_j <= k: bit 7 of byte j of
//        X = 0x80 + k - S_j (the bytes stay in [0x70, 0x8F], no borrows)
//   q  = k - S_j* = (position along line j*) - 4, in [-4, -1]: its two low bits are the position
// One asm block: in C, hipcc re-derives n and X from the multiply that made S (more ops).
__device__ __forceinline__ void spawn_slot(uint32_t M0, uint32_t M1, uint32_t M2, uint32_t N3,
                                           uint32_t f01, uint32_t f_cd, uint32_t w, uint32_t& n,
                                           uint32_t& j8, uint32_t& q) {
    uint32_t e, t, u, k;
    asm("v_and_b32 %3, 0x1010101, %7\n\t"
        "v_and_b32 %4, 0x1010101, %8\n\t"
        "v_and_b32 %5, 0x1010101, %9\n\t"
        "v_add3_u32 %3, %3, %4, %5\n\t"
        "v_lshrrev_b32 %4, 7, %10\n\t"
        "v_bfi_b32 %4, %4, 0, %14\n\t"
        "v_add3_u32 %4, %4, %11, %12\n\t"
        "v_add_u32 %3, %3, %4\n\t"
        "v_mul_lo_u32 %3, %3, %14\n\t"
        "v_bfe_u32 %0, %3, 24, 4\n\t"
        "v_lshlrev_b32 %4, 3, %13\n\t"
        "v_mul_hi_u32 %6, %4, %0\n\t"
        "v_mad_u32_u24 %4, %6, %15, %16\n\t"
        "v_sub_u32 %4, %4, %3\n\t"
        "v_and_b32 %4, 0x808080, %4\n\t"
        "v_bcnt_u32_b32 %4, %4, 0\n\t"
        "v_lshlrev_b32 %1, 3, %4\n\t"
        "v_bfe_u32 %4, %3, %1, 8\n\t"
        "v_sub_u32 %2, %6, %4"
        : "=&v"(n), "=&v"(j8), "=&v"(q), "=&v"(e), "=&v"(t), "=&v"(u), "=&v"(k)
        : "v"(M0), "v"(M1), "v"(M2), "v"(N3), "v"(f01), "v"(f_cd), "v"(w), "v"(0x01010101u),
          "v"(0x010101u), "v"(0x808080u));
}

// The merges of the compacted line words C0..C3 from the pair flags (0x80: ab = cells 0, 1 equal,
// bc_raw / cd_raw = cells 1, 2 / 2, 3 equal; see pair_flags):
//   bc = bc_raw & ~ab              (bitop3 0x30: S0 & ~S1)
//   cd = cd_raw & (ab | ~bc_raw)   (bitop3 0xD0: S0 & (S1 | ~S2))
//   f_* = flag >> 7 (0x01 per merging line), AB / BC / CD = f_* * 255 (byte masks, expand01)
//   b1 = C1 + f_bc, c1 = C2 + f_cd, o0 = C0 + f_ab
//   o1 = AB ? c1 : b1,  o2 = AB ? C3 & ~CD : (BC ? C3 : c1),  o3 = C3 & ~(AB | BC | CD)
//   e01 = AB ? o0 : b1 (the merged exponent of an a+b or b+c merge), f01 = f_ab | f_bc
// (bitop3 table index S0*4 + S1*2 + S2; v_bfi_b32 d = S0 ? S1 : S2 per bit.)  One asm block, so
// the selects stay v_bfi (hipcc splits them into and/or pairs once the masks have other users).
__device__ __forceinline__ void merge_lines(uint32_t C0, uint32_t C1, uint32_t C2, uint32_t C3,
                                            uint32_t ab, uint32_t bc_raw, uint32_t cd_raw,
                                            uint32_t k255, uint32_t& o0, uint32_t& o1,
                                            uint32_t& o2, uint32_t& o3, uint32_t& e01,
                                            uint32_t& c1, uint32_t& f01, uint32_t& f_cd) {
    uint32_t fab, fbc, AB, BC, CD, b1;
    asm("v_bitop3_b32 %9, %17, %16, %16 bitop3:0x30\n\t"   // bc
        "v_bitop3_b32 %7, %18, %16, %17 bitop3:0xd0\n\t"   // cd
        "v_lshrrev_b32 %8, 7, %16\n\t"                     // f_ab
        "v_lshrrev_b32 %9, 7, %9\n\t"                      // f_bc
        "v_lshrrev_b32 %7, 7, %7\n\t"                      // f_cd
        "v_mul_lo_u32 %10, %8, %19\n\t"                    // AB
        "v_mul_lo_u32 %11, %9, %19\n\t"                    // BC
        "v_mul_lo_u32 %12, %7, %19\n\t"                    // CD
        "v_add_u32 %13, %21, %9\n\t"                       // b1 = C1 + f_bc
        "v_add_u32 %5, %14, %7\n\t"                        // c1 = C2 + f_cd
        "v_add_u32 %0, %8, %15\n\t"                        // o0 = C0 + f_ab
        "v_or_b32 %6, %8, %9\n\t"                          // f01
        "v_bfi_b32 %1, %10, %5, %13\n\t"                   // o1
        "v_bfi_b32 %2, %11, %20, %5\n\t"                   // BC ? C3 : c1
        "v_bitop3_b32 %3, %20, %12, %12 bitop3:0x30\n\t"   // C3 & ~CD
        "v_bfi_b32 %4, %10, %0, %13\n\t"                   // e01
        "v_bfi_b32 %2, %10, %3, %2\n\t"                    // o2
        "v_bitop3_b32 %3, %3, %10, %11 bitop3:0x10"          // o3 = (C3 & ~CD) & ~AB & ~BC
        : "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3), "=&v"(e01), "=&v"(c1), "=&v"(f01),
          "=&v"(f_cd), "=&v"(fab), "=&v"(fbc), "=&v"(AB), "=&v"(BC), "=&v"(CD), "=&v"(b1)
        : "v"(C2), "v"(C0), "v"(ab), "v"(bc_raw), "v"(cd_raw), "v"(k255), "v"(C3), "v"(C1));
}

// bits [31:0] of {hi, lo} >> s
__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

// ------------------------------------------------------------------ random-policy draws (ABI v3)
// Step t of board g takes ONE 32-bit word w = word (t & 3) of the DOMAIN_RANDOM block t >> 2 (a
// Philox block per four steps).  Bits of w:
//   action              w >> 30                      (np.random.randint(4), src/dqn_lib.py:20)
//   spawn cell          k = floor((w << 3) * n / 2^32), bits 0..28: the k-th empty cell of the
//                       slid board in move-space line-major order (see lean_step)
//   spawn value         a 4 iff bit 29 is set (p(4) = 0.5, src/board.py:12,49)
//   auto-reset (terminal steps, which spawn nothing): first tile at cell (w >> 26) & 15, a 4 iff
//                       bit 25; second at the k2-th of the other 15 cells (row-major),
//                       k2 = floor((w << 8) * 15 / 2^32), a 4 iff bit 24
// With G2048_P4_10 the values come from two more blocks of the same quad, at counters
// (t >> 2) | 2^63 (v: the spawn and the reset's first tile) and (t >> 2) | 2^62 (v2: the reset's
// second tile), word t & 3 of each: a 4 iff v < round(0.1 * 2^32) -- exact 32-bit thresholds.
struct RandWords {
    uint32_t w, v, v2;
};

__device__ __forceinline__ uint32_t word_of(const uint4& u, uint32_t k) {
    return k == 0u ? u.x : k == 1u ? u.y : k == 2u ? u.z : u.w;
}

template <bool kP410>
__device__ __forceinline__ void value_blocks(uint32_t seed_lo, uint32_t seed_hi, uint64_t gid,
                                             uint64_t quad, uint4& vb, uint4& vb2) {
    if constexpr (kP410) {
        vb = draw(seed_lo, seed_hi, gid, DOMAIN_RANDOM, quad | (1ull << 63));
        vb2 = draw(seed_lo, seed_hi, gid, DOMAIN_RANDOM, quad | (1ull << 62));
    }
}

// The draws of step t (any t; the rollout kernels fetch one block per quad instead)
__device__ __forceinline__ RandWords random_words(uint32_t seed_lo, uint32_t seed_hi, uint64_t gid,
                                                  uint64_t t, bool p410) {
    const uint4 u = draw(seed_lo, seed_hi, gid, DOMAIN_RANDOM, t >> 2);
    RandWords r{word_of(u, (uint32_t)t & 3u), 0u, 0u};
    if (p410) {
        uint4 vb, vb2;
        value_blocks<true>(seed_lo, seed_hi, gid, t >> 2, vb, vb2);
        r.v = word_of(vb, (uint32_t)t & 3u);
        r.v2 = word_of(vb2, (uint32_t)t & 3u);
    }
    return r;
}

// Spawn exponent of a moving step: 2 (a "4") or 1 (a "2").
template <bool kP410>
__device__ __forceinline__ uint32_t spawn_exp(uint32_t w, uint32_t v, uint32_t p4_thresh) {
    if constexpr (kP410) return v < p4_thresh ? 2u : 1u;
    else return 1u + ((w >> 29) & 1u);
}

// Auto-reset board of a terminal random-policy step (bits: see above).  The two tiles are placed
// with 64-bit shifts into the board's halves {r0, r1} / {r2, r3}.
template <bool kP410>
__device__ __forceinline__ Board fresh_board_w(uint32_t w, uint32_t v, uint32_t v2,
                                               uint32_t p4_thresh) {
    const uint32_t ca = (w >> 26) & 15u;
    const uint32_t k2 = __umulhi(w << 8, 15u);
    const uint32_t cb = k2 + (uint32_t)(k2 >= ca);
    // a tile of exponent 1 + x is 1 << x: the value bit joins the 64-bit shift amount
    const uint32_t xa = kP410 ? (uint32_t)(v < p4_thresh) : (w >> 25) & 1u;
    const uint32_t xb = kP410 ? (uint32_t)(v2 < p4_thresh) : (w >> 24) & 1u;
    const uint64_t ta = 1ull << (((ca << 3) & 56u) + xa);
    const uint64_t tb = 1ull << (((cb << 3) & 56u) + xb);
    // half masks: bit 3 of the cell sign-extended (cells 8..15 live in {r2, r3})
    const uint32_t ma = (uint32_t)__builtin_amdgcn_sbfe((int32_t)ca, 3u, 1u);
    const uint32_t mb = (uint32_t)__builtin_amdgcn_sbfe((int32_t)cb, 3u, 1u);
    return Board{((uint32_t)ta & ~ma) | ((uint32_t)tb & ~mb),
                 ((uint32_t)(ta >> 32) & ~ma) | ((uint32_t)(tb >> 32) & ~mb),
                 ((uint32_t)ta & ma) | ((uint32_t)tb & mb),
                 ((uint32_t)(ta >> 32) & ma) | ((uint32_t)(tb >> 32) & mb)};
}

// The selector quads of action a from the constant table (the kernels that run one step per
// launch; the rollout stages the table in LDS).
__device__ __forceinline__ void dir_sel_const(uint32_t a, uint4& F, uint4& I) {
    const uint4* t = reinterpret_cast<const uint4*>(&kDirNet[0][0][0]);
    F = t[2u * a];
    I = t[2u * a + 1u];
}

// The same quads selected in registers (immediate operands, three v_cndmask per word): the
// one-launch-per-step kernel's table load was a dependent memory round trip (a fresh dispatch
// misses L1) between the step's action draw and its slide.
__device__ __forceinline__ uint32_t sel4(uint32_t a, uint32_t v0, uint32_t v1, uint32_t v2,
                                         uint32_t v3) {
    const uint32_t lo = (a & 1u) ? v1 : v0, hi = (a & 1u) ? v3 : v2;
    return (a & 2u) ? hi : lo;
}

__device__ __forceinline__ void dir_sel_reg(uint32_t a, uint4& F, uint4& I) {
#define G2048_SEL(h, k) sel4(a, kDirNetH[0][h][k], kDirNetH[1][h][k], kDirNetH[2][h][k], kDirNetH[3][h][k])
    constexpr uint32_t kDirNetH[4][2][4] = {
        {{0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u},
         {0x03020100u, 0x07060504u, 0x03020100u, 0x07060504u}},
        {{0x07060504u, 0x03020100u, 0x07060504u, 0x03020100u},
         {0x07060504u, 0x03020100u, 0x07060504u, 0x03020100u}},
        {{0x06020400u, 0x07030501u, 0x05040100u, 0x07060302u},
         {0x06020400u, 0x07030501u, 0x05040100u, 0x07060302u}},
        {{0x05010703u, 0x04000602u, 0x05040100u, 0x07060302u},
         {0x02060004u, 0x03070105u, 0x01000504u, 0x03020706u}},
    };
    F = make_uint4(G2048_SEL(0, 0), G2048_SEL(0, 1), G2048_SEL(0, 2), G2048_SEL(0, 3));
    I = make_uint4(G2048_SEL(1, 0), G2048_SEL(1, 1), G2048_SEL(1, 2), G2048_SEL(1, 3));
#undef G2048_SEL
}

// The random-policy transition of board b (rows) along the line words given by the selector
// quads F (rows -> lines) and I (lines -> rows): slide, terminal test of the board as given,
// spawn of exponent e (1 or 2) when the board moved.  The spawn cell is the k-th empty cell,
// k = floor((w << 3) * n / 2^32), in MOVE-SPACE LINE-MAJOR order: lines j = 0..3 (byte j of the
// line words), within a line positions q = 0..3 along the move -- after the slide a line's empties
// are its last E_j positions, so the k-th is line j* (the first with S_j* > k, S = inclusive
// prefix of E over lines) at position q = 4 + k - S_j*.  Any fixed order of the empty cells gives
// the reference's uniform choice (src/board.py:41-51); this one needs no search.  Returns the merge
// gain; done: the board as given was terminal (no legal move, src/dqn_lib.py:17-18).
// Domain: exponents < 32 (the 0x20-flag sums below; a 4x4 game cannot pass 17).
//   k255: 255, passed by the rollout kernels as an opaque loop-invariant register (expand01).
__device__ __forceinline__ uint32_t lean_step(Board& b, uint32_t w, uint32_t e, const uint4& F,
                                              const uint4& I, bool& done, uint32_t k255 = 255u) {
    uint32_t L0, L1, L2, L3;
    G2048_MARK(net_fwd, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
    dir_net(b.r0, b.r1, b.r2, b.r3, F, L0, L1, L2, L3);
    G2048_MARK(compact, "+v"(L0), "+v"(L1), "+v"(L2), "+v"(L3));
    // bit 7 of byte j of D_k: cell k of line j is empty
    const uint32_t D0 = K80 - L0, D1 = K80 - L1, D2 = K80 - L2;
    // 1) stable compaction toward L0, back to front
    const uint32_t M2 = zmask(D2);
    uint32_t C2 = bsel(M2, L3, L2), C3 = L3 & ~M2;
    const uint32_t M1 = zmask(D1);
    uint32_t C1 = bsel(M1, C2, L1);
    C2 = bsel(M1, C3, C2);
    C3 &= ~M1;
    const uint32_t M0 = zmask(D0);
    uint32_t C0 = bsel(M0, C1, L0);
    C1 = bsel(M0, C2, C1);
    C2 = bsel(M0, C3, C2);
    C3 &= ~M0;
    G2048_MARK(merge, "+v"(C0), "+v"(C1), "+v"(C2), "+v"(C3));
    // 2) merges, front first (the later cell is non-empty => so is the earlier one)
    //    (v_xad: bit 7 of (x ^ y) + 0x7F set iff the bytes differ; of y + 0x7F iff y != 0)
    uint32_t ab, bc_raw, cd_raw;
    pair_flags(C0, C1, C2, C3, ab, bc_raw, cd_raw);
    //    bc = bc_raw & ~ab (a+b taken first), cd = cd_raw & (ab | ~bc_raw) (c not used by b+c);
    //    then the merged line words o0..o3, and for the score (3): e01 = the exponents of the
    //    a+b or b+c merges (a line merges one or neither), c1 = of the c+d merges, and their 0x01
    //    flags f01, f_cd
    uint32_t o0, o1, o2, o3, e01, c1, f01, f_cd;
    merge_lines(C0, C1, C2, C3, ab, bc_raw, cd_raw, k255, o0, o1, o2, o3, e01, c1, f01, f_cd);
    G2048_MARK(score, "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
    // 3) score = sum of 2^e over the merged tiles: two words of candidates; shifting the 0x01
    //    merge flag (not 1) by each byte makes a line without a merge contribute 0 (so the
    //    exponent bytes need no mask)
    uint32_t gain = merge_gain(e01, f01, c1, f_cd);
    G2048_MARK(moved_done, "+v"(gain));
    // 4) moved: a hole before a tile along a line, or a merge
    const uint32_t N3 = L3 + K7F;  // bit 7: cell 3 holds a tile
    uint32_t mv = moved_flags(D0, D1, D2, N3, ab | bc_raw | cd_raw);
    G2048_MARK(spawn, "+v"(mv));
    // 5) spawn in line space (see above)
    uint32_t n, j8, q;
    spawn_slot(M0, M1, M2, N3, f01, f_cd, w, n, j8, q);
    // the tile min(e, mv) (mv is 0 -- no move, no spawn -- or >= 0x80) at bit 8 j* + 32 (q & 1)
    // of the half {o0, o1} (q & 2 clear) or {o2, o3}: v_lshlrev_b64 reads 6 bits of the shift,
    // and the half's mask is bit 1 of q sign-extended (without a move the tile is 0)
    const uint64_t tile = (uint64_t)min(e, mv) << ((q << 5) + j8);
    const uint32_t qm = (uint32_t)__builtin_amdgcn_sbfe((int32_t)q, 1u, 1u);
    o0 |= (uint32_t)tile & ~qm;
    o1 |= (uint32_t)(tile >> 32) & ~qm;
    o2 |= (uint32_t)tile & qm;
    o3 |= (uint32_t)(tile >> 32) & qm;
    // 6) terminal (board as given, src/dqn_lib.py:17-18): no empty cell after a non-move (a move
    //    always leaves one, so n == 0 iff nothing moved and the board is full) and no equal
    //    neighbours across the lines (adjacent bytes of a line word; v_xad: bit 7 of
    //    (x ^ y) + 0x7F is set iff the bytes differ) -- or the board is empty (16 empties, n mod
    //    16 = 0).  The empty board's zero bytes compare equal in across_pairs, so its flags are
    //    masked with N3 (bit 7 of byte j: cell 3 of line j holds a tile), which is all ones on a
    //    full board -- the only other board with n == 0 -- and zero on the empty one.
    done = (n | (across_pairs(L0, L1, L2, L3) & N3)) == 0u;
    // 7) back to rows
    G2048_MARK(net_inv, "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
    dir_net(o0, o1, o2, o3, I, b.r0, b.r1, b.r2, b.r3);
    G2048_MARK(stores, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
    return gain;
}

}  // namespace g2048
