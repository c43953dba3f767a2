// g2048_roll.hpp -- the random-policy step of the rollout kernel (k_rollout_lean), rewritten for
// the instruction budget of ONE wave per SIMD (64k boards on 256 CUs).  Measured on gfx950
// (tools/opcost.hip, tools/pairbench.hip): with one wave per SIMD every VALU op costs one issue
// turn of ~5.1-5.9 shader cycles whatever it computes, v_mad_u64_u32 / v_lshlrev_b64 / v_mov
// cost 8-10, SALU ops 8-10; a second wave per SIMD adds throughput only for plain VOP2 ops.  So the
// step is bound by its instruction count, and this file minimises it.  Same results as
// random_step + fresh_board_random (g2048_board.hpp), bit for bit (tests/test_env_gpu.py and
// tools/rollexp.hip compare the two kernels on every output).
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

// bits [31:0] of {hi, lo} >> s
__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

// The random-policy transition of board b (rows) along the line words given by the selector
// quads F (rows -> lines) and I (lines -> rows): slide, terminal test of the board as given,
// spawn (k-th empty cell of the result in row-major order, spawn_at) when the board moved.
// Returns the merge gain; done as random_step.
__device__ __forceinline__ uint32_t lean_step(Board& b, uint32_t wa, uint32_t wb,
                                              uint32_t p4_thresh, const uint4& F, const uint4& I,
                                              bool& done) {
    uint32_t L0, L1, L2, L3;
    G2048_MARK(net_fwd, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
    dir_net(b.r0, b.r1, b.r2, b.r3, F, L0, L1, L2, L3);
    G2048_MARK(compact, "+v"(L0), "+v"(L1), "+v"(L2), "+v"(L3));
    // bit 7 of byte j of D_k: cell k of line j is empty
    const uint32_t D0 = K80 - L0, D1 = K80 - L1, D2 = K80 - L2, D3 = K80 - L3;
    // 1) stable compaction toward L0, back to front
    uint32_t M = zmask(D2);
    uint32_t C2 = bsel(M, L3, L2), C3 = L3 & ~M;
    M = zmask(D1);
    uint32_t C1 = bsel(M, C2, L1);
    C2 = bsel(M, C3, C2);
    C3 &= ~M;
    M = zmask(D0);
    uint32_t C0 = bsel(M, C1, L0);
    C1 = bsel(M, C2, C1);
    C2 = bsel(M, C3, C2);
    C3 &= ~M;
    G2048_MARK(merge, "+v"(C0), "+v"(C1), "+v"(C2), "+v"(C3));
    // 2) merges, front first (the later cell is non-empty => so is the earlier one)
    //    (v_xad: bit 7 of (x ^ y) + 0x7F set iff the bytes differ; of y + 0x7F iff y != 0)
    const uint32_t ab = ~xad(C0, C1, K7F) & (C1 + K7F) & K80;
    const uint32_t bc_raw = ~xad(C1, C2, K7F) & (C2 + K7F) & K80;
    const uint32_t cd_raw = ~xad(C2, C3, K7F) & (C3 + K7F) & K80;
    const uint32_t bc = bc_raw & ~ab;
    const uint32_t cd = cd_raw & (ab | ~bc_raw);
    const uint32_t AB = expand80(ab), BC = expand80(bc), CD = expand80(cd);
    const uint32_t c1 = C2 + (cd >> 7);
    const uint32_t b1 = C1 + (bc >> 7);
    uint32_t o0 = C0 + (ab >> 7);
    uint32_t o1 = bsel(AB, c1, b1);
    uint32_t o2 = bsel(AB, C3 & ~CD, bsel(BC, C3, c1));
    uint32_t o3 = C3 & ~(AB | BC | CD);
    G2048_MARK(score, "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
    const uint32_t e01 = (o0 & AB) | (b1 & BC), e2 = c1 & CD;
    uint32_t gain = (pow2_bytes(e01) + pow2_bytes(e2)) -
                          (8u - (uint32_t)(__popc(ab | bc) + __popc(cd)));
    G2048_MARK(moved_done, "+v"(gain));
    // 3) moved: a hole before a tile along a line, or a merge
    const uint32_t hb = ((D0 & ~D1) | (D1 & ~D2) | (D2 & ~D3)) & K80;
    uint32_t mv = hb | or3_v(ab, bc_raw, cd_raw);
    // 4) terminal (board as given): nothing moves along these lines, no empty cell, no equal
    //    neighbours across them (adjacent bytes of a line word; v_xad: bit 7 of (x ^ y) + 0x7F
    //    is set iff the bytes differ), or the board is empty
    const uint32_t Y0 = xad(L0, alignbit(L1, L0, 8u), K7F), Y1 = xad(L1, alignbit(L2, L1, 8u), K7F);
    const uint32_t Y2 = xad(L2, alignbit(L3, L2, 8u), K7F), Y3 = xad(L3, L3 >> 8, K7F);
    const uint32_t across = ~(Y0 & Y1 & Y2 & Y3) & 0x00808080u;
    const uint32_t zany = (D0 | D1 | D2 | D3) & K80;
    done = min(or3_v(mv, zany, across), or3_v(L0, L1, L2 | L3)) == 0u;
    // 5) back to rows, spawn iff moved (min(e, mv) = 0 iff mv == 0: mv is 0 or >= 0x80)
    G2048_MARK(net_inv, "+v"(mv));
    dir_net(o0, o1, o2, o3, I, b.r0, b.r1, b.r2, b.r3);
    G2048_MARK(spawn, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
    spawn_at(b, wa << 2, min(wb < p4_thresh ? 2u : 1u, mv));
    G2048_MARK(stores, "+v"(b.r0), "+v"(b.r1), "+v"(b.r2), "+v"(b.r3));
    return gain;
}

}  // namespace g2048
