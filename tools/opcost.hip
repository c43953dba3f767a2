// Issue cost of single VALU instructions for ONE wave per SIMD on gfx950: 256 workgroups of 4
// waves, each wave runs a loop of 8 independent (or 8 dependent) copies of one instruction;
// s_memtime around the loop gives shader cycles per instruction.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/opcost.hip -o tools/opcost
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

constexpr int kIters = 4096;  // long enough that all resident waves overlap

// independent: x[k] = op(x[k], ...) for k = 0..7 (a chain of length kIters per register, 8 chains)
#define KERNEL(NAME, ASM)                                                                   \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* cyc) {   \
        uint32_t x0 = threadIdx.x, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u, x4 = x0 + 11u,   \
                 x5 = x0 + 13u, x6 = x0 ^ 17u, x7 = x0 ^ 19u;                                 \
        uint64_t y0 = x0, y1 = x1, y2 = x2, y3 = x3, y4 = x4, y5 = x5, y6 = x6, y7 = x7;      \
        (void)y0; (void)y1; (void)y2; (void)y3; (void)y4; (void)y5; (void)y6; (void)y7;      \
        const uint32_t c = 0xD2511F53u;                                                       \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                            \
        for (int it = 0; it < kIters; ++it) {                                                  \
            ASM                                                                                \
        }                                                                                      \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                            \
        out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^          \
                                             (uint32_t)(y0 ^ y1 ^ y2 ^ y3 ^ y4 ^ y5 ^ y6 ^ y7);  \
        if ((threadIdx.x & 63) == 0) {                                                         \
            cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = t0;                                   \
            cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = t1;                               \
        }                                                                                      \
    }

#define I_ADD(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##k) : "v"(x##k));
#define I_PERM(k) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x##k) : "s"(c));
#define I_BITOP3(k) asm volatile("v_bitop3_b32 %0, %0, %0, %1 bitop3:0x96" : "+v"(x##k) : "s"(c));
#define I_MULHI(k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x##k) : "s"(c));
#define I_MULLO(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x##k) : "s"(c));
#define I_MUL24(k) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x##k) : "s"(c));
#define I_MAD64(k) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(y##k) : "v"((uint32_t)y##k), "s"(c) : "vcc");
#define I_SHL64(k) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(y##k) : "v"(x##k));
#define I_CND(k) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x##k) : "v"(x##k));
#define I_SDWA(k) asm volatile("v_lshlrev_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(x##k) : "v"(x##k));
#define I_BCNT(k) asm volatile("v_bcnt_u32_b32 %0, %0, 0" : "+v"(x##k));
#define I_ALIGN(k) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x##k));
#define I_CMPCND(k) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x##k) : "v"(x##k) : "vcc");
#define I_DOT4(k) asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(x##k) : "v"(x##k));
#define I_SADU8(k) asm volatile("v_sad_u8 %0, %0, %1, %0" : "+v"(x##k) : "v"(x##k));
#define I_PKADD(k) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x##k) : "v"(x##k));
#define I_MOV64(k) asm volatile("v_mov_b64 %0, %1" : "=v"(y##k) : "v"(y##k));
#define I_LSHLADD(k) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x##k) : "v"(x##k));

KERNEL(k_add, REP8(I_ADD))
KERNEL(k_perm, REP8(I_PERM))
KERNEL(k_bitop3, REP8(I_BITOP3))
KERNEL(k_mulhi, REP8(I_MULHI))
KERNEL(k_mullo, REP8(I_MULLO))
KERNEL(k_mul24, REP8(I_MUL24))
KERNEL(k_mad64, REP8(I_MAD64))
KERNEL(k_shl64, REP8(I_SHL64))
KERNEL(k_cnd, REP8(I_CND))
KERNEL(k_sdwa, REP8(I_SDWA))
KERNEL(k_bcnt, REP8(I_BCNT))
KERNEL(k_align, REP8(I_ALIGN))
KERNEL(k_cmpcnd, REP8(I_CMPCND))
KERNEL(k_dot4, REP8(I_DOT4))
KERNEL(k_sad, REP8(I_SADU8))
KERNEL(k_pkadd, REP8(I_PKADD))
KERNEL(k_mov64, REP8(I_MOV64))
KERNEL(k_lshladd, REP8(I_LSHLADD))
// mixes: 8 independent adds + other instruction types per body
#define I_SALU(k) asm volatile("s_mul_i32 %0, %0, 3" : "+s"(sc##k));  // leaves SCC alone
#define I_DSR(k) asm volatile("ds_read_b32 %0, %1" : "=v"(lv##k) : "v"(0u));
#define I_DSW(k) asm volatile("ds_write_b32 %0, %1" : : "v"(0u), "v"(x##k));
#define KERNEL_MIX(NAME, ASM)                                                               \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* cyc) {   \
        __shared__ uint32_t lds[64];                                                         \
        if (threadIdx.x < 64) lds[threadIdx.x] = threadIdx.x;                                \
        __syncthreads();                                                                     \
        uint32_t x0 = threadIdx.x, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u, x4 = x0 + 11u,   \
                 x5 = x0 + 13u, x6 = x0 ^ 17u, x7 = x0 ^ 19u;                                 \
        uint32_t sc0 = blockIdx.x, sc1 = sc0 + 1, sc2 = sc0 + 2, sc3 = sc0 + 3;               \
        uint32_t lv0 = 0, lv1 = 0, lv2 = 0, lv3 = 0;                                         \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                            \
        for (int it = 0; it < kIters; ++it) {                                                  \
            ASM                                                                                \
        }                                                                                      \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                            \
        out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ sc0 ^    \
                                             sc1 ^ sc2 ^ sc3 ^ lv0 ^ lv1 ^ lv2 ^ lv3;          \
        if ((threadIdx.x & 63) == 0) {                                                         \
            cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = t0;                                   \
            cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = t1;                               \
        }                                                                                      \
    }
#define A8 REP8(I_ADD)
KERNEL_MIX(k_mix_add, A8)
KERNEL_MIX(k_mix_salu2, A8 I_SALU(0) I_SALU(1))
KERNEL_MIX(k_mix_salu4, A8 I_SALU(0) I_SALU(1) I_SALU(2) I_SALU(3))
KERNEL_MIX(k_mix_dsr2, A8 I_DSR(0) I_DSR(1))
KERNEL_MIX(k_mix_dsw2, A8 I_DSW(0) I_DSW(1))
// dependent chains: one register, 8 ops in a row
#define D8(X) X(0) X(0) X(0) X(0) X(0) X(0) X(0) X(0)
KERNEL(k_add_dep, D8(I_ADD))
KERNEL(k_perm_dep, D8(I_PERM))
KERNEL(k_mulhi_dep, D8(I_MULHI))
KERNEL(k_mad64_dep, D8(I_MAD64))
KERNEL(k_sdwa_dep, D8(I_SDWA))
KERNEL(k_cmpcnd_dep, D8(I_CMPCND))

int main(int argc, char** argv) {
    const int wgs = argc > 1 ? atoi(argv[1]) : 256;
    uint32_t* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, (size_t)wgs * 256 * 4);
    (void)hipMalloc(&cyc, (size_t)wgs * 4 * 16);
    std::vector<unsigned long long> h((size_t)wgs * 8);
    struct K {
        const char* name;
        void (*fn)(uint32_t*, unsigned long long*);
        int per;  // instructions per loop body copy
    } ks[] = {{"v_add_u32", k_add, 1},           {"v_perm_b32", k_perm, 1},
              {"v_bitop3_b32", k_bitop3, 1},     {"v_mul_hi_u32", k_mulhi, 1},
              {"v_mul_lo_u32", k_mullo, 1},      {"v_mul_u32_u24", k_mul24, 1},
              {"v_mad_u64_u32", k_mad64, 1},     {"v_lshlrev_b64", k_shl64, 1},
              {"v_cndmask_b32", k_cnd, 1},       {"v_lshlrev_b32_sdwa", k_sdwa, 1},
              {"v_bcnt_u32_b32", k_bcnt, 1},     {"v_alignbit_b32", k_align, 1},
              {"v_cmp+v_cndmask", k_cmpcnd, 2},  {"v_dot4_u32_u8", k_dot4, 1},
              {"v_sad_u8", k_sad, 1},            {"v_pk_add_u16", k_pkadd, 1},
              {"v_mov_b64", k_mov64, 1},         {"v_lshl_add_u32", k_lshladd, 1},
              {"DEP v_add_u32", k_add_dep, 1},   {"DEP v_perm_b32", k_perm_dep, 1},
              {"DEP v_mul_hi_u32", k_mulhi_dep, 1}, {"DEP v_mad_u64_u32", k_mad64_dep, 1},
              {"DEP v_lshlrev_sdwa", k_sdwa_dep, 1}, {"DEP v_cmp+v_cndmask", k_cmpcnd_dep, 2},
              {"MIX 8 add", k_mix_add, 1}, {"MIX 8 add + 2 s_add", k_mix_salu2, 1},
              {"MIX 8 add + 4 s_add", k_mix_salu4, 1}, {"MIX 8 add + 2 ds_read", k_mix_dsr2, 1},
              {"MIX 8 add + 2 ds_write", k_mix_dsw2, 1}};
    printf("%d workgroups of 4 waves (%.1f waves per SIMD); per-wave cycles per VALU instruction\n", wgs, wgs / 256.0);
    for (int rep = 0; rep < 2; ++rep)
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.fn, dim3(wgs), dim3(256), 0, 0, out, cyc);
            (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            if (rep == 0) continue;
            unsigned long long lo = ~0ull, hi = 0;
            double sum = 0;
            for (int w = 0; w < wgs * 4; ++w) {
                lo = std::min(lo, h[2 * w]);
                hi = std::max(hi, h[2 * w + 1]);
                sum += (double)(h[2 * w + 1] - h[2 * w]);
            }
            const double per = 4096.0 * 8.0 * k.per;
            printf("%-24s per wave %6.2f cyc/instr   span %6.2f cyc/instr (x %.1f waves/SIMD = %5.2f cyc per SIMD-instr)\n",
                   k.name, sum / (wgs * 4) / per, (hi - lo) / per, wgs / 256.0,
                   (hi - lo) / per / (wgs / 256.0));
        }
    return 0;
}
