// VALU throughput classes on gfx950 with one and with two waves per SIMD.  A 512-thread workgroup
// holds waves 0-7; wave w and wave w + 4 share a SIMD (checked through HW_ID).  Each test runs a
// block of 200 instructions of one kind (8 independent chains) per wave, then an s_barrier, 64
// times.  "solo": only waves 0-3 run the stream (4-7 just meet the barriers); "pair": all eight
// run it.  Cycles per instruction per SIMD = block cycles / instructions the SIMD executed.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pairbench.hip -o tools/pairbench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define R8(OP) OP(x0) OP(x1) OP(x2) OP(x3) OP(x4) OP(x5) OP(x6) OP(x7)
#define O_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(x1));
#define O_SUB(x) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(x) : "s"(c));
#define O_AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(x2));
#define O_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(x2));
#define O_LSHR(x) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x));
#define O_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "s"(c));
#define O_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "v"(x4));
#define O_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(x3), "s"(c));
#define O_OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "v"(x4));
#define O_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "v"(x4));
#define O_MIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(x3));
#define O_BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(x3));
#define O_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "s"(c));
#define O_SDWA(x) asm volatile("v_lshlrev_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(x) : "v"(x3));
#define O_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, s[20:21]" : "+v"(x) : "v"(x3));
#define O_LSHL64(x) asm volatile("v_lshlrev_b64 v[40:41], %0, v[40:41]" : : "v"(x) : "v40", "v41");
#define O_MOV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x3));
#define O_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(x3));
#define O_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "v"(x4));
#define O_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x) : "v"(x3));
#define O_PKADD(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(x3));
#define O_SALU(x) asm volatile("s_mul_i32 %0, %0, 3" : "+s"(s0));
#define O_FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(x3), "v"(x4));

#define KERN(NAME, OP)                                                                        \
    __global__ __launch_bounds__(512) void NAME(uint32_t* out, unsigned long long* cyc,       \
                                                uint32_t* hwid, int pair) {                   \
        const int w = threadIdx.x >> 6;                                                       \
        const bool run = __builtin_amdgcn_readfirstlane(w < 4 || pair) != 0;                  \
        uint32_t x0 = threadIdx.x, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u, x4 = x0 + 11u,    \
                 x5 = x0 + 13u, x6 = x0 ^ 17u, x7 = x0 ^ 19u, s0 = blockIdx.x;                 \
        const uint32_t c = 0x05010400u;                                                        \
        asm volatile("s_mov_b64 s[20:21], -1" ::: "s20", "s21");                              \
        __syncthreads();                                                                       \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                             \
        for (int b = 0; b < 64; ++b) {                                                          \
            if (run) {                                                                          \
                _Pragma("unroll") for (int i = 0; i < 25; ++i) { R8(OP) }                       \
            }                                                                                   \
            __syncthreads();                                                                    \
        }                                                                                       \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                             \
        out[blockIdx.x * 512 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ s0;      \
        if ((threadIdx.x & 63) == 0) {                                                         \
            cyc[blockIdx.x * 8 + w] = t1 - t0;                                                  \
            hwid[blockIdx.x * 8 + w] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)); \
        }                                                                                       \
    }

KERN(k_add, O_ADD)
KERN(k_sub, O_SUB)
KERN(k_and, O_AND)
KERN(k_xor, O_XOR)
KERN(k_lshr, O_LSHR)
KERN(k_perm, O_PERM)
KERN(k_bfi, O_BFI)
KERN(k_bitop3, O_BITOP3)
KERN(k_or3, O_OR3)
KERN(k_add3, O_ADD3)
KERN(k_min, O_MIN)
KERN(k_bcnt, O_BCNT)
KERN(k_mulhi, O_MULHI)
KERN(k_sdwa, O_SDWA)
KERN(k_cnd, O_CND)
KERN(k_lshl64, O_LSHL64)
KERN(k_mov, O_MOV)
KERN(k_align, O_ALIGN)
KERN(k_andor, O_ANDOR)
KERN(k_lshlor, O_LSHLOR)
KERN(k_pkadd, O_PKADD)
KERN(k_salu, O_SALU)
KERN(k_fma, O_FMA)

int main() {
    const int wgs = 256;
    uint32_t *out, *hw;
    unsigned long long* cyc;
    (void)hipMalloc(&out, wgs * 512 * 4);
    (void)hipMalloc(&cyc, wgs * 8 * 8);
    (void)hipMalloc(&hw, wgs * 8 * 4);
    std::vector<unsigned long long> h(wgs * 8);
    std::vector<uint32_t> hh(wgs * 8);
    struct K {
        const char* name;
        void (*fn)(uint32_t*, unsigned long long*, uint32_t*, int);
    } ks[] = {{"v_add_u32", k_add},       {"v_sub_u32", k_sub},         {"v_and_b32", k_and},
              {"v_xor_b32", k_xor},       {"v_lshrrev_b32", k_lshr},    {"v_perm_b32", k_perm},
              {"v_bfi_b32", k_bfi},       {"v_bitop3_b32", k_bitop3},   {"v_or3_b32", k_or3},
              {"v_add3_u32", k_add3},     {"v_min_u32", k_min},         {"v_bcnt_u32_b32", k_bcnt},
              {"v_mul_hi_u32", k_mulhi},  {"v_lshlrev_b32_sdwa", k_sdwa}, {"v_cndmask_b32 (sgpr)", k_cnd},
              {"v_lshlrev_b64", k_lshl64}, {"v_mov_b32", k_mov},        {"v_alignbit_b32", k_align},
              {"v_and_or_b32", k_andor},  {"v_lshl_or_b32", k_lshlor},  {"v_pk_add_u16", k_pkadd},
              {"s_mul_i32 (SALU)", k_salu}, {"v_fma_f32", k_fma}};
    int same = 0;
    printf("%-22s %14s %14s\n", "instruction", "1 wave/SIMD", "2 waves/SIMD");
    for (auto& k : ks) {
        double res[2];
        for (int pair = 0; pair < 2; ++pair) {
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(k.fn, dim3(wgs), dim3(512), 0, 0, out, cyc, hw, pair);
            (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(hh.data(), hw, hh.size() * 4, hipMemcpyDeviceToHost);
            double a = 0;
            for (int g = 0; g < wgs; ++g)
                for (int w = 0; w < 4; ++w) {
                    a += (double)h[g * 8 + w];
                    same += ((hh[g * 8 + w] >> 4) & 3) == ((hh[g * 8 + 4 + w] >> 4) & 3);
                }
            a /= wgs * 4;
            res[pair] = a / (64 * 200.0 * (pair ? 2 : 1));  // cycles per instruction per SIMD
        }
        printf("%-22s %10.2f cyc %10.2f cyc   (per SIMD-instruction, barrier every 200)\n", k.name,
               res[0], res[1]);
    }
    printf("wave w / w+4 on one SIMD: %d of %d checks\n", same,
           (int)(sizeof(ks) / sizeof(ks[0])) * 2 * wgs * 4);
    return 0;
}
