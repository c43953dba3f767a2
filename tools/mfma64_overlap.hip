// Does VALU work hide under f64 MFMAs on gfx950?  The fused float64 conv learner runs one wave
// per SIMD and spends about a third of each tile in VALU / LDS phases between its MFMA phases
// (DESIGN §4.7); the eight-wave train A (two waves per SIMD) did not overlap them.  This probe
// measures, with s_memtime around each wave's loop (256 workgroups, one per CU):
//   same wave : 4 MFMA chains (v_mfma_f64_16x16x4_f64, VGPR accumulators), each MFMA followed by
//               NV independent VALU ops of one kind -> ticks per MFMA (64 = the VALU is hidden)
//   two waves : waves 0-3 run the MFMA-only loop, waves 4-7 (the same four SIMDs) a VALU-only loop
//               of 4*NV ops per iteration, the same iteration count -> ticks per iteration of each
//   VALU only : the VALU loop alone at one wave per SIMD (the issue cost to compare with)
//   and the two-wave case with the VALU waves as the older half, or at s_setprio 3, or with the
//   MFMA waves' loop as one asm block with the accumulators in AGPRs (or VGPRs); and the VALU
//   loop at two waves per SIMD (the SIMD's VALU throughput with a second wave)
// Kinds: v_add_u32, v_fma_f64, v_pk_fma_f32; the same with v_mfma_f32_16x16x4_f32 (32 cycles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma64_overlap.hip -o tools/mfma64_overlap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
struct Valu {
    unsigned u[8];
    double d[8];
    f2 p[8];
    __device__ void init(int l) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u[k] = l * 7u + k;
            d[k] = 1.0 + l * 1e-9 + k * 1e-7;
            p[k] = f2{1.0f + k * 1e-3f, 1.0f - l * 1e-6f};
        }
    }
    __device__ __forceinline__ void op(int k) {
        if constexpr (KIND == 0) asm volatile("v_add_u32 %0, %0, %0" : "+v"(u[k & 7]));
        if constexpr (KIND == 1) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[k & 7]));
        if constexpr (KIND == 2) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p[k & 7]));
    }
    __device__ double sum() const {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += u[k] + d[k] + p[k][0] + p[k][1];
        return s;
    }
};

typedef float f4 __attribute__((ext_vector_type(4)));
// F32 = false: v_mfma_f64_16x16x4_f64 (64 cycles); true: v_mfma_f32_16x16x4_f32 (32 cycles)
template <bool F32>
struct Acc {
    d4 c;
    f4 cf;
    __device__ void zero() {
        c = d4{0, 0, 0, 0};
        cf = f4{0, 0, 0, 0};
    }
    __device__ __forceinline__ void mfma(double a, double b) {
        if constexpr (F32)
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(cf) : "v"((float)a), "v"((float)b));
        else
            asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    }
    __device__ double get(int k) const { return c[k] + cf[k]; }
};

// The MFMA wave's whole loop as one asm block, accumulators pinned in AGPRs (kAgpr) or VGPRs.
#define MF64(i) "v_mfma_f64_16x16x4_f64 %" #i ", %[a], %[b], %" #i "\n\t"
#define MF32(i) "v_mfma_f32_16x16x4_f32 %" #i ", %[af], %[bf], %" #i "\n\t"
#define LOOP_HEAD "1:\n\t"
#define LOOP_TAIL "s_sub_u32 %[n], %[n], 1\n\ts_cmp_lg_u32 %[n], 0\n\ts_cbranch_scc1 1b\n\t"
template <bool F32, bool kAgpr>
__device__ __forceinline__ double mfma_loop(double a, double b, int iters) {
    unsigned n = (unsigned)iters;
    const float af = (float)a, bf = (float)b;
    if constexpr (F32) {
        f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        if constexpr (kAgpr)
            asm volatile(LOOP_HEAD MF32(0) MF32(1) MF32(2) MF32(3) LOOP_TAIL
                         : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), [n] "+s"(n)
                         : [af] "v"(af), [bf] "v"(bf) : "scc");
        else
            asm volatile(LOOP_HEAD MF32(0) MF32(1) MF32(2) MF32(3) LOOP_TAIL
                         : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), [n] "+s"(n)
                         : [af] "v"(af), [bf] "v"(bf) : "scc");
        return c0[0] + c1[1] + c2[2] + c3[3];
    } else {
        d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        if constexpr (kAgpr)
            asm volatile(LOOP_HEAD MF64(0) MF64(1) MF64(2) MF64(3) LOOP_TAIL
                         : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), [n] "+s"(n)
                         : [a] "v"(a), [b] "v"(b) : "scc");
        else
            asm volatile(LOOP_HEAD MF64(0) MF64(1) MF64(2) MF64(3) LOOP_TAIL
                         : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), [n] "+s"(n)
                         : [a] "v"(a), [b] "v"(b) : "scc");
        return c0[0] + c1[1] + c2[2] + c3[3];
    }
}

// MODE 0: every wave MFMA + NV VALU per MFMA.  MODE 1: waves < 4 MFMA only, waves >= 4 VALU only
// (4*NV per iteration).  MODE 2: VALU only (4*NV per iteration), every wave.
template <int MODE, int NV, int KIND, bool F32>
__global__ __launch_bounds__(512) void kmix(double* out, unsigned long long* ticks, int iters) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    Acc<F32> c0, c1, c2, c3;
    c0.zero();
    c1.zero();
    c2.zero();
    c3.zero();
    const float af = (float)a, bf = (float)b;
    (void)af;
    (void)bf;
    Valu<KIND> v;
    v.init(l);
    // MODE 3: the roles of MODE 1 swapped (the VALU waves are the older half); MODE 4: MODE 1
    // with the VALU waves at s_setprio 3
    const bool do_mfma = MODE == 0 || ((MODE == 1 || MODE == 4) && w < 4) || (MODE == 3 && w >= 4);
    const bool do_valu = MODE == 0 || MODE == 2 || MODE == 7 || ((MODE == 1 || MODE == 4) && w >= 4) ||
                         (MODE == 3 && w < 4);
    if (MODE == 4 && do_valu) __builtin_amdgcn_s_setprio(3);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double extra = 0;
    if (MODE == 5 || MODE == 6) {  // MODE 1 with the asm-loop MFMA waves: 5 AGPR, 6 VGPR accumulators
        if (w < 4)
            extra = mfma_loop<F32, MODE == 5>(a, b, iters);
        else
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int k = 0; k < 4 * NV; ++k) v.op(k);
            }
    } else if (do_mfma && do_valu) {
        for (int it = 0; it < iters; ++it) {
            c0.mfma(a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(k);
            c1.mfma(a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(1 * NV + k);
            c2.mfma(a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(2 * NV + k);
            c3.mfma(a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(3 * NV + k);
        }
    } else if (do_mfma) {
        for (int it = 0; it < iters; ++it) {
            c0.mfma(a, b);
            c1.mfma(a, b);
            c2.mfma(a, b);
            c3.mfma(a, b);
        }
    } else {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 4 * NV; ++k) v.op(k);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = c0.get(0) + c1.get(1) + c2.get(2) + c3.get(3) + v.sum() + extra;
    if (l == 0) ticks[blockIdx.x * 8 + w] = t1 - t0;
    // SIMD of this wave (HW_ID bits 5:4) for block 0, to check the two-wave pairing
    if (MODE == 1 && blockIdx.x == 0 && l == 0)
        ticks[256 * 8 + w] = (unsigned)__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);
}

template <int MODE, int NV, int KIND, bool F32>
void run(double* d, unsigned long long* tk, int iters, const char* kind) {
    const int nt = (MODE == 1 || MODE >= 3) ? 512 : 256;  // MODE 7: VALU only, two waves per SIMD
    kmix<MODE, NV, KIND, F32><<<256, nt>>>(d, tk, iters / 4);  // warm
    kmix<MODE, NV, KIND, F32><<<256, nt>>>(d, tk, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long h[256 * 8 + 8];
    (void)hipMemcpy(h, tk, sizeof h, hipMemcpyDeviceToHost);
    double lo = 0, hi = 0;  // average ticks of waves 0-3 and 4-7
    for (int g = 0; g < 256; ++g)
        for (int w = 0; w < 8; ++w) (w < 4 ? lo : hi) += (double)h[g * 8 + w];
    lo /= 1024.0 * iters;
    hi /= 1024.0 * iters;
    if (MODE == 0)
        printf("%s same wave  %-12s NV %2d : %6.1f ticks per MFMA (%5.1f per iteration of 4)\n",
               F32 ? "f32" : "f64", kind, NV, lo / 4, lo);
    else if (MODE == 1) {
        if (NV == 1) {
            printf("two waves: SIMD of waves 0..7 in workgroup 0:");
            for (int w = 0; w < 8; ++w) printf(" %llu", h[256 * 8 + w]);
            printf("\n");
        }
        printf("%s two waves  %-12s NV %2d : MFMA wave %6.1f, VALU wave %6.1f ticks per iteration\n",
               F32 ? "f32" : "f64", kind, NV, lo, hi);
    } else if (MODE == 7) {
        printf("%s VALU only, two waves per SIMD  %-12s NV %2d : %6.1f / %6.1f ticks per iteration of each wave (%4.2f per op per SIMD)\n",
               F32 ? "f32" : "f64", kind, NV, lo, hi, 0.5 * (lo + hi) / (2 * 4 * NV));
    } else if (MODE >= 5) {
        printf("%s two waves  %-12s NV %2d : MFMA wave %6.1f, VALU wave %6.1f ticks per iteration (asm loop, acc %s)\n",
               F32 ? "f32" : "f64", kind, NV, lo, hi, MODE == 5 ? "AGPR" : "VGPR");
    } else if (MODE >= 3) {
        const double mf = MODE == 3 ? hi : lo, va = MODE == 3 ? lo : hi;
        printf("%s two waves  %-12s NV %2d : MFMA wave %6.1f, VALU wave %6.1f ticks per iteration (%s)\n",
               F32 ? "f32" : "f64", kind, NV, mf, va, MODE == 3 ? "VALU wave older" : "VALU wave s_setprio 3");
    } else
        printf("%s VALU only  %-12s NV %2d : %6.1f ticks per iteration (%4.1f per op)\n",
               F32 ? "f32" : "f64", kind, NV, lo, lo / (4 * NV));
}

template <int KIND, bool F32>
void sweep(double* d, unsigned long long* tk, int iters, const char* kind) {
    run<0, 0, KIND, F32>(d, tk, iters, kind);
    run<0, 1, KIND, F32>(d, tk, iters, kind);
    run<0, 2, KIND, F32>(d, tk, iters, kind);
    run<0, 4, KIND, F32>(d, tk, iters, kind);
    run<0, 8, KIND, F32>(d, tk, iters, kind);
    run<2, 1, KIND, F32>(d, tk, iters, kind);
    run<2, 4, KIND, F32>(d, tk, iters, kind);
    run<2, 8, KIND, F32>(d, tk, iters, kind);
    run<1, 1, KIND, F32>(d, tk, iters, kind);
    run<1, 2, KIND, F32>(d, tk, iters, kind);
    run<1, 4, KIND, F32>(d, tk, iters, kind);
    run<1, 8, KIND, F32>(d, tk, iters, kind);
    run<3, 1, KIND, F32>(d, tk, iters, kind);
    run<3, 4, KIND, F32>(d, tk, iters, kind);
    run<3, 8, KIND, F32>(d, tk, iters, kind);
    run<4, 1, KIND, F32>(d, tk, iters, kind);
    run<4, 4, KIND, F32>(d, tk, iters, kind);
    run<4, 8, KIND, F32>(d, tk, iters, kind);
    run<5, 1, KIND, F32>(d, tk, iters, kind);
    run<5, 4, KIND, F32>(d, tk, iters, kind);
    run<5, 8, KIND, F32>(d, tk, iters, kind);
    run<6, 1, KIND, F32>(d, tk, iters, kind);
    run<6, 4, KIND, F32>(d, tk, iters, kind);
    run<6, 8, KIND, F32>(d, tk, iters, kind);
    run<7, 4, KIND, F32>(d, tk, iters, kind);
    run<7, 8, KIND, F32>(d, tk, iters, kind);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    double* d;
    unsigned long long* tk;
    (void)hipMalloc(&d, 256 * 512 * 8);
    (void)hipMalloc(&tk, (256 * 8 + 8) * 8);
    sweep<0, false>(d, tk, iters, "v_add_u32");
    sweep<1, false>(d, tk, iters, "v_fma_f64");
    sweep<2, false>(d, tk, iters, "v_pk_fma_f32");
    sweep<0, true>(d, tk, iters, "v_add_u32");
    sweep<2, true>(d, tk, iters, "v_pk_fma_f32");
    return 0;
}
