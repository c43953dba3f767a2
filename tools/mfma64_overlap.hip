// Does VALU work hide under f64 MFMAs on gfx950?  The fused float64 conv learner runs one wave
// per SIMD and spends about a third of each tile in VALU / LDS phases between its MFMA phases
// (DESIGN §4.7); the eight-wave train A (two waves per SIMD) did not overlap them.  This probe
// measures, with s_memtime around each wave's loop (256 workgroups, one per CU):
//   same wave : 4 MFMA chains (v_mfma_f64_16x16x4_f64, VGPR accumulators), each MFMA followed by
//               NV independent VALU ops of one kind -> ticks per MFMA (64 = the VALU is hidden)
//   two waves : waves 0-3 run the MFMA-only loop, waves 4-7 (the same four SIMDs) a VALU-only loop
//               of 4*NV ops per iteration, the same iteration count -> ticks per iteration of each
//   VALU only : the VALU loop alone at one wave per SIMD (the issue cost to compare with)
// Kinds: v_add_u32, v_fma_f64, v_pk_fma_f32.
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

__device__ __forceinline__ void mfma(d4& c, double a, double b) {
    asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

// MODE 0: every wave MFMA + NV VALU per MFMA.  MODE 1: waves < 4 MFMA only, waves >= 4 VALU only
// (4*NV per iteration).  MODE 2: VALU only (4*NV per iteration), every wave.
template <int MODE, int NV, int KIND>
__global__ __launch_bounds__(512) void kmix(double* out, unsigned long long* ticks, int iters) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    Valu<KIND> v;
    v.init(l);
    const bool do_mfma = MODE == 0 || (MODE == 1 && w < 4);
    const bool do_valu = MODE == 0 || MODE == 2 || (MODE == 1 && w >= 4);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (do_mfma && do_valu) {
        for (int it = 0; it < iters; ++it) {
            mfma(c0, a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(k);
            mfma(c1, a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(1 * NV + k);
            mfma(c2, a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(2 * NV + k);
            mfma(c3, a, b);
#pragma unroll
            for (int k = 0; k < NV; ++k) v.op(3 * NV + k);
        }
    } else if (do_mfma) {
        for (int it = 0; it < iters; ++it) {
            mfma(c0, a, b);
            mfma(c1, a, b);
            mfma(c2, a, b);
            mfma(c3, a, b);
        }
    } else {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 4 * NV; ++k) v.op(k);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + v.sum();
    if (l == 0) ticks[blockIdx.x * 8 + w] = t1 - t0;
    // SIMD of this wave (HW_ID bits 5:4) for block 0, to check the two-wave pairing
    if (MODE == 1 && blockIdx.x == 0 && l == 0)
        ticks[256 * 8 + w] = (unsigned)__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);
}

template <int MODE, int NV, int KIND>
void run(double* d, unsigned long long* tk, int iters, const char* kind) {
    const int nt = MODE == 1 ? 512 : 256;
    kmix<MODE, NV, KIND><<<256, nt>>>(d, tk, iters / 4);  // warm
    kmix<MODE, NV, KIND><<<256, nt>>>(d, tk, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long h[256 * 8 + 8];
    (void)hipMemcpy(h, tk, sizeof h, hipMemcpyDeviceToHost);
    double lo = 0, hi = 0;  // average ticks of waves 0-3 and 4-7
    for (int g = 0; g < 256; ++g)
        for (int w = 0; w < 8; ++w) (w < 4 ? lo : hi) += (double)h[g * 8 + w];
    lo /= 1024.0 * iters;
    hi /= 1024.0 * iters;
    if (MODE == 0)
        printf("same wave  %-12s NV %2d : %6.1f ticks per MFMA (%5.1f per iteration of 4)\n", kind,
               NV, lo / 4, lo);
    else if (MODE == 1) {
        if (NV == 1) {
            printf("two waves: SIMD of waves 0..7 in workgroup 0:");
            for (int w = 0; w < 8; ++w) printf(" %llu", h[256 * 8 + w]);
            printf("\n");
        }
        printf("two waves  %-12s NV %2d : MFMA wave %6.1f, VALU wave %6.1f ticks per iteration\n",
               kind, NV, lo, hi);
    } else
        printf("VALU only  %-12s NV %2d : %6.1f ticks per iteration (%4.1f per op)\n", kind, NV, lo,
               lo / (4 * NV));
}

template <int KIND>
void sweep(double* d, unsigned long long* tk, int iters, const char* kind) {
    run<0, 0, KIND>(d, tk, iters, kind);
    run<0, 1, KIND>(d, tk, iters, kind);
    run<0, 2, KIND>(d, tk, iters, kind);
    run<0, 4, KIND>(d, tk, iters, kind);
    run<0, 8, KIND>(d, tk, iters, kind);
    run<2, 1, KIND>(d, tk, iters, kind);
    run<2, 4, KIND>(d, tk, iters, kind);
    run<2, 8, KIND>(d, tk, iters, kind);
    run<1, 1, KIND>(d, tk, iters, kind);
    run<1, 2, KIND>(d, tk, iters, kind);
    run<1, 4, KIND>(d, tk, iters, kind);
    run<1, 8, KIND>(d, tk, iters, kind);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    double* d;
    unsigned long long* tk;
    (void)hipMalloc(&d, 256 * 512 * 8);
    (void)hipMalloc(&tk, (256 * 8 + 8) * 8);
    sweep<0>(d, tk, iters, "v_add_u32");
    sweep<1>(d, tk, iters, "v_fma_f64");
    sweep<2>(d, tk, iters, "v_pk_fma_f32");
    return 0;
}
