// Probe the operand / result layout of v_mfma_f64_16x16x4f64 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
    const int l = threadIdx.x;
    // A[i][k] = 1 if (i,k) == probe; use A = e_i (row one-hot through k), B encodes j
    // A[i][k] = (i + 1) * (k == 0); B[k][j] = (j + 1) * 100 * (k == 0)  => D[i][j] = (i+1)(j+1)100
    const int ai = l % 16, ak = l / 16;
    const double a = ak == 0 ? (double)(ai + 1) : 0.0;
    const int bj = l % 16, bk = l / 16;
    const double b = bk == 0 ? (double)(bj + 1) * 100.0 : 0.0;
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
    // second probe: verify k mapping: A[i][k] = (k+1) for i==0 only, B[k][j] = 10^k for j==0
    const double a2 = ai == 0 ? (double)(ak + 1) : 0.0;
    const double b2 = bj == 0 ? (ak == 0 ? 1.0 : ak == 1 ? 10.0 : ak == 2 ? 100.0 : 1000.0) : 0.0;
    d4 c2 = {0, 0, 0, 0};
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, c2, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[256 + l * 4 + r] = c2[r];
}
int main() {
    double* d;
    hipMalloc(&d, 512 * 8);
    k<<<1, 64>>>(d);
    double h[512];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int r = 0; r < 4; ++r) {
            const double v = h[l * 4 + r];
            const int i = (int)(v / 100.0 + 0.5), j = 0;
            // v = (i+1)*(j+1)*100 -> can't separate; print raw
            printf(" %8.0f", v);
        }
        printf("   | k-probe:");
        for (int r = 0; r < 4; ++r) printf(" %6.0f", h[256 + l * 4 + r]);
        printf("\n");
    }
    extern int main2();
    return main2();
}
// ---- throughput: f64 MFMA (4 chains) and v_fma_f64 (8 chains), whole chip
__global__ __launch_bounds__(256) void kmfma(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < iters; ++it) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + l] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void kmfma8(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c[8];
    for (int k = 0; k < 8; ++k) c[k] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k][k & 3];
    out[blockIdx.x * 256 + l] = s;
}
// 8 chains, every MFMA with its own A and B registers (no reuse), operands fixed in registers
__global__ __launch_bounds__(256) void kmfma_distinct(double* out, int iters) {
    const int l = threadIdx.x;
    double a[8], b[8];
    for (int k = 0; k < 8; ++k) {
        a[k] = 1.0 + (l + k) * 1e-9;
        b[k] = 1.0 - (l * k) * 1e-9;
    }
    d4 c[8];
    for (int k = 0; k < 8; ++k) c[k] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[k], b[k], c[k], 0, 0, 0);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k][k & 3];
    out[blockIdx.x * 256 + l] = s;
}
__global__ __launch_bounds__(256) void kfma(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    double x[8];
    for (int k = 0; k < 8; ++k) x[k] = k;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = fma(a, x[k], b);
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * 256 + l] = s;
}
// co-issue probes: (a) 2 waves per SIMD, one running 8 f64 MFMA chains, the other 8 v_fma_f64
// chains (fiters FMAs per chain); (b) one wave interleaving 8 MFMA chains with 8 FMA chains
__global__ __launch_bounds__(512) void kmix2(double* out, int iters, int fiters) {
    const int l = threadIdx.x, w = l >> 6;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    double s = 0;
    if (w < 4) {
        d4 c[8];
        for (int k = 0; k < 8; ++k) c[k] = d4{0, 0, 0, 0};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
        }
        for (int k = 0; k < 8; ++k) s += c[k][k & 3];
    } else {
        double x[8];
        for (int k = 0; k < 8; ++k) x[k] = k;
        for (int it = 0; it < fiters; ++it) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = fma(a, x[k], b);
        }
        for (int k = 0; k < 8; ++k) s += x[k];
    }
    out[blockIdx.x * 512 + l] = s;
}
__global__ __launch_bounds__(256) void kmix1(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c[8];
    double x[8];
    for (int k = 0; k < 8; ++k) { c[k] = d4{0, 0, 0, 0}; x[k] = k; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
            x[k] = fma(a, x[k], b);
        }
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k][k & 3] + x[k];
    out[blockIdx.x * 256 + l] = s;
}
// 8 chains at one wave per SIMD with the accumulators pinned by inline asm: in AGPRs ("+a") or in
// VGPRs ("+v") -- the compiler-generated kmfma8 loop above copies its accumulators between the
// register files every iteration, which is what capped it at 47.6 TF
template <bool kAgpr>
__global__ __launch_bounds__(256) void kmfma_pinned(double* out, int iters) {
    const int l = threadIdx.x;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c[8];
    for (int k = 0; k < 8; ++k) c[k] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (kAgpr)
                asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c[k]) : "v"(a), "v"(b));
            else
                asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
        }
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += c[k][k & 3];
    out[blockIdx.x * 256 + l] = s;
}
// the same for f32 v_mfma_f32_16x16x4_f32 (8 chains, accumulators pinned)
typedef float f4 __attribute__((ext_vector_type(4)));
template <bool kAgpr>
__global__ __launch_bounds__(256) void kmfma32_pinned(double* out, int iters) {
    const int l = threadIdx.x;
    float a = 1.0f + l * 1e-6f, b = 1.0f - l * 1e-6f;
    f4 c[8];
    for (int k = 0; k < 8; ++k) c[k] = f4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (kAgpr)
                asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c[k]) : "v"(a), "v"(b));
            else
                asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c[k]) : "v"(a), "v"(b));
        }
    }
    float s = 0;
    for (int k = 0; k < 8; ++k) s += c[k][k & 3];
    out[blockIdx.x * 256 + l] = s;
}
struct Tm { hipEvent_t a, b; };
int main2() {
    double* d;
    (void)hipMalloc(&d, 2048 * 256 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        const int it = 20000;
        for (int pin = 0; pin < 2; ++pin) {
            float ms;
            (void)hipEventRecord(e0);
            if (pin) kmfma_pinned<true><<<1024, 256>>>(d, it / 2);
            else kmfma_pinned<false><<<1024, 256>>>(d, it / 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fm = 1024.0 * 4 * (it / 2) * 8 * 2048.0;
            printf("mfma f64 8 chains, accumulators pinned in %s: %.3f ms  %.1f TF\n",
                   pin ? "AGPRs" : "VGPRs", ms, fm / ms / 1e9);
        }
        for (int pin = 0; pin < 2; ++pin) {
            float ms;
            (void)hipEventRecord(e0);
            if (pin) kmfma32_pinned<true><<<1024, 256>>>(d, it);
            else kmfma32_pinned<false><<<1024, 256>>>(d, it);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fm = 1024.0 * 4 * it * 8 * 2048.0;
            printf("mfma f32 16x16x4 8 chains, accumulators pinned in %s: %.3f ms  %.1f TF\n",
                   pin ? "AGPRs" : "VGPRs", ms, fm / ms / 1e9);
        }
        for (int fit = 0; fit <= 4 * it; fit += it) {
            float ms;
            (void)hipEventRecord(e0);
            kmix2<<<1024, 512>>>(d, it / 2, fit);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fm = 1024.0 * 4 * (it / 2) * 8 * 2048.0;
            const double ff = 1024.0 * 256 * (double)fit * 8 * 2.0;
            printf("mix2 (MFMA wave + FMA wave per SIMD, fma iters %d): %.3f ms  MFMA %.1f + VALU %.1f = %.1f TF\n",
                   fit, ms, fm / ms / 1e9, ff / ms / 1e9, (fm + ff) / ms / 1e9);
        }
        {
            float ms;
            (void)hipEventRecord(e0);
            kmix1<<<1024, 256>>>(d, it / 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fm = 1024.0 * 4 * (it / 2) * 8 * 2048.0;
            const double ff = 1024.0 * 256 * (double)(it / 2) * 8 * 2.0;
            printf("mix1 (one wave, MFMA + FMA interleaved): %.3f ms  MFMA %.1f + VALU %.1f TF\n", ms,
                   fm / ms / 1e9, ff / ms / 1e9);
        }
        (void)hipEventRecord(e0);
        kmfma<<<1024, 256>>>(d, it);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double fl = 1024.0 * 4 * it * 4 * 2048.0;  // blocks*waves*iters*mfma*flop
        printf("mfma f64 16x16x4: %.3f ms  %.1f TF\n", ms, fl / ms / 1e9);
        (void)hipEventRecord(e0);
        kfma<<<1024, 256>>>(d, it);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double fl2 = 1024.0 * 256 * it * 8 * 2.0;
        printf("v_fma_f64 8 chains: %.3f ms  %.1f TF\n", ms, fl2 / ms / 1e9);
        {
            (void)hipEventRecord(e0);
            kmfma_distinct<<<1024, 256>>>(d, it / 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fl3 = 1024.0 * 4 * (it / 2) * 8 * 2048.0;
            printf("mfma f64 8 chains, distinct A/B per MFMA: %.3f ms  %.1f TF\n", ms, fl3 / ms / 1e9);
        }
        for (int blocks = 1024; blocks <= 2048; blocks *= 2) {
            (void)hipEventRecord(e0);
            kmfma8<<<blocks, 256>>>(d, it / 2);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double fl3 = (double)blocks * 4 * (it / 2) * 8 * 2048.0;
            printf("mfma f64 8 chains, %d waves/SIMD: %.3f ms  %.1f TF\n", blocks / 1024, ms,
                   fl3 / ms / 1e9);
        }
    }
    return 0;
}
