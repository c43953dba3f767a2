// f64 MFMA (v_mfma_f64_16x16x4_f64) cadence at ONE wave per SIMD -- the occupancy of the fused
// float64 learner kernels (csrc/g2048_conv64.hip: 256 workgroups x 4 waves, one per CU).
// For C independent accumulation chains (C = 1 .. 16) with the accumulators pinned in VGPRs or in
// AGPRs (inline asm), cycles per MFMA from s_memtime around the loop of every wave and TF/s of the
// whole grid from HIP events.  Also: the same loop with A read from LDS each step (ds_read_b64)
// and B in registers, the conv2 pattern.  Usage: ./mfma64_chains [iters]
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int C, bool kAgpr, bool kLds>
__global__ __launch_bounds__(256) void kchain(double* out, unsigned long long* ticks, int iters) {
    __shared__ double sa[4][16][64 + 2];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4 * 16 * 66; i += 256) (&sa[0][0][0])[i] = 1.0 + i * 1e-9;
    __syncthreads();
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c[C];
#pragma unroll
    for (int k = 0; k < C; ++k) c[k] = d4{0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < C; ++k) {
            double av = a;
            if constexpr (kLds) av = sa[w][k & 15][l];
            if constexpr (kAgpr)
                asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c[k]) : "v"(av), "v"(b));
            else
                asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c[k]) : "v"(av), "v"(b));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) s += c[k][k & 3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (l == 0) ticks[blockIdx.x * 4 + w] = t1 - t0;
}

// The whole loop as ONE asm block, so the accumulators stay where the constraint puts them (with
// one asm per MFMA the compiler kept "a"-constrained accumulators in VGPRs and copied them into
// AGPRs and back around every MFMA).
#define MF(R, i) "v_mfma_f64_16x16x4_f64 %" #i ", %[a], %[b], %" #i "\n\t"
#define LOOP_HEAD "1:\n\t"
#define LOOP_TAIL "s_sub_u32 %[n], %[n], 1\n\ts_cmp_lg_u32 %[n], 0\n\ts_cbranch_scc1 1b\n\t"
template <bool kAgpr>
__global__ __launch_bounds__(256) void kpinned4(double* out, unsigned long long* ticks, int iters) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    unsigned n = (unsigned)iters;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (kAgpr)
        asm volatile(LOOP_HEAD MF(R, 0) MF(R, 1) MF(R, 2) MF(R, 3) LOOP_TAIL
                     : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), [n] "+s"(n)
                     : [a] "v"(a), [b] "v"(b) : "scc");
    else
        asm volatile(LOOP_HEAD MF(R, 0) MF(R, 1) MF(R, 2) MF(R, 3) LOOP_TAIL
                     : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), [n] "+s"(n)
                     : [a] "v"(a), [b] "v"(b) : "scc");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (l == 0) ticks[blockIdx.x * 4 + w] = t1 - t0;
}
template <bool kAgpr>
__global__ __launch_bounds__(256) void kpinned1(double* out, unsigned long long* ticks, int iters) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c0 = {0, 0, 0, 0};
    unsigned n = (unsigned)iters * 4u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (kAgpr)
        asm volatile(LOOP_HEAD MF(R, 0) LOOP_TAIL : "+a"(c0), [n] "+s"(n) : [a] "v"(a), [b] "v"(b) : "scc");
    else
        asm volatile(LOOP_HEAD MF(R, 0) LOOP_TAIL : "+v"(c0), [n] "+s"(n) : [a] "v"(a), [b] "v"(b) : "scc");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = c0[0];
    if (l == 0) ticks[blockIdx.x * 4 + w] = t1 - t0;
}

template <typename K>
void run_k(K kern, double* d, unsigned long long* tk, int iters, const char* what) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<256, 256>>>(d, tk, iters / 4);
    (void)hipEventRecord(e0);
    kern<<<256, 256>>>(d, tk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long h[256 * 4];
    (void)hipMemcpy(h, tk, sizeof h, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < 1024; ++i) avg += (double)h[i];
    avg /= 1024;
    const double n_mfma = (double)iters * 4;
    printf("%-40s %7.1f ticks/MFMA  %6.1f TF\n", what, avg / n_mfma, 1024.0 * n_mfma * 2048.0 / ms / 1e9);
}

template <int C, bool kAgpr, bool kLds>
void run(double* d, unsigned long long* tk, int iters, const char* what) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int grid = 256;
    kchain<C, kAgpr, kLds><<<grid, 256>>>(d, tk, iters / 4);  // warm
    (void)hipEventRecord(e0);
    kchain<C, kAgpr, kLds><<<grid, 256>>>(d, tk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    static unsigned long long h[256 * 4];
    (void)hipMemcpy(h, tk, sizeof h, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < grid * 4; ++i) avg += (double)h[i];
    avg /= grid * 4;
    const double n_mfma = (double)iters * C;
    const double fl = grid * 4.0 * n_mfma * 2048.0;
    printf("%-26s chains %2d: %7.1f ticks/MFMA  %6.1f TF (%.3f ms)\n", what, C, avg / n_mfma,
           fl / ms / 1e9, ms);
}

template <bool kAgpr, bool kLds>
void sweep(double* d, unsigned long long* tk, int iters, const char* what) {
    run<1, kAgpr, kLds>(d, tk, iters, what);
    run<2, kAgpr, kLds>(d, tk, iters, what);
    run<3, kAgpr, kLds>(d, tk, iters, what);
    run<4, kAgpr, kLds>(d, tk, iters, what);
    run<6, kAgpr, kLds>(d, tk, iters, what);
    run<8, kAgpr, kLds>(d, tk, iters, what);
    run<9, kAgpr, kLds>(d, tk, iters, what);
    run<12, kAgpr, kLds>(d, tk, iters, what);
    run<16, kAgpr, kLds>(d, tk, iters, what);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    double* d;
    unsigned long long* tk;
    (void)hipMalloc(&d, 256 * 256 * 8);
    (void)hipMalloc(&tk, 256 * 4 * 8);
    run_k(kpinned4<false>, d, tk, iters, "asm loop, 4 chains, acc VGPR");
    run_k(kpinned4<true>, d, tk, iters, "asm loop, 4 chains, acc AGPR");
    run_k(kpinned1<false>, d, tk, iters, "asm loop, 1 chain, acc VGPR");
    run_k(kpinned1<true>, d, tk, iters, "asm loop, 1 chain, acc AGPR");
    sweep<false, false>(d, tk, iters, "acc VGPR, A/B in regs");

    sweep<false, true>(d, tk, iters, "acc VGPR, A from LDS");

    return 0;
}
