// Rate of v_mfma_f64_16x16x4_f64 in the fp64 conv2 pattern (9 accumulator chains, 16 k-steps per
// tile), one wave per SIMD (256 workgroups of 4 waves), by operand source:
//   0: A and B fixed registers (the pinned microbenchmark)
//   1: A from LDS (ds_read_b64 per MFMA, one k-step ahead), B fixed
//   2: A fixed, B from global (one load per MFMA, two k-steps ahead, L2-resident 72 KB slice)
//   3: A from LDS and B from global (the conv2 loop)
//   7: as 3 with per-lane (VGPR) B addresses, as hipcc builds them when the wave index is t >> 6
//   11: as 3 with the B slice alternating between two nets' operands per tile (590 KB)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma64_feed.hip -o tools/mfma64_feed
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const double gdouble;

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int MODE>
__global__ __launch_bounds__(256) void kfeed(const double* __restrict__ gB, double* out, int tiles) {
    __shared__ double V[9 * 16 * 66];
    const int t = threadIdx.x, l = t & 63, lr = l & 15, lk = l >> 4;
    const int w = (MODE & 4) ? (t >> 6) : __builtin_amdgcn_readfirstlane(t >> 6);
    for (int k = t; k < 9 * 16 * 66; k += 256) V[k] = 1.0 + k * 1e-9;
    __syncthreads();
    d4 acc[9];
    for (int x = 0; x < 9; ++x) acc[x] = d4{0, 0, 0, 0};
    const double af = 1.0 + l * 1e-9, bf = 1.0 - l * 1e-9;
    for (int tile = 0; tile < tiles; ++tile) {
        const gdouble* base = (const gdouble*)gB;
        asm volatile("" : "+s"(base));  // opaque per tile: the B loads stay in their k-steps
        const gdouble* bp = base + (size_t)w * 9 * 16 * 64 + l +
                            ((MODE & 8) && (tile & 1) ? 4 * 9 * 16 * 64 : 0);
        auto ld9 = [&](double(&b)[9], int s) {
#pragma unroll
            for (int x = 0; x < 9; ++x) b[x] = (MODE & 2) ? bp[(x * 16 + s) * 64] : bf;
        };
        auto la9 = [&](double(&a)[9], int s) {
            const double* vr = V + lr * 66 + 4 * s + lk;
#pragma unroll
            for (int x = 0; x < 9; ++x) a[x] = (MODE & 1) ? vr[x * 16 * 66] : af;
        };
        double bb[3][9], aa[2][9];
        ld9(bb[0], 0);
        ld9(bb[1], 1);
        la9(aa[0], 0);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if (s + 1 < 16) la9(aa[(s + 1) & 1], s + 1);
            if (s + 2 < 16) ld9(bb[(s + 2) % 3], s + 2);
#pragma unroll
            for (int x = 0; x < 9; ++x) acc[x] = mfma(aa[s & 1][x], bb[s % 3][x], acc[x]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    double s = 0;
    for (int x = 0; x < 9; ++x) s += acc[x][x & 3];
    out[blockIdx.x * 256 + t] = s;
}

int main() {
    double *gB, *out;
    (void)hipMalloc(&gB, 8 * 9 * 16 * 64 * 8);
    (void)hipMemset(gB, 0, 8 * 9 * 16 * 64 * 8);
    (void)hipMalloc(&out, 256 * 256 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int tiles = 200;
    auto run = [&](int mode) {
        auto go = [&] {
            switch (mode) {
                case 0: kfeed<0><<<256, 256>>>(gB, out, tiles); break;
                case 1: kfeed<1><<<256, 256>>>(gB, out, tiles); break;
                case 2: kfeed<2><<<256, 256>>>(gB, out, tiles); break;
                case 3: kfeed<3><<<256, 256>>>(gB, out, tiles); break;
                case 7: kfeed<7><<<256, 256>>>(gB, out, tiles); break;
                default: kfeed<11><<<256, 256>>>(gB, out, tiles); break;
            }
        };
        go();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) go();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double mf = 5.0 * tiles * 144;  // MFMAs per wave
        const double us = ms * 1e3;
        printf("mode %d: %.1f us  %.2f ns per MFMA per wave  %.1f TF\n", mode, us, us * 1e3 / mf,
               1024.0 * mf * 2048.0 / (us * 1e-6) / 1e12);
    };
    for (int m : {0, 1, 2, 3, 7, 11}) run(m);
    for (int m : {0, 1, 2, 3, 7, 11}) run(m);
    return 0;
}
