// Fixed-order slab reduction microbenchmark: NS slabs of S doubles (the float64 conv update:
// 256 x 33 480, 68.6 MB), summed per position in slab order -- the shape of k_conv64_reduce and,
// in float, of k_reduce_slabs.  Variants of the block shape / loads in flight, each timed right
// after a kernel that rewrites the slabs (as the train kernels do) and back to back, against a
// plain streaming read of the same bytes.  Every variant's sums are checked bitwise against
// variant 0 (the same per-position order).  Usage: ./slabred [ns] [s]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int MAXS = 256;

__global__ void k_fill(double* slab, int64_t n, uint32_t salt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        slab[i] = (double)((i * 2654435761u + salt) % 1000003) * 1e-3;
}

// RW waves per block, P positions per lane (P = 2: double2), wave w sums slabs w, w + RW, ...
// with all of its loads in flight, then wave 0 adds the RW partials in wave order.
template <int RW, int P>
__global__ __launch_bounds__(64 * RW) void k_red(const double* __restrict__ slab, int ns, int S,
                                                 double* __restrict__ out) {
    __shared__ double part[RW][64 * P];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pos = blockIdx.x * (64 * P) + P * lane;
    double r[P];
#pragma unroll
    for (int h = 0; h < P; ++h) r[h] = 0.0;
    if (pos < S) {
        constexpr int NK = MAXS / RW;
        double v[NK][P];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int g = wave + RW * k;
            if (g < ns) {
                if constexpr (P == 2) {
                    const double2 x = *reinterpret_cast<const double2*>(slab + (int64_t)g * S + pos);
                    v[k][0] = x.x;
                    v[k][1] = x.y;
                } else if constexpr (P == 4) {
                    const double2 x = *reinterpret_cast<const double2*>(slab + (int64_t)g * S + pos);
                    const double2 y = *reinterpret_cast<const double2*>(slab + (int64_t)g * S + pos + 2);
                    v[k][0] = x.x;
                    v[k][1] = x.y;
                    v[k][2] = y.x;
                    v[k][3] = y.y;
                } else {
                    v[k][0] = slab[(int64_t)g * S + pos];
                }
            } else {
#pragma unroll
                for (int h = 0; h < P; ++h) v[k][h] = 0.0;
            }
        }
#pragma unroll
        for (int k = 0; k < NK; ++k)
#pragma unroll
            for (int h = 0; h < P; ++h) r[h] += v[k][h];
    }
#pragma unroll
    for (int h = 0; h < P; ++h) part[wave][P * lane + h] = r[h];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int h = 0; h < P; ++h) {
            double s = part[0][P * lane + h];
            for (int k = 1; k < RW; ++k) s += part[k][P * lane + h];
            if (pos + h < S) out[pos + h] = s;
        }
    }
}

// Streaming read of the same bytes (no reduction order): the memory-side ceiling.
__global__ __launch_bounds__(256) void k_stream(const double2* __restrict__ p, int64_t n2, double* out) {
    double2 acc = make_double2(0, 0);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const double2 x = p[i];
        acc.x += x.x;
        acc.y += x.y;
    }
    if (acc.x == 12345.678) out[0] = acc.y;
}

int main(int argc, char** argv) {
    const int ns = argc > 1 ? atoi(argv[1]) : 256;
    const int S = argc > 2 ? atoi(argv[2]) : 33480;
    const int64_t n = (int64_t)ns * S;
    double *slab, *out, *ref;
    (void)hipMalloc(&slab, n * 8);
    (void)hipMalloc(&out, S * 8);
    (void)hipMalloc(&ref, S * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct V {
        const char* name;
        void (*fn)(const double*, int, int, double*);
    };
    const V vs[] = {
        {"RW16 P2 (k_conv64_reduce)", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<16, 2>), dim3((b + 127) / 128), dim3(1024), 0, nullptr, s, a, b, o); }},
        {"RW8 P2", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<8, 2>), dim3((b + 127) / 128), dim3(512), 0, nullptr, s, a, b, o); }},
        {"RW4 P2", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<4, 2>), dim3((b + 127) / 128), dim3(256), 0, nullptr, s, a, b, o); }},
        {"RW16 P1", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<16, 1>), dim3((b + 63) / 64), dim3(1024), 0, nullptr, s, a, b, o); }},
        {"RW8 P1", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<8, 1>), dim3((b + 63) / 64), dim3(512), 0, nullptr, s, a, b, o); }},
        {"RW16 P4", [](const double* s, int a, int b, double* o) {
             hipLaunchKernelGGL((k_red<16, 4>), dim3((b + 255) / 256), dim3(1024), 0, nullptr, s, a, b, o); }},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    std::vector<double> h0(S), h1(S);
    for (int rep = 0; rep < 2; ++rep) {
        for (int v = 0; v < nv; ++v) {
            float ms_after = 0, ms_b2b = 0, ms;
            for (int it = 0; it < 10; ++it) {
                hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, nullptr, slab, n, 7u);
                (void)hipEventRecord(e0);
                vs[v].fn(slab, ns, S, v ? out : ref);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
                ms_after += ms / 10;
            }
            (void)hipEventRecord(e0);
            for (int it = 0; it < 20; ++it) vs[v].fn(slab, ns, S, v ? out : ref);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms_b2b = ms / 20;
            bool ok = true;
            if (v) {
                (void)hipMemcpy(h0.data(), ref, S * 8, hipMemcpyDeviceToHost);
                (void)hipMemcpy(h1.data(), out, S * 8, hipMemcpyDeviceToHost);
                ok = h0 == h1;
            }
            printf("%-28s after fill %7.2f us (%5.2f TB/s)  back to back %7.2f us (%5.2f TB/s)  %s\n",
                   vs[v].name, ms_after * 1e3, n * 8 / (ms_after * 1e9), ms_b2b * 1e3,
                   n * 8 / (ms_b2b * 1e9), ok ? "bitwise = v0" : "MISMATCH");
        }
        float ms;
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, nullptr, slab, n, 7u);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, nullptr, reinterpret_cast<const double2*>(slab), n / 2, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s after fill %7.2f us (%5.2f TB/s)\n", "stream read", ms * 1e3, n * 8 / (ms * 1e9));
    }
    return 0;
}
