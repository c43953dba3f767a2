// Launch floor on this GPU: per-launch time of hipGraph-replayed kernels (100 per graph).
//   empty      : no work
//   touch64k   : 65536 lanes, one dwordx4 load + store each (the step kernel's minimum traffic)
//   copy32B    : 65536 lanes, 2 x dwordx4 load + store (board + meta)
//   copy32B_s  : the same, pointers in a by-value struct (read from the kernarg segment, never
//                preloaded into SGPRs)
// hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o tools/bin/launch_floor
// hipcc ... -mllvm -amdgpu-kernarg-preload-count=8 -o tools/bin/launch_floor_pre  (leading
//   non-aggregate kernel arguments arrive in SGPRs: no scalar-load round trip before the loads)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}
__global__ __launch_bounds__(256) void k_touch(uint4* p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    uint4 v = p[i];
    v.x += 1u;
    p[i] = v;
}
__global__ __launch_bounds__(256) void k_copy(uint4* a, uint4* b) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    uint4 x = a[i], y = b[i];
    x.x += y.y;
    y.x ^= x.z;
    a[i] = x;
    b[i] = y;
}

struct CopyArgs {
    uint4* a;
    uint4* b;
    int64_t pad[6];
};
__global__ __launch_bounds__(256) void k_copy_s(CopyArgs A) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    uint4 x = A.a[i], y = A.b[i];
    x.x += y.y;
    y.x ^= x.z;
    A.a[i] = x;
    A.b[i] = y;
}

template <typename F>
float per_launch_us(F launch, hipStream_t st) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int k = 0; k < 100; ++k) launch();
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, st);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, st);
    for (int r = 0; r < 20; ++r) (void)hipGraphLaunch(ge, st);
    (void)hipEventRecord(b, st);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / 2000.f;
}

int main() {
    hipStream_t st;
    (void)hipStreamCreate(&st);
    uint4 *p, *q;
    (void)hipMalloc(&p, 65536 * 16);
    (void)hipMalloc(&q, 65536 * 16);
    (void)hipMemset(p, 0, 65536 * 16);
    (void)hipMemset(q, 0, 65536 * 16);
    printf("empty    %.3f us\n", per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); }, st));
    printf("empty256 %.3f us\n", per_launch_us([&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st); }, st));
    printf("touch64k %.3f us\n", per_launch_us([&] { hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, st, p); }, st));
    printf("copy32B  %.3f us\n", per_launch_us([&] { hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, st, p, q); }, st));
    CopyArgs ca{p, q, {0, 0, 0, 0, 0, 0}};
    printf("copy32B_s %.3f us\n", per_launch_us([&] { hipLaunchKernelGGL(k_copy_s, dim3(256), dim3(256), 0, st, ca); }, st));
    return 0;
}
