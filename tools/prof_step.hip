// Incremental cost of the env step's stages at 64k boards (hipGraph of 100 launches each):
// load+store floor, + Philox, + legal mask, + move, + spawn, + terminal reset.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prof_step.hip -o tools/prof_step
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../reinforcement-learning-2048_amd/csrc/g2048_board.hpp"

using namespace g2048;

template <int STAGE, int BS = 256>
__global__ __launch_bounds__(BS) void k_stage(uint4* board, uint4* meta, uint32_t* out) {
    const int i = blockIdx.x * BS + threadIdx.x;
    Board b{board[i].x, board[i].y, board[i].z, board[i].w};
    uint4 m = meta[i];
    const uint64_t t = (uint64_t)m.z | ((uint64_t)m.w << 32);
    uint4 u = make_uint4(m.x * 0x9E3779B9u, i, m.z, m.y);
    if constexpr (STAGE >= 1) u = draw(0x2048u, 0u, (uint64_t)i, DOMAIN_STEP, t);
    uint32_t legal = u.y & 15u;
    if constexpr (STAGE >= 2) legal = legal_mask(b);
    const uint32_t act = u.x >> 30;
    uint32_t r = 0;
    if constexpr (STAGE >= 3) {
        if (legal && ((legal >> act) & 1u)) {
            r = apply_move(b, act);
            if constexpr (STAGE >= 4) spawn(b, u.z, u.w, 2147483648u);
        }
    }
    if constexpr (STAGE >= 5) {
        if (legal == 0u) b = fresh_board(u, 2147483648u);
    }
    m.x += r;
    m.y += 1u;
    m.z += 1u;
    board[i] = make_uint4(b.r0, b.r1, b.r2, b.r3);
    meta[i] = m;
    out[i] = legal | (r << 4);
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
    const int n = 65536;
    hipStream_t st;
    (void)hipStreamCreate(&st);
    uint4 *board, *meta;
    uint32_t* out;
    (void)hipMalloc(&board, n * 16);
    (void)hipMalloc(&meta, n * 16);
    (void)hipMalloc(&out, n * 4);
    (void)hipMemset(meta, 0, n * 16);
    // mid-game boards: a few tiles
    uint4* hb = new uint4[n];
    for (int i = 0; i < n; ++i) {
        uint32_t x = 2654435761u * (i + 1);
        hb[i] = make_uint4(0x01000201u & (x | 0x01000001u), 0x00020100u, (x >> 8) & 0x03000103u, 0x01u);
    }
    (void)hipMemcpy(board, hb, n * 16, hipMemcpyHostToDevice);
#define RUN(S)                                                                              \
    printf("stage %d %.3f us\n", S,                                                        \
           per_launch_us([&] { hipLaunchKernelGGL(k_stage<S>, dim3(n / 256), dim3(256), 0, st, \
                                                  board, meta, out); }, st))
    RUN(0); RUN(1); RUN(2); RUN(3); RUN(4); RUN(5);
    // the full stage with other workgroup sizes (same 64k lanes)
    printf("stage 5, 64-thread blocks %.3f us\n",
           per_launch_us([&] { hipLaunchKernelGGL((k_stage<5, 64>), dim3(n / 64), dim3(64), 0, st,
                                                  board, meta, out); }, st));
    printf("stage 5, 128-thread blocks %.3f us\n",
           per_launch_us([&] { hipLaunchKernelGGL((k_stage<5, 128>), dim3(n / 128), dim3(128), 0, st,
                                                  board, meta, out); }, st));
    return 0;
}
