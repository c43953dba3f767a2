// Per-pair timeline of the rollout (k_rollout's lean loop) for a few waves: s_memtime at the top of
// every pair iteration, to see whether a launch's first steps run slower than its steady state.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude tools/prof_roll.hip -o tools/prof_roll
#include <cstdint>
__device__ unsigned long long g_tick[8][260];
#define G2048_ROLL_TICK(np)                                                               \
    do {                                                                                   \
        const unsigned wv = (unsigned)(blockIdx.x * 4 + (threadIdx.x >> 6));               \
        if ((threadIdx.x & 63) == 0 && (wv % 128) == 0 && wv / 128 < 8)                    \
            g_tick[wv / 128][(rest >> 1) - (np)] = __builtin_amdgcn_s_memtime();            \
    } while (0)
#define G2048_ROLL_MARK(k)                                                                \
    do {                                                                                   \
        const unsigned wv = (unsigned)(blockIdx.x * 4 + (threadIdx.x >> 6));               \
        if ((threadIdx.x & 63) == 0 && (wv % 128) == 0 && wv / 128 < 8)                    \
            g_tick[wv / 128][256 + (k)] = __builtin_amdgcn_s_memtime();                     \
    } while (0)
#include "../reinforcement-learning-2048_amd/csrc/g2048.hip"
#include <cstdio>
#include <vector>
int main(int argc, char** argv) {
    const int64_t n = 65536;
    const int K = argc > 1 ? atoi(argv[1]) : 64;
    g2048_env* e = nullptr;
    g2048_replay* rb = nullptr;
    if (g2048_env_create(&e, n, 7, 0, 0, 0, nullptr)) { printf("env_create failed\n"); return 1; }
    if (g2048_replay_create(&rb, n * K, 0, nullptr)) { printf("replay failed\n"); return 1; }
    for (int it = 0; it < 20; ++it) g2048_env_rollout(e, K, rb, nullptr, nullptr);
    (void)hipDeviceSynchronize();
    g2048_env_rollout(e, K, rb, nullptr, nullptr);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(8 * 260);
    (void)hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_tick), h.size() * 8);
    for (int wv = 0; wv < 8; ++wv) {
        const unsigned long long* m = &h[wv * 260 + 256];
        printf("marks wave %4d: entry %llu  prologue %llu  loop %llu  epilogue %llu\n", wv * 128,
               m[0] - h[0 * 260 + 256], m[1] - m[0], m[2] - m[1], m[3] - m[2]);
    }
    for (int wv = 0; wv < 8; ++wv) {
        printf("wave %4d:", wv * 128);
        for (int p = 1; p < K / 2; ++p) printf(" %llu", h[wv * 260 + p] - h[wv * 260 + p - 1]);
        printf("\n");
    }
    return 0;
}
