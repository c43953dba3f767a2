// Rollout variants side by side: each variant steps its own env (same seed) through the same
// launches, the results are compared byte for byte with variant 0 (boards, meta, episode
// counters, clocks, every ring section), then each is timed over graph-replayed launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rollexp.hip -o tools/rollexp
//   tools/rollexp [n=65536] [K=64]
#include "../reinforcement-learning-2048_amd/csrc/g2048.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

void launch_old(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout<true, true, false>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

void launch_lean(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    hipLaunchKernelGGL((k_rollout_lean<false, false, true>), dim3(grid_for(e->n)), dim3(kBlock), 0, st, A);
}

struct Variant {
    const char* name;
    void (*fn)(g2048_env*, g2048_replay*, int, hipStream_t);
};

const Variant kVariants[] = {
    {"k_rollout (general path)", launch_old},
    {"k_rollout_lean", launch_lean},
};

template <typename T>
std::vector<T> fetch(const T* d, size_t n) {
    std::vector<T> h(n);
    (void)hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost);
    return h;
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const int K = argc > 2 ? atoi(argv[2]) : 64;
    const int nv = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
    hipStream_t st;
    (void)hipStreamCreate(&st);
    std::vector<g2048_env*> envs(nv);
    std::vector<g2048_replay*> rbs(nv);
    for (int v = 0; v < nv; ++v) {
        if (g2048_env_create(&envs[v], n, 7, 0, 0, 0, nullptr) ||
            g2048_replay_create(&rbs[v], n * K, 0, nullptr)) {
            printf("create failed: %s\n", g2048_last_error());
            return 1;
        }
    }
    // parity: 5 launches from the same start (an odd K first moves every clock to an odd step)
    for (int v = 0; v < nv; ++v) {
        kVariants[v].fn(envs[v], rbs[v], 3, st);
        for (int it = 0; it < 4; ++it) kVariants[v].fn(envs[v], rbs[v], K, st);
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    const size_t C = (size_t)n * K;
    auto b0 = fetch(envs[0]->board, n * 16);
    auto m0 = fetch(envs[0]->meta, n * 2);
    auto e0 = fetch(envs[0]->ep, n * 4);
    auto c0 = fetch(envs[0]->clock, (n + 63) / 64);
    auto s0 = fetch(rbs[0]->s, C * 16);
    auto t0 = fetch(rbs[0]->s2, C * 16);
    auto a0 = fetch(rbs[0]->a, C);
    auto r0 = fetch(rbs[0]->r, C);
    auto d0 = fetch(rbs[0]->d, C);
    int bad = 0;
    for (int v = 1; v < nv; ++v) {
        const bool ok = fetch(envs[v]->board, n * 16) == b0 && fetch(envs[v]->meta, n * 2) == m0 &&
                        fetch(envs[v]->ep, n * 4) == e0 &&
                        fetch(envs[v]->clock, (n + 63) / 64) == c0 &&
                        fetch(rbs[v]->s, C * 16) == s0 && fetch(rbs[v]->s2, C * 16) == t0 &&
                        fetch(rbs[v]->a, C) == a0 && fetch(rbs[v]->r, C) == r0 &&
                        fetch(rbs[v]->d, C) == d0;
        printf("parity %-34s %s\n", kVariants[v].name, ok ? "bitwise equal" : "MISMATCH");
        bad += !ok;
    }
    // timing: graphs of 20 launches, each replayed once untimed, then 10 timed replays
    hipEvent_t ev0, ev1;
    (void)hipEventCreate(&ev0);
    (void)hipEventCreate(&ev1);
    for (int rep = 0; rep < 3; ++rep) {
        for (int v = 0; v < nv; ++v) {
            hipGraph_t g;
            hipGraphExec_t ge;
            (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
            for (int it = 0; it < 20; ++it) kVariants[v].fn(envs[v], rbs[v], K, st);
            (void)hipStreamEndCapture(st, &g);
            (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev0, st);
            for (int it = 0; it < 10; ++it) (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev1, st);
            (void)hipEventSynchronize(ev1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev0, ev1);
            const double us = 1e3 * ms / 200.0;
            printf("%-36s n=%-8lld K=%-4d %8.2f us/launch  %7.1f G steps/s  %6.3f of 8 TB/s\n",
                   kVariants[v].name, (long long)n, K, us, n * K / us * 1e-3,
                   38.0 * n * K / us * 1e-6 / 8.0);
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        }
    }
    return bad ? 2 : 0;
}
