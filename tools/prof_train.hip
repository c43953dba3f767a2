// Per-kernel event timing of the float32 conv train launches (train fwd, train bwd, the slab
// reduce) at B = 8192 and phase ticks of k_conv_train_fwd / bwd (s_memtime deltas of thread 0
// of block 0, charged to the phase that ENDS at the marker), built only for kernel tuning:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prof_train.hip -o tools/prof_train
// Argument: "nopre" (the reduce sums train fwd's slab terms too).
#define G2048_PHASE_PROF 1
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>
int g2048_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    return code;
}
#include "../reinforcement-learning-2048_amd/csrc/g2048_qtrain.hip"
// libg2048.so symbols that g2048_convnet_update links against (unused here)
extern "C" int g2048_replay_views(g2048_replay*, uint8_t**, uint8_t**, uint8_t**, int32_t**,
                                  uint8_t**, uint64_t**) { return 1; }
extern "C" int g2048_conv_targets_launch(const g2048_convnet_params*, const g2048_convnet_params*,
                                         g2048_replay*, const int64_t*, int64_t, uint64_t,
                                         const uint64_t*, float, int, int64_t*, float*, float*,
                                         void*) { return 1; }

__global__ void k_nop(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) *p = 0;
}

int main(int argc, char** argv) {
    const int B = 8192, C = 1 << 20;
    const int sizes[8] = {256, 64, 16384, 64, 16384, 64, 256, 4};
    float* w[8];
    for (int i = 0; i < 8; ++i) {
        std::vector<float> h(sizes[i]);
        for (int j = 0; j < sizes[i]; ++j) h[j] = 0.01f * ((j * 37 + i) % 17 - 8);
        (void)hipMalloc(&w[i], sizes[i] * 4);
        (void)hipMemcpy(w[i], h.data(), sizes[i] * 4, hipMemcpyHostToDevice);
    }
    uint8_t *rows, *acts;
    int64_t* idx;
    float *y, *grad, *loss, *ws;
    (void)hipMalloc(&rows, (size_t)C * 16);
    (void)hipMalloc(&acts, C);
    (void)hipMalloc(&idx, B * 8);
    (void)hipMalloc(&y, B * 4);
    (void)hipMalloc(&grad, 33476 * 4);
    (void)hipMalloc(&loss, 4);
    std::vector<uint8_t> hb((size_t)C * 16);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = (uint8_t)((i * 2654435761u >> 13) % 12);
    (void)hipMemcpy(rows, hb.data(), hb.size(), hipMemcpyHostToDevice);
    (void)hipMemset(acts, 1, C);
    std::vector<int64_t> hi(B);
    for (int i = 0; i < B; ++i) hi[i] = ((int64_t)i * 7919) % C;
    (void)hipMemcpy(idx, hi.data(), B * 8, hipMemcpyHostToDevice);
    (void)hipMemset(y, 0, B * 4);
    const int64_t nws = g2048_convnet_train_workspace(B);
    (void)hipMalloc(&ws, nws * 4);
    g2048_convnet_params p{w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]};
    for (int it = 0; it < 3; ++it)
        g2048_convnet_train_grad(&p, rows, acts, idx, y, B, ws, grad, loss, nullptr, nullptr);
    (void)hipDeviceSynchronize();
    unsigned long long zero[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tphase), zero, sizeof(zero));
    TrainArgs A{};
    A.W = NetW{w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]};
    A.rows = rows;
    A.actions = acts;
    A.idx = idx;
    A.y = y;
    A.batch = B;
    A.slab = ws;
    const int grid = (int)train_grid(B);
    A.dm = ws + (int64_t)grid * SLAB;
    // train bwd sums train fwd's slab terms into pre (the library's layout, pre_offset); argv[1]
    // == "nopre": the reduce sums every slab term itself
    const bool nopre = argc > 1 && strcmp(argv[1], "nopre") == 0;
    A.pre = grid >= SHADOW_MIN_GRID && !nopre ? ws + pre_offset(B) : nullptr;
    A.step = nullptr;
    ReduceAdam R;
    memset(&R, 0, sizeof(R));
    // argv[1] or argv[2] == "adam": Adam folded into the reduce (the learner's update)
    bool with_adam = false;
    for (int a = 1; a < argc; ++a) with_adam |= strcmp(argv[a], "adam") == 0;
    if (with_adam) {
        float *m, *v;
        unsigned long long* stepc;
        (void)hipMalloc(&m, 33476 * 4);
        (void)hipMalloc(&v, 33476 * 4);
        (void)hipMemset(m, 0, 33476 * 4);
        (void)hipMemset(v, 0, 33476 * 4);
        (void)hipMalloc(&stepc, 8);
        const unsigned long long one = 1;
        (void)hipMemcpy(stepc, &one, 8, hipMemcpyHostToDevice);
        for (int k = 0; k < 8; ++k) R.p[k] = w[k];
        R.m = m;
        R.v = v;
        R.step = stepc;
        R.lr = 1e-9;
        R.b1 = 0.9;
        R.b2 = 0.999;
        R.eps = 1e-8;
        R.on = 1;
    }
    // the library's choice (train_launch): the four-wave reduce of the pre path, else the
    // 16-wave one over every slab term
    auto reduce = [&]() {
        if (A.pre)
            hipLaunchKernelGGL(k_reduce_pre, dim3(NB_PRE4 + C1_BLOCKS), dim3(256), 0, nullptr, ws,
                               grid, A.pre, grad, loss, R);
        else
            hipLaunchKernelGGL(k_reduce_slabs, dim3((SL_LOSS / 4 + 64) / 64), dim3(64 * RW), 0,
                               nullptr, ws, grid, grad, loss, R);
    };
    hipEvent_t ev[4];
    for (int i = 0; i < 4; ++i) (void)hipEventCreate(&ev[i]);
    float tk[3] = {0, 0, 0};
    const int N = 20;
    for (int it = 0; it < N; ++it) {
        (void)hipEventRecord(ev[0], nullptr);
        hipLaunchKernelGGL(k_conv_train_fwd, dim3(grid), dim3(NT), 0, nullptr, A);
        (void)hipEventRecord(ev[1], nullptr);
        hipLaunchKernelGGL(k_conv_train_bwd, dim3(grid), dim3(NT), 0, nullptr, A);
        (void)hipEventRecord(ev[2], nullptr);
        reduce();
        (void)hipEventRecord(ev[3], nullptr);
        (void)hipEventSynchronize(ev[3]);
        for (int k = 0; k < 3; ++k) {
            float ms;
            (void)hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
            tk[k] += ms * 1e3f / N;
        }
    }
    // the phase ticks of the N timed updates only
    unsigned long long ph[16];
    (void)hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_tphase), sizeof(ph));
    printf("%s", with_adam ? "(Adam folded in) " : "");
    printf("B=%d grid=%d%s  fwd %.2f us  bwd %.2f us  reduce %.2f us\n", B, grid,
           A.pre ? "" : " (nopre)", tk[0], tk[1], tk[2]);
    {  // the reduce alone, back to back (nothing dirty from the train kernels)
        float ms;
        (void)hipEventRecord(ev[0], nullptr);
        for (int it = 0; it < N; ++it) reduce();
        (void)hipEventRecord(ev[1], nullptr);
        (void)hipEventSynchronize(ev[1]);
        (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
        printf("reduce alone, back to back: %.2f us\n", ms * 1e3f / N);
    }
    {  // the launch after each train kernel: what does the boundary cost the next kernel?
        auto timed = [&](auto&& before, auto&& after) {
            float tot = 0.f, ms;
            for (int it = 0; it < N; ++it) {
                before();
                (void)hipEventRecord(ev[2], nullptr);
                after();
                (void)hipEventRecord(ev[3], nullptr);
                (void)hipEventSynchronize(ev[3]);
                (void)hipEventElapsedTime(&ms, ev[2], ev[3]);
                tot += ms * 1e3f / N;
            }
            return tot;
        };
        auto fwd = [&]() { hipLaunchKernelGGL(k_conv_train_fwd, dim3(grid), dim3(NT), 0, nullptr, A); };
        auto bwd = [&]() { hipLaunchKernelGGL(k_conv_train_bwd, dim3(grid), dim3(NT), 0, nullptr, A); };
        auto nop = [&]() { hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, nullptr, nullptr); };
        auto fb = [&]() { fwd(); bwd(); };
        printf("nop after nop %.2f, after fwd %.2f, after fwd+bwd %.2f us\n", timed(nop, nop),
               timed(fwd, nop), timed(fb, nop));
        printf("reduce after nop %.2f, after fwd %.2f, after fwd+bwd %.2f us\n", timed(nop, reduce),
               timed(fwd, reduce), timed(fb, reduce));
    }
    const char* names[8] = {"stage", "conv1+V", "conv2", "fc1", "loss+df", "dWf1+dY", "dM+dU+st", "slab"};
    const double tiles = (double)N * ((B / 16 + grid - 1) / grid);
    for (int k = 0; k < 8; ++k)
        printf("%-10s %9.0f ticks/%s\n", names[k], ph[k] / (k == 0 || k == 7 ? N : tiles),
               k == 0 || k == 7 ? "launch" : "tile");
    const char* n2[4] = {"bwd stage", "bwd dM ld", "bwd dV", "bwd epi"};
    for (int k = 8; k < 12; ++k)
        printf("%-10s %9.0f ticks/%s\n", n2[k - 8], ph[k] / (k == 8 ? N : tiles), k == 8 ? "launch" : "tile");
    return 0;
}
