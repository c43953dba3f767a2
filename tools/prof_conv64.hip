// Per-kernel event timing of the float64 conv update (g2048_conv64.hip) at B = 8192 and the phase
// ticks of its targets / train kernels (s_memtime deltas of wave 0 of workgroup 0, charged to
// the phase that ENDS at the marker), built only for kernel tuning:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prof_conv64.hip -o tools/prof_conv64
// (-DG2048_NO_PHASE_PROF: no markers, the library's code generation -- the event times to trust;
// the markers make train B spill).  Arguments: [B [nopre]].
#ifndef G2048_NO_PHASE_PROF
#define G2048_PHASE_PROF 1
#endif
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
#include "../reinforcement-learning-2048_amd/csrc/g2048_conv64.hip"
// libg2048.so symbols the file's ABI functions link against (unused here)
extern "C" int g2048_replay_views(g2048_replay*, uint8_t**, uint8_t**, uint8_t**, int32_t**,
                                  uint8_t**, uint64_t**) { return 1; }
extern "C" int g2048_env_views(g2048_env*, uint8_t**, uint32_t**, uint32_t**, uint64_t**) { return 1; }
extern "C" int64_t g2048_env_size(const g2048_env*) { return 0; }
extern "C" int g2048_env_rng(const g2048_env*, uint64_t*, uint64_t*) { return 1; }

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 8192;
    const int C = 1 << 20;
    const int sizes[8] = {256, 64, 16384, 64, 16384, 64, 256, 4};
    double* w[2][8];
    for (int n = 0; n < 2; ++n)
        for (int i = 0; i < 8; ++i) {
            std::vector<double> h(sizes[i]);
            for (int j = 0; j < sizes[i]; ++j) h[j] = 0.02 * ((j * 37 + i * 11 + n * 5) % 17 - 8);
            (void)hipMalloc(&w[n][i], sizes[i] * 8);
            (void)hipMemcpy(w[n][i], h.data(), sizes[i] * 8, hipMemcpyHostToDevice);
        }
    uint8_t *s, *s2, *a, *d;
    int32_t* r;
    unsigned long long *count, *step;
    (void)hipMalloc(&s, (size_t)C * 16);
    (void)hipMalloc(&s2, (size_t)C * 16);
    (void)hipMalloc(&a, C);
    (void)hipMalloc(&d, C);
    (void)hipMalloc(&r, (size_t)C * 4);
    (void)hipMalloc(&count, 8);
    (void)hipMalloc(&step, 8);
    std::vector<uint8_t> hb((size_t)C * 16);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = (uint8_t)((i * 2654435761u >> 13) % 12);
    (void)hipMemcpy(s, hb.data(), hb.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(s2, hb.data() + 16, hb.size() - 16, hipMemcpyHostToDevice);
    (void)hipMemset(a, 2, C);
    (void)hipMemset(d, 0, C);
    (void)hipMemset(r, 0, (size_t)C * 4);
    const unsigned long long hc = C, hs = 0;
    (void)hipMemcpy(count, &hc, 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(step, &hs, 8, hipMemcpyHostToDevice);
    int64_t* idx;
    double *y, *grad, *loss, *ws, *m, *v;
    (void)hipMalloc(&idx, B * 8);
    (void)hipMalloc(&y, B * 8);
    (void)hipMalloc(&grad, P_N * 8);
    (void)hipMalloc(&loss, 8);
    (void)hipMalloc(&m, P_N * 8);
    (void)hipMalloc(&v, P_N * 8);
    (void)hipMemset(m, 0, P_N * 8);
    (void)hipMemset(v, 0, P_N * 8);
    const int64_t nws = g2048_convnet_update_f64_workspace(B);
    (void)hipMalloc(&ws, nws * 8);
    const int grid = grid_of(B);
    const int64_t tiles = (B + TB - 1) / TB;
    double* pk = ws;
    unsigned long long* step_next = reinterpret_cast<unsigned long long*>(ws + WS_STEP);
    double* slab = ws + WS_SLAB;
    double* dz2 = slab + (int64_t)grid * SLAB;
    // argv[2] == "nopre": train A's slab terms summed by the reduce, not in train B's shadow
    const bool nopre = argc > 2 && strcmp(argv[2], "nopre") == 0;
    double* pre = grid >= SHADOW_MIN_GRID && !nopre ? dz2 + tiles * TB * 256 : nullptr;

    PackArgs P{w[0][2], w[0][4], w[1][2], w[1][4], pk};
    Ring R{reinterpret_cast<const uint4*>(s), reinterpret_cast<const uint4*>(s2), a, d, r, count};
    FusedArgs FA{};
    TgtArgs& T = FA.T;
    T.on = Net{w[0][0], w[0][1], w[0][2], w[0][3], w[0][4], w[0][5], w[0][6], w[0][7]};
    T.tg = Net{w[1][0], w[1][1], w[1][2], w[1][3], w[1][4], w[1][5], w[1][6], w[1][7]};
    T.pon = Packed{pk + O_U_ON, pk + O_F1_ON};
    T.ptg = Packed{pk + O_U_TG, pk + O_F1_TG};
    T.R = R;
    T.step = step;
    T.batch = B;
    T.seed_lo = 7;
    T.gamma = 0.8f;
    T.double_dqn = 1;
    T.idx_out = idx;
    T.y_out = y;
    T.step_next = step_next;
    TrainArgs& A = FA.A;
    A.on = T.on;
    A.pon = T.pon;
    A.pf1b = pk + O_F1B;
    A.p2b = pk + O_UB;
    A.R = R;
    A.idx = idx;
    A.y = y;
    A.batch = B;
    A.dz2 = dz2;
    A.slab = slab;
    A.pre = pre;
    RedArgs D{};
    D.slab = slab;
    D.pre = pre;
    D.nslab = grid;
    D.grad = grad;
    D.loss = loss;
    D.step_next = step_next;
    double* ps[8];
    for (int k = 0; k < 8; ++k) ps[k] = w[0][k];
    memcpy(D.p, ps, sizeof(ps));
    memcpy(D.tp, ps, sizeof(ps));
    D.m = m;
    D.v = v;
    D.lr = 1e-6;
    D.b1 = 0.9;
    D.b2 = 0.999;
    D.eps = 1e-8;
    D.adam = 1;
    D.pk = pk;  // the reduce re-packs (k_pack is timed separately: the update no longer runs it)

    auto launch = [&](int k) {
        switch (k) {
            case 0: hipLaunchKernelGGL(k_pack, dim3(PACK_ALL / NT), dim3(NT), 0, nullptr, P); break;
            case 1: break;  // (targets: fused into train A)
            case 2: hipLaunchKernelGGL(k_conv64_train_a, dim3(grid), dim3(NT), 0, nullptr, FA); break;
            case 3: hipLaunchKernelGGL(k_conv64_train_b, dim3(grid), dim3(NT), 0, nullptr, A); break;
            default:
                hipLaunchKernelGGL(k_conv64_reduce, dim3((P_N + 1 + 127) / 128), dim3(64 * RW), 0,
                                   nullptr, D);
        }
    };
    for (int it = 0; it < 3; ++it)
        for (int k = 0; k < 5; ++k) launch(k);
    (void)hipDeviceSynchronize();
#ifdef G2048_PHASE_PROF
    unsigned long long zero[32] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_cphase), zero, sizeof(zero));
#endif
    hipEvent_t ev[6];
    for (int i = 0; i < 6; ++i) (void)hipEventCreate(&ev[i]);
    float tk[5] = {0, 0, 0, 0, 0};
    const int N = 20;
    for (int it = 0; it < N; ++it) {
        (void)hipEventRecord(ev[0], nullptr);
        for (int k = 0; k < 5; ++k) {
            launch(k);
            (void)hipEventRecord(ev[k + 1], nullptr);
        }
        (void)hipEventSynchronize(ev[5]);
        for (int k = 0; k < 5; ++k) {
            float ms;
            (void)hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
            tk[k] += ms * 1e3f / N;
        }
    }
    // the phase ticks of the N timed updates only (the loops below launch train B again)
    unsigned long long ph[32] = {0};
#ifdef G2048_PHASE_PROF
    (void)hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_cphase), sizeof(ph));
#endif
    printf("B=%d grid=%d  pack %.2f  targets %.2f  train_a %.2f  train_b %.2f  reduce %.2f  "
           "(us)  update (no pack) %.2f\n", B, grid, tk[0], tk[1], tk[2], tk[3], tk[4],
           tk[1] + tk[2] + tk[3] + tk[4]);
    {  // the reduce alone, back to back (slabs resident, nothing dirty from the train kernels)
        float ms;
        (void)hipEventRecord(ev[0], nullptr);
        for (int it = 0; it < N; ++it) launch(4);
        (void)hipEventRecord(ev[1], nullptr);
        (void)hipEventSynchronize(ev[1]);
        (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
        printf("reduce alone, back to back: %.2f us\n", ms * 1e3f / N);
        (void)hipEventRecord(ev[0], nullptr);
        for (int it = 0; it < N; ++it) {
            launch(3);
            (void)hipEventRecord(ev[2], nullptr);
            launch(4);
            (void)hipEventRecord(ev[3], nullptr);
        }
        (void)hipEventSynchronize(ev[3]);
        (void)hipEventElapsedTime(&ms, ev[2], ev[3]);
        printf("reduce right after train_b (last pair): %.2f us\n", ms * 1e3f);
    }
    const double tpw = (double)N * ((tiles + grid - 1) / grid);  // tiles per workgroup x N
    const char* names[20] = {"-", "sample+put s'", "y + put s", "conv1+V", "conv2 wino", "fc1",
                             "fc2", "tgt y", "A load", "A loss/dq", "A fc2 grad+dZ3",
                             "A dWf1", "A dH2+store", "A slab", "B load", "B conv1",
                             "B db2+dW2", "B dD", "B dW1", "B slab"};
    for (int k = 1; k < 20; ++k) {
        const bool per_launch = k == 13 || k == 19;
        printf("%-16s %10.0f ticks/%s\n", names[k], ph[k] / (per_launch ? (double)N : tpw),
               per_launch ? "launch" : "tile (all nets)");
    }
    return 0;
}
