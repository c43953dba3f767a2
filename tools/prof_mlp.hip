// Phase ticks of k_mlp_update (thread 0 of every workgroup stamps s_memtime at 7 points; the
// averages over workgroups of the deltas are printed), built only for kernel tuning:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prof_mlp.hip -o tools/prof_mlp
#define G2048_MLP_PHASE 1
#include <cstdarg>
#include <cstdio>
#include <vector>
int g2048_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    return code;
}
// ring views for the update ABI: a synthetic ring (set up in main)
static uint8_t *g_s, *g_s2, *g_a, *g_d;
static int32_t* g_r;
static uint64_t* g_count;
extern "C" int g2048_replay_views(struct g2048_replay*, uint8_t** s, uint8_t** s2, uint8_t** a,
                                  int32_t** r, uint8_t** d, uint64_t** count) {
    if (s) *s = g_s;
    if (s2) *s2 = g_s2;
    if (a) *a = g_a;
    if (r) *r = g_r;
    if (d) *d = g_d;
    if (count) *count = g_count;
    return 0;
}
#include "../reinforcement-learning-2048_amd/csrc/g2048_mlp.hip"

int main() {
    const int B = 8192;
    const long C = 1 << 20;
    (void)hipMalloc(&g_s, C * 16);
    (void)hipMalloc(&g_s2, C * 16);
    (void)hipMalloc(&g_a, C);
    (void)hipMalloc(&g_d, C);
    (void)hipMalloc(&g_r, C * 4);
    (void)hipMalloc(&g_count, 8);
    std::vector<uint8_t> hb(C * 16);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = (uint8_t)((i * 2654435761u >> 13) % 12);
    (void)hipMemcpy(g_s, hb.data(), hb.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(g_s2, hb.data(), hb.size(), hipMemcpyHostToDevice);
    (void)hipMemset(g_a, 1, C);
    (void)hipMemset(g_d, 0, C);
    (void)hipMemset(g_r, 0, C * 4);
    const unsigned long long hc = C;
    (void)hipMemcpy(g_count, &hc, 8, hipMemcpyHostToDevice);
    const int sizes[4] = {1024, 64, 256, 4};
    float* w[4];
    for (int i = 0; i < 4; ++i) {
        std::vector<float> h(sizes[i]);
        for (int j = 0; j < sizes[i]; ++j) h[j] = 0.05f * ((j * 37 + i) % 17 - 8);
        (void)hipMalloc(&w[i], sizes[i] * 4);
        (void)hipMemcpy(w[i], h.data(), sizes[i] * 4, hipMemcpyHostToDevice);
    }
    g2048_dense64_params p{w[0], w[1], w[2], w[3]};
    int64_t* idx;
    float *y, *grad, *loss, *ws;
    uint64_t* step;
    (void)hipMalloc(&idx, B * 8);
    (void)hipMalloc(&y, B * 4);
    (void)hipMalloc(&grad, 1348 * 4);
    (void)hipMalloc(&loss, 4);
    (void)hipMalloc(&step, 8);
    (void)hipMemset(step, 0, 8);
    const int64_t nws = g2048_dense64_update_workspace(B);
    (void)hipMalloc(&ws, nws * 4);
    const int grid = (int)((B + S_UPD - 1) / S_UPD < MAX_SLABS ? (B + S_UPD - 1) / S_UPD : MAX_SLABS);
    long long* ph = reinterpret_cast<long long*>(ws + (int64_t)grid * SLAB + 2);
    std::vector<double> acc(7, 0.0);
    const int N = 20;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float tot = 0.f;
    for (int it = 0; it < N + 2; ++it) {
        (void)hipEventRecord(a, nullptr);
        g2048_dense64_update(&p, &p, reinterpret_cast<g2048_replay*>(g_count) /* (stub views) */,
                             nullptr, B, 7, step, 0.8f, 1, idx, y, ws, grad, loss,
                             nullptr, nullptr, 0, 0, 0, 0, 0, nullptr);
        (void)hipEventRecord(b, nullptr);
        (void)hipEventSynchronize(b);
        if (it < 2) continue;  // warm-up
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        tot += ms;
        std::vector<long long> h(grid * 8);
        (void)hipMemcpy(h.data(), ph, h.size() * 8, hipMemcpyDeviceToHost);
        for (int g = 0; g < grid; ++g)
            for (int k = 0; k < 6; ++k) acc[k] += (double)(h[g * 8 + k + 1] - h[g * 8 + k]) / grid;
    }
    printf("dense64 update B=%d grid=%d: %.2f us (update + reduce, events)\n", B, grid,
           tot * 1e3f / N);
    const char* names[6] = {"sample+loads", "stage s'", "2 fwd + y", "stage s", "fwd+bwd", "slab"};
    for (int k = 0; k < 6; ++k) printf("  %-13s %8.0f ticks\n", names[k], acc[k] / N);
    return 0;
}
