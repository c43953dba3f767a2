// Phase timing of k_conv_train (s_memtime deltas of block 0 per wave; each delta is charged to
// the phase that ENDS at the marker), built only for kernel tuning:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/prof_train.hip -o tools/prof_train
#define G2048_PHASE_PROF 1
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
#include "../reinforcement-learning-2048_amd/csrc/g2048_qtrain.hip"

int main() {
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
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int it = 0; it < 3; ++it)
        g2048_convnet_train_grad(&p, rows, acts, idx, y, B, ws, grad, loss, nullptr, nullptr);
    (void)hipEventRecord(a, nullptr);
    for (int it = 0; it < 20; ++it)
        g2048_convnet_train_grad(&p, rows, acts, idx, y, B, ws, grad, loss, nullptr, nullptr);
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long ph[4][16];
    (void)hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_tphase), sizeof(ph));
    printf("B=%d  train+reduce %.2f us/launch\n", B, ms * 1e3 / 20);
    const char* names[13] = {"start", "A stage", "B conv2 fwd", "C Wf1t", "D fc1 fwd", "E loss",
                             "F dWf2+Wf1r", "G df", "H dWf1+dh2", "I dh2+W2r", "J dW2",
                             "K dP+dW1", "slab"};
    for (int k = 0; k < 13; ++k) {
        printf("%-12s", names[k]);
        for (int wv = 0; wv < 4; ++wv) printf(" %8llu", ph[wv][k]);
        printf("\n");
    }
    return 0;
}
