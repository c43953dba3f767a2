// The rollout's ring stores alone (rollexp's k_store_only: s 16 + s' 16 + a 1 + r 4 + d 1 bytes
// per board and step, sc1 buffer stores) with a board spread over 1, 2 or 4 lanes -- at 64k boards
// that is one, two or four waves per SIMD for the same bytes.  Prices the store side of a rollout
// that splits each board over several lanes: does a second wave per SIMD lower the
// store floor the one-wave-per-SIMD rollout sits on?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_lanes.hip -o tools/store_lanes
//   tools/store_lanes [n=65536] [K=64]
#include "../reinforcement-learning-2048_amd/csrc/g2048.hip"

#include <cstdio>
#include <cstdlib>

namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// kL lanes per board: lane h of board b stores bytes [h*16/kL, (h+1)*16/kL) of s and s', and
// the a / r / d bytes go to lanes 0 / (1 % kL) / (2 % kL).
template <int kL>
__global__ __launch_bounds__(kBlock) void k_store_lanes(StepArgs A) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t b = i / kL;
    const uint32_t h = (uint32_t)(i % kL);
    if (b >= A.n) return;
    const uint32_t n32 = (uint32_t)A.n, cap32 = (uint32_t)A.rb.capacity, bl = (uint32_t)b;
    const uint64_t t0 = load_clock(A.clock, b);
    uint32_t soff = (uint32_t)ring_row(t0, A.rb.rows) * n32;
    __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(A.rb.win, 0, (int)A.rb.win_bytes, 0x00020000);
    constexpr uint32_t W = 16 / kL;  // bytes of s (and of s') per lane
    const uint32_t v_s = A.rb.o_s + 16u * bl + W * h, v_s2 = A.rb.o_s2 + 16u * bl + W * h;
    const uint32_t v_a = A.rb.o_a + bl, v_r = A.rb.o_r + 4u * bl, v_d = A.rb.o_d + bl;
    uint32_t x = (uint32_t)i * 2654435761u;
    for (int s = 0; s < A.k_steps; ++s) {
        x = x * 1664525u + 1013904223u;
        if constexpr (kL == 1) {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{x, x + 1u, x + 2u, x + 3u}, rw, v_s, soff * 16u, 16);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{x ^ 1u, x ^ 2u, x ^ 3u, x}, rw, v_s2, soff * 16u, 16);
        } else if constexpr (kL == 2) {
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{x, x + 1u}, rw, v_s, soff * 16u, 16);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{x ^ 1u, x ^ 2u}, rw, v_s2, soff * 16u, 16);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(x, rw, v_s, soff * 16u, 16);
            __builtin_amdgcn_raw_buffer_store_b32(x ^ 1u, rw, v_s2, soff * 16u, 16);
        }
        if (h == 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)x, rw, v_a, soff, 16);
        if (h == 1u % kL) __builtin_amdgcn_raw_buffer_store_b32(x, rw, v_r, soff * 4u, 16);
        if (h == 2u % kL) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(x >> 8), rw, v_d, soff, 16);
        soff = soff + n32 == cap32 ? 0u : soff + n32;
    }
}

template <int kL>
void launch(g2048_env* e, g2048_replay* rb, int K, hipStream_t st) {
    StepArgs A;
    make_args(e, rb, A);
    A.k_steps = K;
    const int64_t threads = e->n * kL;
    hipLaunchKernelGGL((k_store_lanes<kL>), dim3((unsigned)((threads + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, st, A);
}

}  // namespace

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const int K = argc > 2 ? atoi(argv[2]) : 64;
    hipStream_t st;
    (void)hipStreamCreate(&st);
    g2048_env* e;
    g2048_replay* rb;
    if (g2048_env_create(&e, n, 7, 0, 0, 0, nullptr) || g2048_replay_create(&rb, n * K, 0, nullptr)) {
        printf("create failed: %s\n", g2048_last_error());
        return 1;
    }
    void (*fns[3])(g2048_env*, g2048_replay*, int, hipStream_t) = {launch<1>, launch<2>, launch<4>};
    const int lanes[3] = {1, 2, 4};
    hipEvent_t ev0, ev1;
    (void)hipEventCreate(&ev0);
    (void)hipEventCreate(&ev1);
    for (int rep = 0; rep < 3; ++rep) {
        for (int v = 0; v < 3; ++v) {
            hipGraph_t g;
            hipGraphExec_t ge;
            (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
            for (int it = 0; it < 20; ++it) fns[v](e, rb, K, st);
            (void)hipStreamEndCapture(st, &g);
            (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev0, st);
            for (int it = 0; it < 10; ++it) (void)hipGraphLaunch(ge, st);
            (void)hipEventRecord(ev1, st);
            if (hipEventSynchronize(ev1) != hipSuccess) {
                printf("kernel failed\n");
                return 1;
            }
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, ev0, ev1);
            const double us = 1e3 * ms / 200.0;
            printf("stores only, %d lane(s) per board  n=%lld K=%d  %8.2f us/launch  %6.3f of 8 TB/s\n",
                   lanes[v], (long long)n, K, us, 38.0 * n * K / us * 1e-6 / 8.0);
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        }
    }
    return 0;
}
