/* abi_demo.c -- a plain-C caller of the g2048 C ABI (include/g2048.h), the way a non-Python host
 * (cgo, JNI, N-API) would bind it: opaque handles, device pointers, status codes.
 * Build:  gcc -std=c11 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ examples/abi_demo.c \
 *             -Lreinforcement-learning-2048_amd/g2048 -l:libg2048.so -L/opt/rocm/lib -lamdhip64 \
 *             -Wl,-rpath,<those dirs> -o abi_demo
 * Usage:  abi_demo [n_boards [steps [rollout_k [out.bin]]]]   (default 65536 1000 0)
 * Runs `steps` random-policy g2048_env_step calls and one g2048_env_rollout of rollout_k steps
 * on device 0 with a replay ring of 16 rows per board, samples one B = 8192 f32 minibatch, and
 * (with out.bin) writes the final boards u8[n][16] then {score, moves} u32[n][2]
 * (g2048_env_score_moves) to out.bin, so a test can compare them with the CPU oracle
 * (tests/test_abi_gpu.py).  Needs an MI355X at run time. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_runtime_api.h>

#include "g2048.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_ != G2048_OK) {                                                \
            fprintf(stderr, "%s -> %d: %s\n", #x, rc_, g2048_last_error());   \
            return 1;                                                         \
        }                                                                     \
    } while (0)

#define HCHECK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s -> %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const int steps = argc > 2 ? atoi(argv[2]) : 1000;
    const int k = argc > 3 ? atoi(argv[3]) : 0;
    const char* out = argc > 4 ? argv[4] : NULL;
    const int64_t cap = 16 * n, batch = 8192;
    g2048_env* env = NULL;
    g2048_replay* rb = NULL;
    CHECK(g2048_env_create(&env, n, 0x2048, 0, 0, 0, NULL));
    CHECK(g2048_replay_create(&rb, cap, 0, NULL));
    for (int t = 0; t < steps; ++t) CHECK(g2048_env_step(env, NULL, NULL, NULL, NULL, rb, NULL));
    CHECK(g2048_env_rollout(env, k, rb, NULL, NULL));
    float *s = NULL, *s2 = NULL, *r = NULL, *d = NULL;
    int64_t* a = NULL;
    HCHECK(hipMalloc((void**)&s, batch * 16 * sizeof(float)));
    HCHECK(hipMalloc((void**)&s2, batch * 16 * sizeof(float)));
    HCHECK(hipMalloc((void**)&r, batch * sizeof(float)));
    HCHECK(hipMalloc((void**)&d, batch * sizeof(float)));
    HCHECK(hipMalloc((void**)&a, batch * sizeof(int64_t)));
    CHECK(g2048_replay_sample_encode(rb, NULL, batch, 7, 0, G2048_F32, s, s2, a, r, d, NULL, NULL));
    int64_t bad = 0;
    CHECK(g2048_env_error_count(env, &bad, NULL));  /* synchronises the stream */
    uint8_t* board = NULL;
    CHECK(g2048_env_views(env, &board, NULL, NULL, NULL));
    if (out) {
        uint8_t* hb = (uint8_t*)malloc((size_t)n * 16);
        uint32_t* hm = (uint32_t*)malloc((size_t)n * 8);
        uint32_t* sm = NULL;  /* {score, moves} per board, derived from meta and the clock */
        if (!hb || !hm) return 1;
        HCHECK(hipMalloc((void**)&sm, (size_t)n * 8));
        CHECK(g2048_env_score_moves(env, sm, NULL));
        HCHECK(hipMemcpy(hb, board, (size_t)n * 16, hipMemcpyDeviceToHost));
        HCHECK(hipMemcpy(hm, sm, (size_t)n * 8, hipMemcpyDeviceToHost));
        hipFree(sm);
        FILE* f = fopen(out, "wb");
        if (!f || fwrite(hb, 1, (size_t)n * 16, f) != (size_t)n * 16 ||
            fwrite(hm, 1, (size_t)n * 8, f) != (size_t)n * 8 || fclose(f) != 0)
            return 1;
        free(hb);
        free(hm);
    }
    printf("stepped %lld boards x %d + rollout %d, %lld input errors, sampled %lld rows\n",
           (long long)n, steps, k, (long long)bad, (long long)batch);
    hipFree(s);
    hipFree(s2);
    hipFree(r);
    hipFree(d);
    hipFree(a);
    g2048_replay_destroy(rb);
    g2048_env_destroy(env);
    return 0;
}
