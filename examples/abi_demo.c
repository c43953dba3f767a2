/* abi_demo.c -- a plain-C caller of the g2048 C ABI (include/g2048.h).
 * Build:  gcc -std=c11 -Iinclude examples/abi_demo.c \
 *             -Lreinforcement-learning-2048_amd/g2048 -lg2048 -Wl,-rpath,<that dir> -o abi_demo
 * Runs 1000 random-policy steps of 65 536 boards with a 1M-transition replay ring, then samples
 * one B = 8192 minibatch, all on device 0.  Needs an MI355X at run time. */
#include <stdint.h>
#include <stdio.h>

#include "g2048.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_ != G2048_OK) {                                                \
            fprintf(stderr, "%s -> %d: %s\n", #x, rc_, g2048_last_error());   \
            return 1;                                                         \
        }                                                                     \
    } while (0)

int main(void) {
    g2048_env* env = NULL;
    g2048_replay* rb = NULL;
    const int64_t n = 65536, cap = 16 * 65536;
    CHECK(g2048_env_create(&env, n, 0x2048, 0, 0, 0, NULL));
    CHECK(g2048_replay_create(&rb, cap, 0, NULL));
    for (int t = 0; t < 1000; ++t) CHECK(g2048_env_step(env, NULL, NULL, NULL, NULL, rb, NULL));
    int64_t bad = 0;
    CHECK(g2048_env_error_count(env, &bad, NULL));
    uint8_t* s = NULL;
    CHECK(g2048_replay_views(rb, &s, NULL, NULL, NULL, NULL, NULL));
    printf("stepped %lld boards x 1000, %lld input errors, ring at %p\n", (long long)n,
           (long long)bad, (void*)s);
    g2048_replay_destroy(rb);
    g2048_env_destroy(env);
    return 0;
}
