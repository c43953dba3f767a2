// g2048_common.hpp -- internal helpers shared by the translation units of libg2048.so.
#pragma once

#include <stdint.h>

// Record a printf-style message for g2048_last_error() and return `code` (hidden symbol).
int g2048_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// The env's Philox seed and global board offset (kernels outside g2048.hip that must repeat the
// step's draws: the greedy-only forward of g2048_qnet.hip).  Hidden symbol.
struct g2048_env;
extern "C" int g2048_env_rng(const g2048_env* e, uint64_t* seed, uint64_t* board_offset);

#ifdef __HIPCC__
#include <hip/hip_runtime.h>

namespace g2048 {

// torch.optim.Adam (single-tensor, amsgrad off, no weight decay) for one element; the scalar
// factors are evaluated in double and rounded to f32 like torch's Python-side scalars.  Shared by
// k_adam (g2048_adam.hip) and the dense-net reduce+Adam (g2048_mlp.hip) so both apply the same
// float sequence.
struct AdamCoef {
    float step_size, bc2_sqrt, w1, b2, w2, eps;
};

__device__ __forceinline__ AdamCoef adam_coef(double t, double lr, double b1, double b2,
                                              double eps) {
    AdamCoef c;
    c.step_size = (float)(lr / (1.0 - pow(b1, t)));
    c.bc2_sqrt = (float)sqrt(1.0 - pow(b2, t));
    c.w1 = (float)(1.0 - b1);
    c.b2 = (float)b2;
    c.w2 = (float)(1.0 - b2);
    c.eps = (float)eps;
    return c;
}

// One element on values: m, v updated; returns the updated parameter.  The fused multiply-adds
// are spelled out: left to contraction, the compiler fused them differently in different
// kernels (k_adam vs the reductions that fold Adam in), so the "bitwise the same update" of
// those kernels depended on their surrounding code.
__device__ __forceinline__ float adam_update(const AdamCoef& c, float g, float& m, float& v,
                                             float p) {
    m = __fmaf_rn(c.w1, g - m, m);                 // lerp(m, g, 1 - b1), weight < 0.5 branch
    v = __fmaf_rn(c.w2 * g, g, v * c.b2);          // mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(v) / c.bc2_sqrt + c.eps;
    return __fmaf_rn(-c.step_size, m / denom, p);  // addcdiv_(m, denom, value=-step_size)
}

// returns the updated parameter; m / v updated in place
__device__ __forceinline__ float adam_apply(const AdamCoef& c, float g, float* m_, float* v_,
                                            float p) {
    float m = *m_, v = *v_;
    const float np = adam_update(c, g, m, v, p);
    *m_ = m;
    *v_ = v;
    return np;
}

// torch.optim.Adam (single tensor, amsgrad off, no weight decay) on one float64 element, the
// scalars as torch forms them in double: m.lerp_(g, 1 - b1); v.mul_(b2).addcmul_(g, g, 1 - b2);
// denom = v.sqrt() / sqrt(1 - b2^t) + eps; p.addcdiv_(m, denom, -lr / (1 - b1^t)).  Shared by the
// float64 reductions (g2048_learn64.hip, g2048_conv64.hip) and g2048_adam_step_sync_f64.
// The step's two scalars (lr / (1 - b1^t), sqrt(1 - b2^t)): two f64 pow calls, so a kernel that
// updates many elements per lane forms them once, off its critical path.
struct Adam64Coef {
    double step_size, bc2_sqrt;
};

__device__ __forceinline__ Adam64Coef adam64_coef(double t, double lr, double b1, double b2) {
#pragma clang fp contract(off)
    return Adam64Coef{lr / (1.0 - pow(b1, t)), sqrt(1.0 - pow(b2, t))};
}

__device__ __forceinline__ double adam64_apply(const Adam64Coef& c, double b1, double b2,
                                               double eps, double g, double& m, double& v,
                                               double p) {
#pragma clang fp contract(off)
    m = m + (1.0 - b1) * (g - m);
    v = v * b2 + (1.0 - b2) * g * g;
    const double denom = sqrt(v) / c.bc2_sqrt + eps;
    return p + (-c.step_size) * (m / denom);
}

__device__ __forceinline__ double adam64(double t, double lr, double b1, double b2, double eps,
                                         double g, double& m, double& v, double p) {
    return adam64_apply(adam64_coef(t, lr, b1, b2), b1, b2, eps, g, m, v, p);
}

// A workgroup's 16-byte slab store: the slab is read only by later launches on other CUs.
// G2048_SLAB_AUX (build flag, default 0 = a plain global store) selects a buffer store with that
// cache-policy word instead (gfx950: 1 sc0, 2 nt, 16 sc1) -- a measurement switch.
#ifndef G2048_SLAB_AUX
#define G2048_SLAB_AUX 0
#endif
typedef uint32_t slab_u32x4 __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ void slab_store16(V* base, int64_t elem, V v) {
    static_assert(sizeof(V) == 16, "16-byte slab stores");
#if G2048_SLAB_AUX == 0
    base[elem] = v;
#else
    // base is the workgroup's slab (wave-uniform); a slab fits 2^31 bytes
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
    slab_u32x4 u;
    __builtin_memcpy(&u, &v, 16);
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, (uint32_t)(elem * 16), 0u, G2048_SLAB_AUX);
#endif
}

// Fixed-order sum of the previous launch's per-workgroup gradient slabs, run in the shadow of
// this launch's MFMA phases instead of in a reduction launch of its own.  Wave w of the block sums
// the slabs w, w + 4, w + 8, ... (ascending) at one vector element per lane; loads go out NB at a
// time into one of two register batches and are added one phase later, so a batch's memory round
// trip overlaps the phase between its issue and its consume:
//   issue(s1); phase 0; consume(s0) ... -- issue(b) / consume(b) alternate b = 0, 1 as the
// caller's phases go by.  The order of the additions is the slab order, whatever the batching,
// so the result is bitwise the same for any phase layout.
template <typename V, int NB>
struct SlabShadow {
    const V* p = nullptr;  // this lane's element in slab 0 (null: the lane sums nothing)
    int64_t stride = 0;    // V elements from one slab to the next
    int next = 0;          // the next slab this wave issues
    int nslab = 0;
    V acc{};
    V buf[2][NB];

    __device__ __forceinline__ void init(const V* lane_p, int64_t stride_v, int nslab_, int wave) {
        p = lane_p;
        stride = stride_v;
        nslab = nslab_;
        next = wave;
    }
    __device__ __forceinline__ bool pending() const { return p != nullptr && next < nslab; }
    template <int B>
    __device__ __forceinline__ void issue() {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int g = next + 4 * u;
            buf[B][u] = (p != nullptr && g < nslab) ? p[(int64_t)g * stride] : V{};
        }
        next += 4 * NB;
    }
    template <int B>
    __device__ __forceinline__ void consume() {
#pragma unroll
        for (int u = 0; u < NB; ++u) acc += buf[B][u];
    }
};

}  // namespace g2048
#endif
