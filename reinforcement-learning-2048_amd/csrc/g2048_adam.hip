// g2048_adam.hip -- one-launch Adam over a flat gradient bucket (the learner's optimizer step).
//
// Replaces torch.optim.Adam(model.parameters(), lr) .step() in the intended zero_grad ->
// backward -> step order (src/configs/double_dqn_conv.py:39; the reference's own call order is a
// no-op).  Same update as torch's single-tensor Adam (amsgrad off, no weight decay):
//   m <- lerp(m, g, 1 - b1);  v <- v*b2 + (1 - b2)*g*g
//   p <- p - (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with the bias corrections evaluated in double and rounded to f32 like torch's Python scalars,
// and t read from the device update counter (bumped by the train-gradient launch), so the step
// is graph-replay safe.  Parameters may be separate tensors; m and v are flat buffers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/g2048.h"
#include "g2048_common.hpp"

namespace {

constexpr int kMaxTensors = 16;

struct AdamArgs {
    float* p[kMaxTensors];
    float* tp[kMaxTensors];  // target-net copies (nullable): written when t % sync_every == 0
    unsigned long long sync_every;
    int64_t off[kMaxTensors + 1];
    int nt;
    const float* g;
    float* m;
    float* v;
    const unsigned long long* step;
    double lr, b1, b2, eps;
    float gscale;  // the gradient's scale: 1, or 1 / world after a SUM all-reduce
};

__global__ __launch_bounds__(256) void k_adam(AdamArgs A) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.off[A.nt]) return;
    int k = 0;
#pragma unroll
    for (int j = 1; j < kMaxTensors; ++j) k += (j < A.nt && i >= A.off[j]) ? 1 : 0;
    float* p = A.p[k] + (i - A.off[k]);
    const unsigned long long t = *A.step;
    const g2048::AdamCoef c = g2048::adam_coef((double)t, A.lr, A.b1, A.b2, A.eps);
    // the scaled gradient is rounded on its own (contraction off: HIP's __fmul_rn is a plain
    // multiply, which the compiler fused into Adam's g - m), so a scaled step is bitwise the
    // unscaled step on the pre-scaled gradient for ANY scale
    float gs;
    {
#pragma clang fp contract(off)
        gs = A.g[i] * A.gscale;
    }
    const float np = g2048::adam_apply(c, gs, A.m + i, A.v + i, *p);
    *p = np;
    // target sync (src/dqn_lib.py:227-228 load_state_dict after the update) on the device
    // counter, so an update that syncs needs no host decision between graph replays
    if (A.sync_every && t % A.sync_every == 0ull) A.tp[k][i - A.off[k]] = np;
}

// The float64 form (the reference's precision): g2048::adam64, the update the float64 fused
// reductions apply, so a data-parallel float64 learner (gradient -> all-reduce -> this step)
// moves the weights exactly as the single-process one on the same gradient.
struct AdamArgs64 {
    double* p[kMaxTensors];
    double* tp[kMaxTensors];
    unsigned long long sync_every;
    int64_t off[kMaxTensors + 1];
    int nt;
    const double* g;
    double* m;
    double* v;
    const unsigned long long* step;
    double lr, b1, b2, eps;
    double gscale;
};

__global__ __launch_bounds__(256) void k_adam64(AdamArgs64 A) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.off[A.nt]) return;
    int k = 0;
#pragma unroll
    for (int j = 1; j < kMaxTensors; ++j) k += (j < A.nt && i >= A.off[j]) ? 1 : 0;
    double* p = A.p[k] + (i - A.off[k]);
    const unsigned long long t = *A.step;
    double m = A.m[i], v = A.v[i];
    double gs;
    {
#pragma clang fp contract(off)
        gs = A.g[i] * A.gscale;
    }
    const double np = g2048::adam64((double)t, A.lr, A.b1, A.b2, A.eps, gs, m, v, *p);
    A.m[i] = m;
    A.v[i] = v;
    *p = np;
    if (A.sync_every && t % A.sync_every == 0ull) A.tp[k][i - A.off[k]] = np;
}

}  // namespace

static int adam_launch(float* const* params, const int64_t* numels, int n_tensors,
                       const float* grad, float* exp_avg, float* exp_avg_sq,
                       const uint64_t* step_dev, double lr, double beta1, double beta2,
                       double eps, float* const* target_params, uint64_t sync_every,
                       double grad_scale, void* stream) {
    if (!params || !numels || n_tensors <= 0 || n_tensors > kMaxTensors || !grad || !exp_avg ||
        !exp_avg_sq || !step_dev)
        return g2048_fail(G2048_EINVAL, "adam_step: bad arguments (n_tensors <= %d)", kMaxTensors);
    if (!(grad_scale > 0.0)) return g2048_fail(G2048_EINVAL, "adam_step: grad_scale must be > 0");
    if (sync_every && !target_params)
        return g2048_fail(G2048_EINVAL, "adam_step: sync_every > 0 needs target_params");
    AdamArgs A;
    A.nt = n_tensors;
    A.off[0] = 0;
    for (int j = 0; j < kMaxTensors; ++j) {
        A.p[j] = j < n_tensors ? params[j] : nullptr;
        A.tp[j] = (sync_every && j < n_tensors) ? target_params[j] : nullptr;
        if (j < n_tensors) A.off[j + 1] = A.off[j] + numels[j];
    }
    for (int j = n_tensors + 1; j <= kMaxTensors; ++j) A.off[j] = A.off[n_tensors];
    A.sync_every = sync_every;
    A.g = grad;
    A.m = exp_avg;
    A.v = exp_avg_sq;
    A.step = reinterpret_cast<const unsigned long long*>(step_dev);
    A.lr = lr;
    A.b1 = beta1;
    A.b2 = beta2;
    A.eps = eps;
    A.gscale = (float)grad_scale;
    const int64_t n = A.off[n_tensors];
    hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK : g2048_fail(G2048_EHIP, "adam_step: %s", hipGetErrorString(e));
}

extern "C" G2048_API int g2048_adam_step(float* const* params, const int64_t* numels,
                                         int n_tensors, const float* grad, float* exp_avg,
                                         float* exp_avg_sq, const uint64_t* step_dev, double lr,
                                         double beta1, double beta2, double eps, void* stream) {
    return adam_launch(params, numels, n_tensors, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1,
                       beta2, eps, nullptr, 0, 1.0, stream);
}

extern "C" G2048_API int g2048_adam_step_sync(float* const* params, const int64_t* numels,
                                              int n_tensors, const float* grad, float* exp_avg,
                                              float* exp_avg_sq, const uint64_t* step_dev,
                                              double lr, double beta1, double beta2, double eps,
                                              float* const* target_params, uint64_t sync_every,
                                              void* stream) {
    return adam_launch(params, numels, n_tensors, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1,
                       beta2, eps, target_params, sync_every, 1.0, stream);
}

// Data-parallel form: the gradient bucket holds the SUM over ranks (the all-reduce captured in the
// same graph, no divide launch) and Adam reads g * grad_scale (grad_scale = 1 / world; exact for
// power-of-two worlds, so the update equals the divide-then-Adam form bit for bit there).
extern "C" G2048_API int g2048_adam_step_scaled(float* const* params, const int64_t* numels,
                                                int n_tensors, const float* grad, float* exp_avg,
                                                float* exp_avg_sq, const uint64_t* step_dev,
                                                double lr, double beta1, double beta2, double eps,
                                                float* const* target_params, uint64_t sync_every,
                                                double grad_scale, void* stream) {
    return adam_launch(params, numels, n_tensors, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1,
                       beta2, eps, target_params, sync_every, grad_scale, stream);
}

static int adam64_launch(double* const* params, const int64_t* numels, int n_tensors,
                         const double* grad, double* exp_avg, double* exp_avg_sq,
                         const uint64_t* step_dev, double lr, double beta1, double beta2,
                         double eps, double* const* target_params, uint64_t sync_every,
                         double grad_scale, void* stream) {
    if (!(grad_scale > 0.0)) return g2048_fail(G2048_EINVAL, "adam_step_f64: grad_scale must be > 0");
    if (!params || !numels || n_tensors <= 0 || n_tensors > kMaxTensors || !grad || !exp_avg ||
        !exp_avg_sq || !step_dev)
        return g2048_fail(G2048_EINVAL, "adam_step_f64: bad arguments (n_tensors <= %d)",
                          kMaxTensors);
    if (sync_every && !target_params)
        return g2048_fail(G2048_EINVAL, "adam_step_f64: sync_every > 0 needs target_params");
    AdamArgs64 A;
    A.nt = n_tensors;
    A.off[0] = 0;
    for (int j = 0; j < kMaxTensors; ++j) {
        A.p[j] = j < n_tensors ? params[j] : nullptr;
        A.tp[j] = (sync_every && j < n_tensors) ? target_params[j] : nullptr;
        if (j < n_tensors) A.off[j + 1] = A.off[j] + numels[j];
    }
    for (int j = n_tensors + 1; j <= kMaxTensors; ++j) A.off[j] = A.off[n_tensors];
    A.sync_every = sync_every;
    A.g = grad;
    A.m = exp_avg;
    A.v = exp_avg_sq;
    A.step = reinterpret_cast<const unsigned long long*>(step_dev);
    A.lr = lr;
    A.b1 = beta1;
    A.b2 = beta2;
    A.eps = eps;
    A.gscale = grad_scale;
    const int64_t n = A.off[n_tensors];
    hipLaunchKernelGGL(k_adam64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), A);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? G2048_OK
                           : g2048_fail(G2048_EHIP, "adam_step_f64: %s", hipGetErrorString(e));
}

extern "C" G2048_API int g2048_adam_step_sync_f64(double* const* params, const int64_t* numels,
                                                  int n_tensors, const double* grad,
                                                  double* exp_avg, double* exp_avg_sq,
                                                  const uint64_t* step_dev, double lr,
                                                  double beta1, double beta2, double eps,
                                                  double* const* target_params,
                                                  uint64_t sync_every, void* stream) {
    return adam64_launch(params, numels, n_tensors, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1,
                         beta2, eps, target_params, sync_every, 1.0, stream);
}

extern "C" G2048_API int g2048_adam_step_scaled_f64(double* const* params, const int64_t* numels,
                                                    int n_tensors, const double* grad,
                                                    double* exp_avg, double* exp_avg_sq,
                                                    const uint64_t* step_dev, double lr,
                                                    double beta1, double beta2, double eps,
                                                    double* const* target_params,
                                                    uint64_t sync_every, double grad_scale,
                                                    void* stream) {
    return adam64_launch(params, numels, n_tensors, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1,
                         beta2, eps, target_params, sync_every, grad_scale, stream);
}
